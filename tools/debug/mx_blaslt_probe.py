"""Which e8m0 scale layout does hipBLASLt's VEC32_UE8M0 mode read, and how fast is it at the Llama-3-8B shapes?

Quantises A [M, K] and B [N, K] with this framework's MX quantiser, hands hipBLASLt the block scales in candidate
layouts and compares each result with the dequantised fp32 product; then times the layout that matches against the
hand-written MX kernel (ext().mx_gemm). One JSON line per probe."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from accelerate_hpc_test_amd.ops import fp8  # noqa: E402
from accelerate_hpc_test_amd.ops._ext import ext  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def layouts(s_nat, R, KB):
    return {"row[R,KB]": s_nat.contiguous(), "col[KB,R]": s_nat.t().contiguous()}


torch.manual_seed(0)
M, N, K = 512, 768, 1024
a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
qa, sa = fp8.mx_quant(a, colwise=False)[:2]
qb, sb = fp8.mx_quant(b, colwise=False)[:2]
ref = fp8.mx_dequant(qa, sa) @ fp8.mx_dequant(qb, sb).t()
na, nb = fp8.mx_scales_natural(sa), fp8.mx_scales_natural(sb)
good = None
for la_name, la in layouts(na, M, K // 32).items():
    for lb_name, lb in layouts(nb, N, K // 32).items():
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ok = ext().blaslt_mx_gemm(qa, qb, la, lb, out, False)
        err = rel(out, ref) if ok else None
        print(json.dumps({"sa": la_name, "sb": lb_name, "ran": ok, "rel_err": err}), flush=True)
        if ok and err is not None and err < 1e-2 and good is None:
            good = (la_name, lb_name)
print(json.dumps({"layout": good}), flush=True)


def tm(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


if good is not None:
    T = 8192
    for name, (n, k) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}.items():
        for tag, (mm, nn, kk) in {"fwd": (T, n, k), "dgrad": (T, k, n), "wgrad": (n, k, T)}.items():
            print(json.dumps({"start": f"{name}.{tag}", "mnk": [mm, nn, kk]}), flush=True)
            x = torch.randn(mm, kk, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(nn, kk, device="cuda", dtype=torch.bfloat16)
            qx, sx = fp8.mx_quant(x, colwise=False)[:2]
            qw, sw = fp8.mx_quant(w, colwise=False)[:2]
            lx = layouts(fp8.mx_scales_natural(sx), mm, kk // 32)[good[0]]
            lw = layouts(fp8.mx_scales_natural(sw), nn, kk // 32)[good[1]]
            out = torch.empty(mm, nn, device="cuda", dtype=torch.bfloat16)
            t_bl = tm(lambda: ext().blaslt_mx_gemm(qx, qw, lx, lw, out, False))
            t_hip = tm(lambda: fp8.mx_gemm(qx, qw, sx, sw))
            fl = 2.0 * mm * nn * kk
            print(json.dumps({"gemm": f"{name}.{tag}", "blaslt_ms": round(t_bl, 3), "blaslt_tflops": round(fl / t_bl / 1e9),
                              "hip_ms": round(t_hip, 3), "hip_tflops": round(fl / t_hip / 1e9)}), flush=True)
            del x, w, qx, qw, out
