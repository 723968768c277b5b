"""GEMM throughput at the Llama-3-8B linear shapes: our MX-fp8 MFMA kernels vs the libraries torch ships — bf16
hipBLASLt (torch.matmul) and fp8 hipBLASLt through `torch._scaled_mm` with per-tensor scales, which is the GEMM the
reference's torchao Float8Linear path calls (`/root/reference/src/accelerate/utils/ao.py:104-143`).

All kernel variants run in ONE process, in interleaved rounds (`ext().fp8_gemm_select`), on random data; one JSON
line per shape with the median ms / TFLOP/s of each variant over the rounds.

    python tools/bench_gemm.py [--tokens 8192] [--iters 20] [--rounds 3] [--variants 2,4] [--shapes qkv,o]

variants: bl = hipBLASLt fp8 via csrc/runtime/blaslt_gemm.cpp (the default per-tensor path), 1 = v1 128x128, 2 = v2 256x256 4 waves, 3 = v2 8 waves, 4 = v3 4-deep ring, 5 = v3 8 waves; "4g8" = v3 with tile rows
grouped by 8 (ext().fp8_gemm_select(variant, group_m)); "mx" = the MXFP8 GEMM (v3 ring with per-32 block scales in the
MFMA), whose row also reports the one-pass row+column MX quantisation of the A operand (mxq_ms).
"""

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tokens", type=int, default=8192)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--variants", default="2,4")
    p.add_argument("--shapes", default="qkv,o,gate_up,down")
    p.add_argument("--no-bf16", action="store_true")
    p.add_argument("--no-scaled-mm", action="store_true")
    p.add_argument("--check", action="store_true", help="compare every hand-written variant's output with hipBLASLt's")
    args = p.parse_args()
    from accelerate_hpc_test_amd.ops import fp8, gemm_tuning
    from accelerate_hpc_test_amd.ops._ext import ext

    gemm_tuning.load_tuned_gemms()
    T = args.tokens
    variants = args.variants.split(",")

    def select(v):
        if v in ("mx", "bl"):
            return
        num, _, g = v.partition("g")
        ext().fp8_gemm_select(int(num), int(g) if g else 0)
    all_shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    shapes = {k: all_shapes[k] for k in args.shapes.split(",")}
    one = torch.ones(1, device="cuda")
    for name, (N, K) in shapes.items():
        # forward (x·Wᵀ), dgrad (dy·W → [T,K] from [T,N]·[N,K]), wgrad (dyᵀ·x → [N,K])
        for kind, (m, n, k) in {"fwd": (T, N, K), "dgrad": (T, K, N), "wgrad": (N, K, T)}.items():
            a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
            flops = 2.0 * m * n * k
            a8, b8 = fp8.cast(a, one), fp8.cast(b, one)
            if "mx" in variants:
                aq, as_ = fp8.mx_quant(a, False, False)
                bq, bs = fp8.mx_quant(b, False, False)
            times = {v: [] for v in variants}
            mxq = []
            bf = []
            smm = []
            smm_ok = not args.no_scaled_mm
            for _ in range(args.rounds):
                if not args.no_bf16:
                    bf.append(timeit(lambda: a @ b.t(), args.iters))
                if smm_ok:
                    try:  # hipBLASLt fp8 (e4m3 x e4m3 -> bf16, per-tensor scales), B column-major as _scaled_mm wants
                        smm.append(timeit(lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one,
                                                                   out_dtype=torch.bfloat16), args.iters))
                    except Exception as exc:  # noqa: BLE001 - report, keep benchmarking the rest
                        smm_ok = False
                        print(json.dumps({"scaled_mm_error": repr(exc)[:300]}), flush=True)
                for v in variants:
                    select(v)
                    if v == "bl":  # hipBLASLt fp8 through our runner (what Fp8Linear uses by default)
                        dst = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
                        times[v].append(timeit(lambda: ext().blaslt_fp8_gemm(a8, b8, one, one, 1.0, dst, False), args.iters))
                    elif v == "mx":
                        times[v].append(timeit(lambda: fp8.mx_gemm(aq, bq, as_, bs), args.iters))
                        mxq.append(timeit(lambda: fp8.mx_quant(a, False, True), args.iters))
                    else:  # the hand-written kernel variant (not the hipBLASLt default of fp8.gemm)
                        fp8._FP8_GEMM_BACKEND = "hip"
                        times[v].append(timeit(lambda: fp8.gemm(a8, b8, one, one), args.iters))
                        fp8._FP8_GEMM_BACKEND = "blaslt"
            errs = {}
            if args.check:  # max |x - ref| / max |ref| against the hipBLASLt runner on the same fp8 operands
                ref = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
                ext().blaslt_fp8_gemm(a8, b8, one, one, 1.0, ref, False)
                scale = ref.float().abs().max().item()
                for v in variants:
                    if v in ("bl", "mx"):
                        continue
                    select(v)
                    fp8._FP8_GEMM_BACKEND = "hip"
                    o = fp8.gemm(a8, b8, one, one)
                    fp8._FP8_GEMM_BACKEND = "blaslt"
                    errs[v] = (o.float() - ref.float()).abs().max().item() / scale
                del ref
            ext().fp8_gemm_select(0, 0)
            row = {"gemm": f"{name}.{kind}", "M": m, "N": n, "K": k}
            for v, e_ in errs.items():
                row[f"v{v}_err"] = float(f"{e_:.3g}")
            if bf:
                ms = statistics.median(bf)
                row.update(bf16_ms=round(ms, 3), bf16_tflops=round(flops / ms / 1e9, 1))
            if smm:
                ms = statistics.median(smm)
                row.update(scaled_mm_ms=round(ms, 3), scaled_mm_tflops=round(flops / ms / 1e9, 1))
            for v in variants:
                ms = statistics.median(times[v])
                row[f"v{v}_ms"] = round(ms, 3)
                row[f"v{v}_tflops"] = round(flops / ms / 1e9, 1)
            if mxq:
                ms = statistics.median(mxq)
                row.update(mxq_ms=round(ms, 3), mxq_gbs=round(a.numel() * 4 / ms / 1e6, 1))
            print(json.dumps(row), flush=True)
            del a, b, a8, b8


if __name__ == "__main__":
    main()
