"""Weight-gradient GEMM layouts at the Llama-3-8B shapes (T = 8192 tokens), fp32 output (the FSDP world-size-1 path):
  nt : dW = dyᵀ·x with both operands token-major (what autograd has)           -> mm(dy.t(), x)
  nn : same product with x pre-transposed once (xT = xᵀ contiguous)             -> mm(dy.t(), xT.t())
  tt : both operands pre-transposed (dyT = dyᵀ, xT = xᵀ contiguous, the forward's NT class) -> mm(dyT, xT.t())
plus the cost of producing xT / dyT, and the layouts with a bf16 output (the flat-grad-buffer path at world size > 1),
and the same GEMMs through hipBLASLt with a per-problem algorithm search (`ext().blaslt_wgrad_f32`, nt layout).
Prints one JSON line per shape."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from accelerate_hpc_test_amd.ops import gemm_tuning

gemm_tuning.load_tuned_gemms()
T = 8192
def tm(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e3
for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}.items():
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.float32)
    xT = x.t().contiguous()
    fl = 2.0 * T * N * K
    nt = tm(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out))
    nn_ = tm(lambda: torch.mm(dy.t(), xT.t(), out_dtype=torch.float32, out=out))
    tr = tm(lambda: x.t().contiguous())
    ob = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    nt16 = tm(lambda: torch.mm(dy.t(), x, out=ob))
    nn16 = tm(lambda: torch.mm(dy.t(), xT.t(), out=ob))
    dyT = dy.t().contiguous()
    tt = tm(lambda: torch.mm(dyT, xT.t(), out_dtype=torch.float32, out=out))
    tt16 = tm(lambda: torch.mm(dyT, xT.t(), out=ob))
    trdy = tm(lambda: dy.t().contiguous())
    from accelerate_hpc_test_amd.ops._ext import ext
    bl = tm(lambda: ext().blaslt_wgrad_f32(dy, x, out, False))
    blx = tm(lambda: ext().blaslt_wgrad_f32(dy, xT, out, False, True))
    ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
    err = (torch.mm(dy.t(), xT.t(), out_dtype=torch.float32) - ref).abs().max().item()
    print(json.dumps({"gemm": name, "nt_ms": round(nt, 3), "nt_tflops": round(fl / nt / 1e9), "nn_ms": round(nn_, 3),
                      "nn_tflops": round(fl / nn_ / 1e9), "transpose_x_ms": round(tr, 3), "nt_bf16_ms": round(nt16, 3), "nn_bf16_ms": round(nn16, 3), "tt_ms": round(tt, 3), "tt_tflops": round(fl / tt / 1e9),
                      "tt_bf16_ms": round(tt16, 3), "transpose_dy_ms": round(trdy, 3), "blaslt_search_nt_ms": round(bl, 3), "blaslt_search_xt_ms": round(blx, 3),
                      "max_abs_diff": err}), flush=True)
