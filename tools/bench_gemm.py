"""GEMM throughput at the Llama-3-8B linear shapes: fp8 (our MX-MFMA kernels, v1 128² / v2 256² glds) vs bf16
hipBLASLt (torch.matmul). Prints one JSON line per shape and variant.

    python tools/bench_gemm.py [--tokens 8192] [--iters 20]
"""

import argparse
import json
import os
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
    args = p.parse_args()
    from accelerate_hpc_test_amd.ops import fp8, gemm_tuning

    gemm_tuning.load_tuned_gemms()
    T = args.tokens
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    one = torch.ones(1, device="cuda")
    for name, (N, K) in shapes.items():
        # forward (x·Wᵀ), dgrad (dy·W → [T,K] from [T,N]·[N,K]), wgrad (dyᵀ·x → [N,K])
        for kind, (m, n, k) in {"fwd": (T, N, K), "dgrad": (T, K, N), "wgrad": (N, K, T)}.items():
            a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
            flops = 2.0 * m * n * k
            ms_bf16 = timeit(lambda: a @ b.t(), args.iters)
            a8, b8 = fp8.cast(a, one), fp8.cast(b, one)
            # the kernel choice (v2, or v1 with ACCELERATE_FP8_GEMM_V1=1) is fixed per process
            ms_v2 = timeit(lambda: fp8.gemm(a8, b8, one, one), args.iters)
            print(json.dumps({"gemm": f"{name}.{kind}", "M": m, "N": n, "K": k, "fp8_kernel": "v1" if os.environ.get("ACCELERATE_FP8_GEMM_V1") else "v2",
                              "bf16_ms": round(ms_bf16, 3), "bf16_tflops": round(flops / ms_bf16 / 1e9, 1),
                              "fp8_ms": round(ms_v2, 3), "fp8_tflops": round(flops / ms_v2 / 1e9, 1)}), flush=True)
            del a, b, a8, b8


if __name__ == "__main__":
    main()
