"""bf16 GEMM throughput at the Llama-3-8B linear shapes: the asm-scheduled kernel (ext().bf16_gemm_asm, the fp8
kernel's schedule with bf16 MFMAs) vs hipBLASLt through torch (a @ bᵀ, both operands contraction-contiguous, the
forward-class "TN" layout) and, for wgrad, torch on the layout the step would otherwise use (fp32 out).

    python tools/bench_gemm_bf16.py [--tokens 8192] [--iters 20] [--rounds 3]"""
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
    args = p.parse_args()
    from accelerate_hpc_test_amd.ops._ext import ext

    T = args.tokens
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336), "lm_head": (128256, 4096)}
    for name, (N, K) in shapes.items():
        for kind, (m, n, k) in {"fwd": (T, N, K), "dgrad": (T, K, N), "wgrad": (N, K, T)}.items():
            a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16)
            out_dt = torch.float32 if kind == "wgrad" else torch.bfloat16
            o1 = torch.empty(m, n, device="cuda", dtype=out_dt)
            o2 = torch.empty(m, n, device="cuda", dtype=out_dt)
            flops = 2.0 * m * n * k
            ref = (a @ b.t()) if out_dt == torch.bfloat16 else torch.mm(a, b.t(), out_dtype=torch.float32)
            assert ext().bf16_gemm_asm(a, b, None, o2, False)
            err = ((o2.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            tt, ta = [], []
            for _ in range(args.rounds):
                if out_dt == torch.bfloat16:
                    tt.append(timeit(lambda: torch.mm(a, b.t(), out=o1), args.iters))
                else:
                    tt.append(timeit(lambda: torch.mm(a, b.t(), out_dtype=torch.float32, out=o1), args.iters))
                ta.append(timeit(lambda: ext().bf16_gemm_asm(a, b, None, o2, False), args.iters))
            mt, ma = statistics.median(tt), statistics.median(ta)
            print(json.dumps({"gemm": f"{name}.{kind}", "M": m, "N": n, "K": k, "out": str(out_dt)[6:],
                              "hipblaslt_tflops": round(flops / mt / 1e9, 1), "asm_tflops": round(flops / ma / 1e9, 1),
                              "asm_vs_hipblaslt": round(mt / ma, 3), "asm_rel_err": float(f"{err:.3g}")}), flush=True)
            del a, b, o1, o2, ref


if __name__ == "__main__":
    main()
