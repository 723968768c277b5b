"""bf16 input-gradient GEMM dx = dy · W at the Llama-3-8B linear shapes (8192 tokens), three ways, in ONE process and
interleaved rounds on random data:

  wt      — HIP transpose of W into a contiguous Wᵀ + the forward-layout (TN) GEMM (the current default);
  nn      — `dy @ W` through torch (hipBLASLt's first heuristic choice for the NN layout);
  searched— the NN layout on the searched hipBLASLt runner (csrc/runtime/blaslt_gemm.cpp::blaslt_dgrad_bf16).

Also checks every variant against the fp32 product. One JSON line per shape.

    python tools/bench_dgrad.py [--tokens 8192] [--iters 20] [--rounds 3]
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
    args = p.parse_args()
    from accelerate_hpc_test_amd.ops import gemm_tuning
    from accelerate_hpc_test_amd.ops._ext import ext

    gemm_tuning.load_tuned_gemms()
    T = args.tokens
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for name, (N, K) in shapes.items():
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        out = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
        ref = dy.float() @ w.float()
        variants = {
            "wt": lambda: torch.nn.functional.linear(dy, ext().transpose_bf16(w)),
            "nn": lambda: dy @ w,
            "searched": lambda: ext().blaslt_dgrad_bf16(dy, w, out) and out,
        }
        errs = {}
        for k, fn in variants.items():
            r = fn()
            errs[k] = round(((r.float() - ref).norm() / ref.norm()).item(), 5) if torch.is_tensor(r) else None
        times = {k: [] for k in variants}
        for _ in range(args.rounds):
            for k, fn in variants.items():
                times[k].append(timeit(fn, args.iters))
        flops = 2.0 * T * N * K
        row = {"gemm": f"{name}.dgrad", "T": T, "N": N, "K": K, "rel_err": errs}
        for k, v in times.items():
            ms = statistics.median(v)
            row[f"{k}_ms"] = round(ms, 3)
            row[f"{k}_tflops"] = round(flops / ms / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
