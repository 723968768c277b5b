"""Fused multi-tensor AdamW bandwidth: fp32 master / fp32 grad / fp32 moments + bf16 shadow (the FSDP world-size-1 step
of the 8B bench), on `--params` elements split into 64 Mi-element tensors. Reports ms per step and the effective HBM
bandwidth at 30 bytes per parameter (read p, g, m, v; write p, m, v, shadow).

    python tools/bench_adam.py [--params 2e9] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=float, default=2e9)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from accelerate_hpc_test_amd.ops.multi_tensor import FusedAdamStep

    n_total = int(args.params)
    chunk = 64 << 20
    ps = []
    left = n_total
    while left > 0:
        n = min(chunk, left)
        p = torch.nn.Parameter(torch.randn(n, device="cuda"))
        p.grad = torch.randn(n, device="cuda") * 1e-3
        p._acc_bf16_shadow = torch.empty(n, device="cuda", dtype=torch.bfloat16)
        ps.append(p)
        left -= n
    opt = torch.optim.AdamW(ps, lr=1e-5, weight_decay=0.01)
    step = FusedAdamStep(opt)
    for _ in range(2):
        step.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        step.step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"params": n_total, "ms_per_step": round(ms, 3), "tb_per_s": round(30 * n_total / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
