"""Diagnose the hand-scheduled fp8 GEMM (variant 18) on small shapes: error maps by output position class."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from accelerate_hpc_test_amd.ops import fp8
from accelerate_hpc_test_amd.ops._ext import ext

fp8._FP8_GEMM_BACKEND = "hip"
one = torch.ones(1, device="cuda")


def run(a, b, v):
    ext().fp8_gemm_select(v)
    o = fp8.gemm(fp8.cast(a, one), fp8.cast(b, one), one, one, out_dtype=torch.float32)
    torch.cuda.synchronize()
    return o


for (M, N, K) in [(256, 256, 256), (256, 256, 384), (512, 512, 512)]:
    ones_a = torch.ones(M, K, device="cuda", dtype=torch.bfloat16)
    ones_b = torch.ones(N, K, device="cuda", dtype=torch.bfloat16)
    o = run(ones_a, ones_b, 18)
    vals, cnts = torch.unique(o, return_counts=True)
    print(f"[{M}x{N}x{K}] ones: values {vals[:12].tolist()} counts {cnts[:12].tolist()}", flush=True)
    torch.manual_seed(0)
    a = torch.randint(-3, 4, (M, K), device="cuda").to(torch.bfloat16)
    b = torch.randint(-3, 4, (N, K), device="cuda").to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    o = run(a, b, 18)
    bad = (o != ref)
    nonint = (o != o.round())
    print(f"  rand: wrong {bad.float().mean().item():.3f}, non-integer {nonint.float().mean().item():.3f}", flush=True)
    r = torch.arange(M, device="cuda").view(-1, 1).expand(M, N)
    c = torch.arange(N, device="cuda").view(1, -1).expand(M, N)
    for name, key in [("row%8 (i)", r % 8), ("col%8 (j)", c % 8), ("(row%128)//32 (g)", (r % 128) // 32),
                      ("(row%32)//8 (q)", (r % 32) // 8), ("(col%128)//8 (lane r)", (c % 128) // 8),
                      ("row//128 (wm)", (r % 256) // 128), ("col//128 (wn)", (c % 256) // 128)]:
        ks = sorted(set(key.flatten().tolist()))
        frac = [round(bad[key == k].float().mean().item(), 2) for k in ks]
        print(f"    {name}: {frac}", flush=True)
    # one-hot K probe: A[:, k0] = 1 only, B = ones -> C = 1 iff column k0 is consumed
    for k0 in (0, 15, 16, 64, 127, 128, 200):
        if k0 >= K:
            continue
        a1 = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
        a1[:, k0] = 1
        o = run(a1, ones_b, 18)
        print(f"    one-hot k={k0}: mean {o.mean().item():.3f} min {o.min().item():.1f} max {o.max().item():.1f}", flush=True)
ext().fp8_gemm_select(0)
