"""Transpose kernel bandwidth at the shapes the step transposes (layer inputs, dy, weights): both kernels.

    python tools/bench_transpose.py      (one JSON line per shape; GB/s counts read + write)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from accelerate_hpc_test_amd.ops._ext import ext  # noqa: E402


def tm(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e3


for shape in [(8192, 4096), (8192, 14336), (8192, 28672), (8192, 6144), (28672, 4096), (4096, 14336), (8192, 128256)]:
    x = torch.randn(shape, device="cuda", dtype=torch.bfloat16)
    ms = tm(lambda: ext().transpose_bf16(x))
    ref = tm(lambda: x.t().contiguous())
    ok = torch.equal(ext().transpose_bf16(x), x.t().contiguous())
    gb = 2 * x.numel() * 2 / 1e9
    print(json.dumps({"shape": shape, "ms": round(ms, 4), "GBps": round(gb / ms * 1e3), "torch_ms": round(ref, 4),
                      "torch_GBps": round(gb / ref * 1e3), "exact": ok}), flush=True)
    del x
