"""RMSNorm backward alone at the Llama-3-8B step shape (T = 8192 tokens, H = 4096, residual gradient added, dweight
accumulated into an fp32 slot): ms per call and effective TB/s (dy, x, dres read, dx written). The workgroup count comes
from ACCELERATE_RMSNORM_BWD_BLOCKS (read once per process).

    ACCELERATE_RMSNORM_BWD_BLOCKS=1024 python tools/bench_rmsnorm_bwd.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from accelerate_hpc_test_amd.ops._ext import ext  # noqa: E402

T, H = 8192, 4096
dy, x, dres = (torch.randn(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(3))
w = torch.rand(H, device="cuda", dtype=torch.bfloat16) + 0.5
rstd = torch.rand(T, device="cuda") + 0.5
dw = torch.zeros(H, device="cuda")
e = ext()
for _ in range(3):
    e.rmsnorm_bwd(dy, x, w, rstd, dres, None, dw, True)
torch.cuda.synchronize()
s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 50
s.record()
for _ in range(n):
    e.rmsnorm_bwd(dy, x, w, rstd, dres, None, dw, True)
t.record()
t.synchronize()
ms = s.elapsed_time(t) / n
print(json.dumps({"blocks": os.environ.get("ACCELERATE_RMSNORM_BWD_BLOCKS", "512"), "ms": round(ms, 4),
                  "tb_per_s": round(4 * T * H * 2 / ms / 1e9, 2)}), flush=True)
