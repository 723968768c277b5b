"""The fused AdamW multi-tensor kernel alone at Llama-3-8B scale: fp32 master weights, fp32 grads, bf16 moments
(ACCELERATE_ADAM_STATE_DTYPE=bf16, the bench's setting), 32 layers of the real shapes plus embedding and lm_head
(8.03 B parameters; 20 bytes each per step here: no bf16 shadow without an FSDP engine, 22 in the step). Prints ms and effective TB/s; the kernel's memory-access form comes from
ACCELERATE_ADAM_NT (0 flat, 1 global, 2 global non-temporal = default), read once per process.

    ACCELERATE_ADAM_NT=2 python tools/bench_adam.py [--iters 10]"""
import argparse
import json
import os
import sys

os.environ.setdefault("ACCELERATE_ADAM_STATE_DTYPE", "bf16")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from accelerate_hpc_test_amd.ops.multi_tensor import FusedAdamStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    shapes = [(128256, 4096), (128256, 4096)] + [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)] * 32
    params = [torch.nn.Parameter(torch.randn(s, device="cuda") * 0.02) for s in shapes]
    for p in params:
        p.grad = torch.randn_like(p) * 1e-3
    opt = torch.optim.AdamW(params, lr=1e-5, weight_decay=0.1)
    step = FusedAdamStep(opt)
    n = sum(p.numel() for p in params)
    for _ in range(2):
        step.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        step.step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(json.dumps({"adam_nt": os.environ.get("ACCELERATE_ADAM_NT", "0"), "params": n, "ms": round(ms, 3),
                      "tb_per_s_at_20B": round(20 * n / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
