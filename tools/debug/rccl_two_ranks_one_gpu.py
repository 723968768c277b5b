"""Probe: can two RCCL ranks share one GPU on this image? Answer measured on MI355X (round 3): no, RCCL 2.26.6 fails
the communicator init with "Duplicate GPU detected : rank 1 and rank 0 both on CUDA device". Multi-rank rehearsal on
one GPU therefore runs over gloo with HIP tensors (tests/test_gpu_multirank.py)."""
import os

import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((1 << 20,), float(dist.get_rank() + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {dist.get_rank()}: all_reduce ok={bool((t == 3).all())}", flush=True)
dist.destroy_process_group()
