"""RCCL collective bandwidth over xGMI at the message sizes this framework issues (SURVEY §5.8 asks to verify the
channel / link use at 2/4/8 GPUs): all-gather and reduce-scatter (FSDP, one ~436 MB bf16 unit per Llama-3-8B layer),
all-reduce (DDP 128 MB buckets), all-to-all (Ulysses / EP). One JSON line per (op, bytes) on rank 0 with the median time,
algorithm bandwidth (bytes / t) and bus bandwidth (the rccl-tests convention: all-gather / reduce-scatter
algbw x (W-1)/W, all-reduce algbw x 2(W-1)/W, all-to-all algbw x (W-1)/W), which a fully used set of 7 links per
GPU puts near 7 x ~150 GB/s.

    python -m torch.distributed.run --nproc-per-node 8 tools/bench_rccl.py [--max-mb 1024] [--dtype bf16]
    python -m torch.distributed.run --nproc-per-node 2 tools/bench_rccl.py --cpu --max-mb 4     # gloo plumbing check
"""

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--min-mb", type=float, default=1.0)
    p.add_argument("--max-mb", type=float, default=1024.0)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--ops", default="all_gather,reduce_scatter,all_reduce,all_to_all")
    p.add_argument("--cpu", action="store_true")
    a = p.parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.cpu:
        dist.init_process_group("gloo")
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        from accelerate_hpc_test_amd.parallel.topology import validate_comm_environment

        if local == 0:
            validate_comm_environment(int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    W, r = dist.get_world_size(), dist.get_rank()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = torch.tensor([], dtype=dt).element_size()
    sync = (lambda: None) if a.cpu else torch.cuda.synchronize
    gloo = a.cpu
    mb = a.min_mb
    sizes = []
    while mb <= a.max_mb + 1e-9:
        sizes.append(int(mb * (1 << 20)) // (es * W) * W)  # elements, divisible by W
        mb *= 2
    for op in a.ops.split(","):
        for n in sizes:
            full = torch.ones(n, dtype=dt, device=dev)
            shard = torch.ones(n // W, dtype=dt, device=dev)
            if op == "all_gather":
                fn = (lambda: dist.all_gather(list(full.chunk(W)), shard)) if gloo else (lambda: dist.all_gather_into_tensor(full, shard))
                factor = (W - 1) / W
            elif op == "reduce_scatter":
                if gloo:
                    continue
                fn = lambda: dist.reduce_scatter_tensor(shard, full)  # noqa: E731
                factor = (W - 1) / W
            elif op == "all_reduce":
                fn = lambda: dist.all_reduce(full)  # noqa: E731
                factor = 2 * (W - 1) / W
            elif op == "all_to_all":
                if gloo:
                    continue
                out = torch.empty_like(full)
                fn = lambda: dist.all_to_all_single(out, full)  # noqa: E731
                factor = (W - 1) / W
            else:
                raise ValueError(op)
            for _ in range(2):
                fn()
            sync()
            times = []
            for _ in range(a.iters):
                dist.barrier()
                sync()
                t = time.perf_counter()
                fn()
                sync()
                times.append(time.perf_counter() - t)
            tt = torch.tensor([statistics.median(times)], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt)
            nbytes = n * es
            if r == 0:
                print(json.dumps({"op": op, "world": W, "bytes": nbytes, "ms": round(t * 1e3, 4),
                                  "algbw_GBs": round(nbytes / t / 1e9, 2), "busbw_GBs": round(nbytes / t / 1e9 * factor, 2),
                                  "dtype": a.dtype, "backend": "gloo" if gloo else "rccl"}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
