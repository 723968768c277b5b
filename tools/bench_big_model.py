"""BASELINE config #4: Llama-3-70B big-model inference with `dispatch_model(device_map="auto")` across the visible
MI355X GPUs, optionally forcing part of the model to pinned host memory (offload streamed back with the async
HIP-stream prefetcher in hooks.py).

Random-init weights are materialised directly on their target device (no checkpoint exists offline; writing a
140 GB synthetic one would only measure the disk), then the hooked model runs prefill forwards.

    python tools/bench_big_model.py --model llama3-70b --gpu-mem 100GiB --tokens 2048 --iters 3
"""

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-70b")
    p.add_argument("--gpu-mem", default=None, help="per-GPU budget for the device map, e.g. 100GiB (forces host offload)")
    p.add_argument("--cpu-mem", default="200GiB")
    p.add_argument("--tokens", type=int, default=2048)
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--iters", type=int, default=3)
    args = p.parse_args()

    from accelerate_hpc_test_amd import dispatch_model, infer_auto_device_map, init_empty_weights
    from accelerate_hpc_test_amd.utils.placement import set_module_tensor_to_device
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM, RMSNorm

    cfg = LLAMA_PRESETS[args.model]
    with init_empty_weights():
        model = LlamaForCausalLM(cfg)
    n_gpu = torch.cuda.device_count()
    max_memory = {i: (args.gpu_mem or "270GiB") for i in range(n_gpu)}
    max_memory["cpu"] = args.cpu_mem
    t0 = time.time()
    device_map = infer_auto_device_map(model, max_memory=max_memory, no_split_module_classes=["LlamaDecoderLayer"], dtype=torch.bfloat16)
    t_plan = time.time() - t0
    placement = {}
    for name, dev in device_map.items():
        placement[str(dev)] = placement.get(str(dev), 0) + 1
    # materialise on the target devices (GPU: N(0, .02) generated in place; CPU: pinned host memory)
    t0 = time.time()
    host_bytes = 0
    for name, param in list(model.named_parameters()):
        dev = None
        for prefix in sorted(device_map, key=len, reverse=True):
            if name == prefix or name.startswith(prefix + ".") or prefix == "":
                dev = device_map[prefix]
                break
        is_norm = name.endswith("layernorm.weight") or name == "norm.weight"
        if dev in ("cpu", "disk"):
            # random values drawn on the GPU and copied into pinned host memory (a CPU normal_ over ~100 GB takes
            # many minutes)
            t = torch.empty(param.shape, dtype=torch.bfloat16, pin_memory=True)
            src = torch.empty(param.shape, dtype=torch.bfloat16, device="cuda:0")
            src.fill_(1.0) if is_norm else src.normal_(0.0, 0.02)
            t.copy_(src)
            del src
            host_bytes += t.numel() * 2
            if host_bytes // (8 << 30) != (host_bytes - t.numel() * 2) // (8 << 30):
                print(f"materialised {host_bytes / 2**30:.0f} GiB of host-offloaded weights", flush=True)
            set_module_tensor_to_device(model, name, "cpu", value=t, dtype=torch.bfloat16)
        else:
            t = torch.empty(param.shape, dtype=torch.bfloat16, device=f"cuda:{dev}")
            t.fill_(1.0) if is_norm else t.normal_(0.0, 0.02)
            set_module_tensor_to_device(model, name, f"cuda:{dev}", value=t, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t_mat = time.time() - t0
    t0 = time.time()
    model = dispatch_model(model, device_map)
    t_dispatch = time.time() - t0
    ids = torch.randint(0, cfg.vocab_size, (args.batch, args.tokens), device="cuda:0")
    with torch.no_grad():
        model(ids, return_logits=False)  # warmup (also pins/uploads once)
        torch.cuda.synchronize()
        print("warmup forward done", flush=True)
        t0 = time.perf_counter()
        for i in range(args.iters):
            model(ids, return_logits=False)
            torch.cuda.synchronize()
            print(f"forward {i} done", flush=True)
        dt = (time.perf_counter() - t0) / args.iters
    rec = {
        "metric": "prefill tokens/s, Llama big-model dispatch (device_map=auto)",
        "model": args.model,
        "value": round(args.batch * args.tokens / dt, 1),
        "unit": "tokens/s",
        "ms_per_forward": round(dt * 1000, 1),
        "n_gpus": n_gpu,
        "placement_counts": placement,
        "host_offload_gib": round(host_bytes / 2**30, 1),
        "h2d_gib_per_s_effective": round(host_bytes / 2**30 / dt, 1) if host_bytes else None,
        "plan_s": round(t_plan, 2),
        "materialize_s": round(t_mat, 1),
        "dispatch_s": round(t_dispatch, 2),
        "data": "synthetic tokens, random-init bf16 weights",
    }
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
