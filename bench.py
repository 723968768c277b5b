#!/usr/bin/env python
"""Headline benchmark: Llama-3-8B FSDP2 bf16 training throughput (tokens/s, whole node) on 1/2/4/8 MI355X.

Reference workload: `examples/torch_native_parallelism/fsdp2_fp8.py` — Llama-3.1-8B, seq 8192,
micro-batch 1 per device, AdamW(lr=1e-5), FSDP2 transformer-wrap of LlamaDecoderLayer, bf16 mixed precision,
forward / backward / optimizer.step / zero_grad each step. The reference builds the model with torch_dtype=bfloat16
(`fsdp2_fp8.py:88-97`), so its AdamW holds bf16 params and bf16 moments; here the params stay fp32 masters (bf16
shadows feed the all-gather) and the moments are bf16 (`--adam-states fp32` for fp32 moments). Same here, on this
framework's stack:
`Accelerator(fsdp_plugin=FSDP2, mixed_precision="bf16")` → native FSDP engine (RCCL all-gather / reduce-scatter per
decoder layer on side streams), HIP kernels (flash attention, RMSNorm, RoPE, SwiGLU, cross-entropy, fused AdamW),
hipBLASLt GEMMs. Synthetic token data (random ids) and random-init weights (no network access).

Usage: python bench.py [--gpus N --steps K --warmup W]   (N>1: launched by torch.distributed.run, one rank per GPU)
Prints ONE JSON line on rank 0.
"""

import argparse
import json
import os
import time

import torch

BASELINE_TOKENS_PER_SEC_PER_DEVICE = 8000.0  # BASELINE.md P1 (8x H100, Llama-3.1-8B FSDP2 bf16)
BASELINE_FP8_TOKENS_PER_SEC_PER_DEVICE = 10000.0  # BASELINE.md P2 (same, torchao fp8)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--seq", type=int, default=8192)
    p.add_argument("--mbs", type=int, default=1)
    p.add_argument("--adam-states", default="bf16", choices=["fp32", "bf16"],
                   help="dtype of the AdamW moments beside the fp32 master weights (ACCELERATE_ADAM_STATE_DTYPE). The "
                        "reference's config builds the model in bf16, so its AdamW keeps bf16 params AND bf16 moments; "
                        "bf16 moments + fp32 master stays at or above that precision in every state")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp8", "mxfp8"],
                   help="fp8: dynamic per-tensor scaling (torchao recipe); mxfp8: TE MXFP8BlockScaling (e8m0 scale per "
                        "32 elements, applied inside the MFMA)")
    p.add_argument("--parallel", default="fsdp", choices=["fsdp", "ddp"],
                   help="fsdp: FSDP2 full shard (headline); ddp: replicated fp32 params + bf16 autocast, RCCL all-reduce "
                        "(BASELINE config 'Llama-3 8B DDP bf16')")
    p.add_argument("--ddp-comm-hook", default="no", choices=["no", "bf16", "fp16"])
    p.add_argument("--activation-checkpointing", action="store_true")
    p.add_argument("--prefetch", type=int, default=1)
    p.add_argument("--reshard-after-forward", default="on", choices=["on", "off"],
                   help="off: keep each unit's gathered bf16 parameters from its forward to its backward (ZeRO-2 style; "
                        "16 GB for Llama-3-8B, small against 288 GB of HBM) so the backward issues no second all-gather")
    p.add_argument("--optimizer-overlap", default="off", choices=["on", "off"],
                   help="on: each FSDP unit's AdamW update runs on a side HIP stream as soon as its gradient is final, "
                        "overlapped with the rest of the backward (RcclKwargs.fsdp_optimizer_overlap); optimizer.step() "
                        "still ends every step inside the timed region")
    p.add_argument("--fsdp-force-sharded", action="store_true",
                   help="at 1 GPU: run the FSDP engine's multi-GPU code path (full buffers resized 0<->full, RCCL "
                        "all-gather / reduce-scatter with nranks=1, bf16 flat grads) instead of the no-collective shortcut")
    p.add_argument("--ddp-force", action="store_true",
                   help="with --parallel ddp at 1 GPU: wrap the model in the DDP reducer anyway (buckets, hooks, RCCL "
                        "all-reduce with nranks=1 on its own communicator) instead of running it unwrapped")
    p.add_argument("--fsdp-cpu-offload", action="store_true",
                   help="FSDP CPU offload: fp32 master/grad shards + AdamW state in pinned host memory, host AdamW")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--no-preflight", action="store_true",
                   help="skip the N>1 communicator self-test (known-value AG/RS/all-reduce + bus bandwidth per group)")
    p.add_argument("--cpu", action="store_true",
                   help="contract check only: run the same loop on CPU ranks (gloo) with a small --model; not a benchmark")
    p.add_argument("--gemm-tuning", default="auto", choices=["auto", "off", "tune"],
                   help="auto: load the committed hipBLASLt per-shape table (ops/tuned); tune: search and write it")
    p.add_argument("--gemm-table", default=None, help="table path for --gemm-tuning auto/tune")
    return p.parse_args()


class SyntheticTokens(torch.utils.data.Dataset):
    """Random token ids of one packed sequence per item (deterministic per index)."""

    def __init__(self, n, seq, vocab):
        self.n, self.seq, self.vocab = n, seq, vocab

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(1234 + i)
        ids = torch.randint(0, self.vocab, (self.seq,), generator=g)
        return {"input_ids": ids, "labels": ids}


def _metric_name(args, is_moe):
    if args.model == "llama3-8b" and args.parallel == "fsdp" and args.precision == "bf16":
        return "tokens/sec (whole node) Llama-3-8B FSDP2 bf16 at 1/2/4/8 MI355X"
    name = "Llama-3-8B" if args.model == "llama3-8b" else args.model
    return f"tokens/sec (whole node) {name} {'FSDP2' if args.parallel == 'fsdp' else 'DDP'} {args.precision}"


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run as a CHILD process (no
    exec, and nothing in this parent touches the GPU) and return its exit code. Each rank re-enters this file with
    WORLD_SIZE set, so only the ranks ever initialise HIP."""
    import subprocess
    import sys

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.adam_states == "bf16":
        os.environ["ACCELERATE_ADAM_STATE_DTYPE"] = "bf16"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    launched_world = os.environ.get("WORLD_SIZE")
    if launched_world is None and args.gpus > 1:
        raise SystemExit(_spawn_ranks(args.gpus))
    if launched_world is not None and int(launched_world) != args.gpus:
        raise SystemExit(f"bench.py: launched with WORLD_SIZE={launched_world} but --gpus {args.gpus}; they must match")
    # A hung collective must end the run non-zero (communicators aborted, rank exits) instead of holding the node
    # until the outer time limit: the step watchdog fires after this many seconds without a heartbeat.
    os.environ.setdefault("ACCELERATE_WATCHDOG_TIMEOUT", "600")
    os.environ.setdefault("ACCELERATE_WATCHDOG_ACTION", "abort")
    from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin
    from accelerate_hpc_test_amd.models import LLAMA_PRESETS, MIXTRAL_PRESETS, LlamaForCausalLM, MixtralForCausalLM

    is_moe = args.model in MIXTRAL_PRESETS
    model_cls = MixtralForCausalLM if is_moe else LlamaForCausalLM
    from accelerate_hpc_test_amd.utils import RcclKwargs, set_seed

    plugin = FullyShardedDataParallelPlugin(
        fsdp_version=2,
        auto_wrap_policy="transformer_based_wrap",
        transformer_cls_names_to_wrap=list(model_cls._no_split_modules),
        reshard_after_forward=args.reshard_after_forward == "on",
        activation_checkpointing=args.activation_checkpointing,
        cpu_offload=args.fsdp_cpu_offload,
    )
    overlap = args.optimizer_overlap == "on" and args.parallel == "fsdp"
    force = args.fsdp_force_sharded and args.parallel == "fsdp"
    force_ddp = args.ddp_force and args.parallel == "ddp"
    if (force or force_ddp) and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not torch.distributed.is_initialized():
        # a one-rank RCCL process group so the sharded path has real collectives to issue
        torch.cuda.set_device(0)
        port = int(os.environ.get("MASTER_PORT", "29533"))
        torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                             device_id=torch.device("cuda", 0))
    handlers = [RcclKwargs(fsdp_prefetch_depth=args.prefetch, fsdp_optimizer_overlap=overlap, fsdp_force_sharded=force,
                           ddp_force=force_ddp)]
    if args.parallel == "ddp":
        from accelerate_hpc_test_amd.utils import DDPCommunicationHookType, DistributedDataParallelKwargs

        plugin = None
        handlers.append(DistributedDataParallelKwargs(comm_hook=DDPCommunicationHookType(args.ddp_comm_hook)))
    if args.precision == "mxfp8":
        from accelerate_hpc_test_amd.utils import TERecipeKwargs

        handlers.append(TERecipeKwargs(use_mxfp8_block_scaling=True))
    mp = "fp8" if args.precision == "mxfp8" else args.precision
    accelerator = Accelerator(mixed_precision=mp, fsdp_plugin=plugin, kwargs_handlers=handlers, cpu=args.cpu)
    sync = (lambda: None) if args.cpu else torch.cuda.synchronize
    set_seed(0)
    world = accelerator.num_processes
    from accelerate_hpc_test_amd.ops import gemm_tuning

    gemm_table = None
    if args.gemm_tuning == "tune":
        gemm_table = args.gemm_table or os.path.join("gpurun_out", "tunableop_gfx950.csv")
        gemm_tuning.start_gemm_tuning(gemm_table)
    elif args.gemm_tuning == "auto":
        gemm_table = (args.gemm_table or gemm_tuning.DEFAULT_TABLE) if gemm_tuning.load_tuned_gemms(args.gemm_table) else None
    cfg = (MIXTRAL_PRESETS if is_moe else LLAMA_PRESETS)[args.model]

    t0 = time.time()
    with torch.device("meta"):
        model = model_cls(cfg)
    if args.parallel == "ddp":  # every rank holds the whole fp32 model (8B: 32 GB params + 32 GB grads + 64 GB Adam)
        model.to_empty(device=accelerator.device)
        model.init_weights()
    optimizer = torch.optim.AdamW(model.parameters(), lr=1e-5)
    total_steps = args.warmup + args.steps
    ds = SyntheticTokens(total_steps * args.mbs * world, args.seq, cfg.vocab_size)
    dl = torch.utils.data.DataLoader(ds, batch_size=args.mbs, num_workers=2)
    model, optimizer, dl = accelerator.prepare(model, optimizer, dl)
    model.train()
    sync()
    accelerator.heartbeat("prepared")
    preflight = None
    if world > 1 and not args.no_preflight:
        # every communicator the run uses, checked before training: a broken one ends the run with a JSON line that
        # names it (exit 3) instead of a hang in the first all-gather
        from accelerate_hpc_test_amd.utils.preflight import preflight_model

        preflight = preflight_model(model, accelerator.device, big_bytes=(1 << 20) if args.cpu else (436 << 20))
        accelerator.heartbeat("preflight")
        if args.verbose:
            accelerator.print(f"preflight: {json.dumps(preflight)}", flush=True)
    if args.verbose and accelerator.is_main_process and not args.cpu:
        print(f"setup {time.time() - t0:.1f}s, mem {torch.cuda.memory_allocated() / 2**30:.1f} GiB", flush=True)

    it = iter(dl)
    last_loss = None

    def step():
        nonlocal last_loss
        batch = next(it)
        out = model(batch["input_ids"], labels=batch["labels"], return_logits=False)
        accelerator.backward(out.loss)
        optimizer.step()
        optimizer.zero_grad()
        last_loss = out.loss.detach()

    for i in range(args.warmup):
        tw = time.time()
        step()
        if args.verbose:
            sync()
            accelerator.print(f"warmup step {i}: {time.time() - tw:.3f}s loss {last_loss.item():.4f}", flush=True)
    if args.gemm_tuning == "tune":
        gemm_tuning.finish_gemm_tuning()  # search done during warmup; the timed steps use the tuned table

    accelerator.wait_for_everyone()
    sync()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    accelerator.wait_for_everyone()
    elapsed = time.perf_counter() - t_start

    el = torch.tensor([elapsed], device=accelerator.device, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = el.item()
    tokens = args.steps * args.mbs * args.seq * world
    tps = tokens / elapsed
    ms = elapsed / args.steps * 1000
    flops_tok = cfg.flops_per_token(args.seq)
    peak = 0.0 if args.cpu else torch.cuda.max_memory_allocated() / 2**30
    if args.verbose and not args.cpu:
        mst = torch.cuda.memory_stats()
        if args.precision == "fp8":
            from accelerate_hpc_test_amd.ops._ext import ext as _ext

            plans = _ext().blaslt_fp8_plans()
            accelerator.print(f"hipBLASLt fp8 problems: {len(plans)}, declined {sum(1 for p in plans if p[4] < 0)}: "
                              f"{[p[:3] for p in plans if p[4] < 0]}", flush=True)
        accelerator.print(f"allocator: alloc_retries {mst.get('num_alloc_retries', 0)}, reserved peak "
                          f"{mst.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB, device frees "
                          f"{mst.get('num_device_free', 0)}", flush=True)
    headline = args.model == "llama3-8b" and args.parallel == "fsdp"
    base_dev = BASELINE_FP8_TOKENS_PER_SEC_PER_DEVICE if args.precision in ("fp8", "mxfp8") else BASELINE_TOKENS_PER_SEC_PER_DEVICE
    if accelerator.is_main_process:
        rec = {
            "metric": _metric_name(args, is_moe),
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(tps / (base_dev * world), 3) if headline else None,
            "dtype": args.precision,
            "data": "synthetic (random token ids, random-init weights)",
            "config": {
                "model": "Llama-3-8B" if args.model.startswith("llama3") and "8b" in args.model else args.model,
                "moe": {"experts": cfg.num_local_experts, "top_k": cfg.num_experts_per_tok} if is_moe else None,
                "global_batch": args.mbs * world,
                "seq_len": args.seq,
                # "-w1": one rank, the engine's no-collective path; "-forced-sharded": one rank running the multi-rank code
                "parallelism": f"{args.parallel}-w{world}" + ("-forced-sharded" if force else "")
                + ("-forced-reducer" if force_ddp else "")
                + ("-shard-grad-op" if args.parallel == "fsdp" and args.reshard_after_forward == "off" else ""),
                "optimizer": "AdamW(lr=1e-5), fp32 master" + (", bf16 moments" if args.adam_states == "bf16" else "")
                + (", per-unit update overlapped with backward" if overlap else "")
                + (", CPU-offloaded (host AdamW)" if args.fsdp_cpu_offload else ""),
                "activation_checkpointing": args.activation_checkpointing,
            },
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "tflops_per_gpu": round(flops_tok * tps / world / 1e12, 1),
            "peak_mem_gib": round(peak, 1),
            "final_loss": round(last_loss.item(), 4) if last_loss is not None else None,
            "baseline_tokens_per_sec": base_dev * world if headline else None,
            "gemm_table": os.path.basename(gemm_table) if gemm_table else None,
            "preflight": preflight,
        }
        print(json.dumps(rec), flush=True)
    accelerator.end_training()


if __name__ == "__main__":
    main()
