"""W ranks sharing ONE MI355X over a gloo group: the sharded engines with real partial shards, on the HIP kernels.

The forced-sharded single-GPU mode runs the W>1 engine code at nranks=1, where every parameter is whole in every
shard. Only W>1 cuts parameters across shard boundaries, and that is what this script drives: FSDP partial-parameter
slices through the fused AdamW / bf16 shadow, `grad_shard_update` with 1/W, the fp8 all-gather's per-segment amax /
cast kernels on partial pieces plus the batched amax all-reduce, the clip-norm reduction across processes (over the
HIP-IPC one-shot all-reduce when `ACCELERATE_SMALL_ALLREDUCE_GLOO=1`), sharded checkpoint save -> load, and the DDP
reducer's bucket all-reduce. RCCL refuses two ranks on one device, so the group is gloo with HIP tensors (the engine
picks the gloo-compatible collective forms by backend).

Launched as `torch.distributed.run --nproc-per-node W test_gpu_ranks.py --mode M --out DIR`, or without a launcher
(W=1: the single-process reference). Rank 0 writes DIR/result_W{W}.json (per-step global loss and grad norm) and
DIR/params_W{W}.pt (full fp32 state dict); `tests/test_gpu_multirank.py` compares W=2/4 against W=1.
Reference: test_utils/scripts/test_sync.py:29-331 (sharded training equals the single-process model).
"""

from __future__ import annotations

import argparse
import json
import os

import torch


GLOBAL_BATCH = 8  # divisible by every rehearsed world size (1 / 2 / 4 / 8)
SEQ = 256


def _batches(steps, vocab):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, vocab, (GLOBAL_BATCH, SEQ), generator=g) for _ in range(steps)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", choices=["fsdp", "fsdp_fp8", "ddp", "hsdp", "tp", "tp_sp", "tp_fsdp", "tp_fsdp_sp", "hsdp_tp", "cp_allgather", "cp_alltoall", "ep", "ulysses"], required=True)
    p.add_argument("--seq", type=int, default=16384)
    p.add_argument("--heads", default="8,2", help="cp modes: query,kv heads")
    p.add_argument("--no-ref", action="store_true", help="cp modes: skip the fp32 reference (long sequences)")
    p.add_argument("--out", required=True)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--preset", default="llama-small")
    p.add_argument("--cpu", action="store_true", help="plumbing check of this script on CPU ranks (not the GPU test)")
    args = p.parse_args()

    if args.mode.startswith("cp_"):
        return run_context_parallel(args)
    if args.mode == "ep":
        return run_expert_parallel(args)
    if args.mode == "ulysses":
        return run_ulysses(args)
    from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM
    from accelerate_hpc_test_amd.parallel import small_allreduce
    from accelerate_hpc_test_amd.utils import AORecipeKwargs, InitProcessGroupKwargs, RcclKwargs

    W = int(os.environ.get("WORLD_SIZE", "1"))
    handlers = [InitProcessGroupKwargs(backend="gloo")] if W > 1 else []
    cfg = LLAMA_PRESETS[args.preset]
    lr = 1e-4
    if args.mode == "ddp":
        acc = Accelerator(mixed_precision="bf16", kwargs_handlers=handlers, cpu=args.cpu)
        torch.manual_seed(0)
        model = LlamaForCausalLM(cfg).to(acc.device)
    elif args.mode in ("tp", "tp_sp"):  # Megatron column / row parallel over W ranks, every rank on the whole batch
        from accelerate_hpc_test_amd import ParallelismConfig
        from accelerate_hpc_test_amd.utils.dataclasses import TorchTensorParallelConfig

        acc = Accelerator(mixed_precision="bf16", kwargs_handlers=handlers, cpu=args.cpu,
                          parallelism_config=ParallelismConfig(tp_size=W, tp_handler=TorchTensorParallelConfig(
                              sequence_parallel=args.mode == "tp_sp")) if W > 1 else None)
        torch.manual_seed(0)
        model = LlamaForCausalLM(cfg).to(acc.device)
    elif args.mode in ("tp_fsdp", "tp_fsdp_sp", "hsdp_tp"):
        # 2-D / 3-D meshes: tp 2 innermost, FSDP over dp_shard (x 2 HSDP replicas); the global grad norm must sum the
        # tp-sharded squares over tp and dp_shard and count the tp-replicated ones once. tp_fsdp_sp: sequence-parallel
        # TP, whose norm weights see 1/tp of the tokens and need the tp all-reduce of their gradients (no FSDP slot)
        from accelerate_hpc_test_amd import ParallelismConfig
        from accelerate_hpc_test_amd.utils.dataclasses import TorchTensorParallelConfig

        pc = None
        if W > 1:
            rep = 2 if args.mode == "hsdp_tp" else 1
            pc = ParallelismConfig(tp_size=2, dp_shard_size=W // (2 * rep), dp_replicate_size=rep,
                                   tp_handler=TorchTensorParallelConfig(sequence_parallel=args.mode == "tp_fsdp_sp"))
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
        acc = Accelerator(mixed_precision="bf16", fsdp_plugin=plugin, kwargs_handlers=handlers + [RcclKwargs()],
                          cpu=args.cpu, parallelism_config=pc)
        torch.manual_seed(0)
        model = LlamaForCausalLM(cfg).to(acc.device)
    else:
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
        if args.mode == "fsdp_fp8":
            handlers.append(AORecipeKwargs(enable_fsdp_float8_all_gather=True))
        handlers.append(RcclKwargs())
        pc = None
        if args.mode == "hsdp" and W > 1:  # 2 replicas x W/2 shards: reduce-scatter in the shard group + replica all-reduce
            from accelerate_hpc_test_amd import ParallelismConfig

            pc = ParallelismConfig(dp_replicate_size=2, dp_shard_size=W // 2)
        acc = Accelerator(mixed_precision="fp8" if args.mode == "fsdp_fp8" else "bf16", fsdp_plugin=plugin,
                          kwargs_handlers=handlers, cpu=args.cpu, parallelism_config=pc)
        with torch.device("meta"):
            model = LlamaForCausalLM(cfg)
    r = acc.process_index
    assert acc.num_processes == W and acc.device.type == ("cpu" if args.cpu else "cuda")
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=0.01)
    model, opt = acc.prepare(model, opt)
    facts = {"world": W, "mode": args.mode}
    tp_modes = ("tp", "tp_sp", "tp_fsdp", "tp_fsdp_sp", "hsdp_tp")
    def _tp_sharded(q):
        return getattr(getattr(q, "_tp_spec", None), "size", 1) > 1

    if args.mode in ("tp", "tp_sp"):
        facts["tp_sharded"] = sum(1 for q in model.parameters() if _tp_sharded(q))
    if args.mode in tp_modes[2:]:
        facts["tp_sharded"] = sum(1 for u in model.engine.units for i in u.infos if _tp_sharded(i.param))
        facts["sharded"] = bool(model.engine.sharded)
        # parameters whose gradient a tp hook all-reduces must not take an FSDP gradient slot
        facts["tp_hooked_with_slot"] = sum(1 for u in model.engine.units for i in u.infos
                                           if i.fused and getattr(i.module, "_tp_grad_allreduce_group", None) is not None)
    elif args.mode not in ("ddp", "tp", "tp_sp"):
        eng = model.engine
        facts["sharded"] = bool(eng.sharded)
        # parameters cut by a shard boundary (the case the forced one-GPU mode never has)
        facts["split_params"] = sum(1 for u in eng.units for i in u.infos if 0 < i.local_hi - i.local_lo < i.numel)
        facts["fp8_units"] = len(eng.f8_units)
        facts["replicated"] = eng.replicate_group is not None
    else:
        facts["ddp_buckets"] = len(getattr(model, "buckets", []))
    if W > 1:
        facts["ipc_allreduce"] = small_allreduce.get(None) is not None
    tp = W if args.mode in ("tp", "tp_sp") else (2 if args.mode in tp_modes and W > 1 else 1)
    bs = GLOBAL_BATCH // (W // tp)
    dp_rank = r // tp  # mesh order: dp_replicate, dp_shard outer, tp inner
    losses, norms = [], []
    for ids in _batches(args.steps, cfg.vocab_size):
        local = ids[dp_rank * bs : (dp_rank + 1) * bs].to(acc.device)
        out = model(local, labels=local)
        acc.backward(out.loss)
        norms.append(float(acc.clip_grad_norm_(model.parameters(), 1e9)))
        opt.step()
        opt.zero_grad()
        losses.append(float(acc.reduce(out.loss.detach().float(), reduction="mean")))
    if not args.cpu:
        torch.cuda.synchronize()
    if args.mode == "ddp":
        state = {k: v.detach().float().cpu() for k, v in acc.unwrap_model(model).state_dict().items()}
    else:
        state = acc.get_state_dict(model)
    if args.mode == "fsdp" and W > 1:
        # sharded checkpoint round trip: every rank writes its shard files, perturb, load, compare
        from accelerate_hpc_test_amd.utils import gather_object

        d = gather_object([os.path.join(args.out, f"ckpt_W{W}")])[0]
        acc.save_state(d)
        with torch.no_grad():
            for q in model.parameters():
                q.add_(1.0)
        acc.load_state(d)
        back = acc.get_state_dict(model)
        if r == 0:
            bad = [n for n in state if not torch.equal(state[n], back[n])]
            facts["ckpt_roundtrip_mismatch"] = bad
    if r == 0:
        os.makedirs(args.out, exist_ok=True)
        torch.save({k: v.float().cpu() for k, v in state.items()}, os.path.join(args.out, f"params_{args.mode}_W{W}.pt"))
        with open(os.path.join(args.out, f"result_{args.mode}_W{W}.json"), "w") as f:
            json.dump(dict(facts, losses=losses, norms=norms), f)
        print(json.dumps(dict(facts, losses=losses, norms=norms)), flush=True)
    acc.wait_for_everyone()
    acc.end_training()


def run_context_parallel(args):
    """Ring attention (parallel/context_parallel.py) of a `--seq`-token causal sequence cut into 2W zig-zag chunks over
    W ranks, forward + backward on the HIP flash kernels; rank 0 reassembles O / dQ / dK / dV and compares them with
    fp32 full attention. Also records each rank's peak transient HBM of the attention call."""
    import math

    import torch.distributed as dist

    from accelerate_hpc_test_amd.parallel.context_parallel import ring_attention, zigzag_shard, zigzag_unshard

    W = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    if W > 1:
        dist.init_process_group("gloo")
    r = dist.get_rank() if W > 1 else 0
    S, D = args.seq, 128
    Hq, Hkv = (int(x) for x in args.heads.split(","))
    g = torch.Generator().manual_seed(11)
    full = {n: torch.randn(1, S, h, D, generator=g).to(torch.bfloat16).cuda() for n, h in
            (("q", Hq), ("k", Hkv), ("v", Hkv), ("do", Hq))}
    local = {n: zigzag_shard(t, 1, W, r).requires_grad_(n != "do") for n, t in full.items()}
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    import time

    t0 = time.perf_counter()
    o = ring_attention(local["q"], local["k"], local["v"], None, strategy=args.mode[3:])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    fwd_peak = torch.cuda.max_memory_allocated() - base
    o.backward(local["do"])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    transient = torch.cuda.max_memory_allocated() - base
    if args.no_ref:
        stats = [None] * W
        mine = {"fwd_peak": int(fwd_peak), "peak": int(transient), "fwd_s": t1 - t0, "bwd_s": t2 - t1}
        if W > 1:
            dist.all_gather_object(stats, mine)
        else:
            stats = [mine]
        if r == 0:
            res = {"world": W, "mode": args.mode, "seq": S, "heads": [Hq, Hkv], "per_rank": stats}
            os.makedirs(args.out, exist_ok=True)
            with open(os.path.join(args.out, f"mem_{args.mode}_W{W}_S{S}.json"), "w") as f:
                json.dump(res, f)
            print(json.dumps(res), flush=True)
        if W > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    def gather(t):
        if W == 1:
            return t.detach()
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t.detach().contiguous())
        return zigzag_unshard(parts, 1)

    outs = {"o": gather(o), "dq": gather(local["q"].grad), "dk": gather(local["k"].grad), "dv": gather(local["v"].grad)}
    peaks = [None] * W
    if W > 1:
        dist.all_gather_object(peaks, int(transient))
    else:
        peaks = [int(transient)]
    if r == 0:
        scale = 1 / math.sqrt(D)
        rep = Hq // Hkv
        ref = {"o": torch.zeros(1, S, Hq, D, device="cuda"), "dq": torch.zeros(1, S, Hq, D, device="cuda"),
               "dk": torch.zeros(1, S, Hkv, D, device="cuda"), "dv": torch.zeros(1, S, Hkv, D, device="cuda")}
        mask = torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1)
        for h in range(Hq):  # fp32 reference, one head at a time (a 16k x 16k fp32 score matrix per head)
            qh = full["q"][0, :, h].float().requires_grad_()
            kh = full["k"][0, :, h // rep].float().requires_grad_()
            vh = full["v"][0, :, h // rep].float().requires_grad_()
            sc = (qh @ kh.t() * scale).masked_fill(mask, float("-inf"))
            oh = torch.softmax(sc, -1) @ vh
            oh.backward(full["do"][0, :, h].float())
            ref["o"][0, :, h] = oh.detach()
            ref["dq"][0, :, h] = qh.grad
            ref["dk"][0, :, h // rep] += kh.grad
            ref["dv"][0, :, h // rep] += vh.grad
            del sc, oh
        rel = {n: ((outs[n].float() - ref[n]).norm() / ref[n].norm()).item() for n in outs}
        res = {"world": W, "mode": args.mode, "seq": S, "rel_err": rel, "peak_transient_bytes": peaks}
        os.makedirs(args.out, exist_ok=True)
        with open(os.path.join(args.out, f"result_{args.mode}_W{W}.json"), "w") as f:
            json.dump(res, f)
        print(json.dumps(res), flush=True)
    if W > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_expert_parallel(args):
    """Expert parallelism (models/moe.py `shard_experts`): W ranks each route their own token slice through an 8-expert
    top-2 MoELayer whose experts are split W ways (variable all-to-all dispatch / combine, local grouped expert GEMMs
    on the HIP kernels); rank 0 compares the gathered output, the summed router gradient and every expert's gradient
    (x W: the EP hook averages expert grads over the group) with ONE process running the unsharded layer on all the
    tokens."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.models.moe import MoELayer

    W = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    if W > 1:
        dist.init_process_group("gloo")
    r = dist.get_rank() if W > 1 else 0
    E, H, I, T = 8, 256, 512, 512  # T tokens per rank
    torch.manual_seed(0)
    ref = MoELayer(H, I, E, 2).to("cuda", torch.bfloat16)
    with torch.no_grad():
        ref.gate.weight.normal_(0, 0.2)
        ref.experts.w_gate_up.normal_(0, 0.05)
        ref.experts.w_down.normal_(0, 0.05)
    g = torch.Generator().manual_seed(5)
    X = torch.randn(W * T, H, generator=g).to("cuda", torch.bfloat16)
    DY = torch.randn(W * T, H, generator=g).to("cuda", torch.bfloat16)
    layer = MoELayer(H, I, E, 2).to("cuda", torch.bfloat16)
    layer.load_state_dict(ref.state_dict())
    if W > 1:
        layer.shard_experts(dist.group.WORLD)
    x = X[r * T : (r + 1) * T].clone().requires_grad_(True)
    y = layer(x)
    y.backward(DY[r * T : (r + 1) * T])
    torch.cuda.synchronize()

    def gather_rows(t):
        if W == 1:
            return t.detach()
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t.detach().contiguous())
        return torch.cat(parts)

    ys, dxs = gather_rows(y), gather_rows(x.grad)
    dgate = layer.gate.weight.grad.float().clone()
    if W > 1:
        dist.all_reduce(dgate)
    # expert grads: this rank holds experts [r E / W, (r + 1) E / W), averaged 1 / W by the EP hook
    ex = {n: gather_rows(getattr(layer.experts, n).grad.float() * W) for n in ("w_gate_up", "w_down")}
    if r == 0:
        xr = X.clone().requires_grad_(True)
        yr = ref(xr)
        yr.backward(DY)

        def rel(a, b):
            return ((a.float() - b.float()).norm() / b.float().norm()).item()

        res = {"world": W, "mode": "ep", "rel_err": {
            "y": rel(ys, yr), "dx": rel(dxs, xr.grad), "dgate": rel(dgate, ref.gate.weight.grad),
            "dw_gate_up": rel(ex["w_gate_up"], ref.experts.w_gate_up.grad),
            "dw_down": rel(ex["w_down"], ref.experts.w_down.grad)}}
        os.makedirs(args.out, exist_ok=True)
        with open(os.path.join(args.out, f"result_ep_W{W}.json"), "w") as f:
            json.dump(res, f)
        print(json.dumps(res), flush=True)
    if W > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_ulysses(args):
    """Ulysses sequence parallelism (parallel/ulysses.py): W ranks hold contiguous sequence slices of q / k / v; the
    all-to-all regroups them by heads, the HIP flash kernels attend over the whole sequence, and the inverse all-to-all
    returns sequence slices. Rank 0 compares the gathered O / dQ / dK / dV with fp32 causal attention."""
    import math

    import torch.distributed as dist

    from accelerate_hpc_test_amd.parallel.ulysses import ulysses_attention

    W = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    if W > 1:
        dist.init_process_group("gloo")
    r = dist.get_rank() if W > 1 else 0
    S, Hq, Hkv, D = 4096, 16, 4, 128
    g = torch.Generator().manual_seed(13)
    full = {n: torch.randn(1, S, h, D, generator=g).to(torch.bfloat16).cuda() for n, h in
            (("q", Hq), ("k", Hkv), ("v", Hkv), ("do", Hq))}
    L = S // W
    local = {n: t[:, r * L : (r + 1) * L].clone().requires_grad_(n != "do") for n, t in full.items()}
    o = ulysses_attention(local["q"], local["k"], local["v"], dist.group.WORLD if W > 1 else None)
    o.backward(local["do"])
    torch.cuda.synchronize()

    def gather(t):
        if W == 1:
            return t.detach()
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t.detach().contiguous())
        return torch.cat(parts, 1)

    outs = {"o": gather(o), "dq": gather(local["q"].grad), "dk": gather(local["k"].grad), "dv": gather(local["v"].grad)}
    if r == 0:
        scale, rep = 1 / math.sqrt(D), Hq // Hkv
        ref = {"o": torch.zeros(1, S, Hq, D, device="cuda"), "dq": torch.zeros(1, S, Hq, D, device="cuda"),
               "dk": torch.zeros(1, S, Hkv, D, device="cuda"), "dv": torch.zeros(1, S, Hkv, D, device="cuda")}
        mask = torch.ones(S, S, device="cuda", dtype=torch.bool).triu(1)
        for h in range(Hq):  # fp32 reference, one head at a time
            qh = full["q"][0, :, h].float().requires_grad_()
            kh = full["k"][0, :, h // rep].float().requires_grad_()
            vh = full["v"][0, :, h // rep].float().requires_grad_()
            oh = torch.softmax((qh @ kh.t() * scale).masked_fill(mask, float("-inf")), -1) @ vh
            oh.backward(full["do"][0, :, h].float())
            ref["o"][0, :, h] = oh.detach()
            ref["dq"][0, :, h] = qh.grad
            ref["dk"][0, :, h // rep] += kh.grad
            ref["dv"][0, :, h // rep] += vh.grad
        rel = {n: ((outs[n].float() - ref[n]).norm() / ref[n].norm()).item() for n in outs}
        res = {"world": W, "mode": "ulysses", "seq": S, "rel_err": rel}
        os.makedirs(args.out, exist_ok=True)
        with open(os.path.join(args.out, f"result_ulysses_W{W}.json"), "w") as f:
            json.dump(res, f)
        print(json.dumps(res), flush=True)
    if W > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
