"""Multi-rank checks run under `debug_launcher` (CPU gloo fake cluster) or torchrun on GPUs.

Parity with the reference's shipped scripts (`test_utils/scripts/test_ops.py`, `test_sync.py`,
`test_distributed_data_loop.py`): collectives against closed-form expectations, and the key oracle for the gradient
sync rebuild — the data-parallel model's gradients / parameters must equal a single-process model trained on the
gathered global batch.
"""

from __future__ import annotations

import copy
import os
import tempfile

import torch
import torch.nn.functional as F

from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin, PartialState
from accelerate_hpc_test_amd.test_utils.training import TinyMLP
from accelerate_hpc_test_amd.utils import (
    DistributedOperationException,
    broadcast,
    gather,
    gather_object,
    pad_across_processes,
    reduce,
    set_seed,
)


def check_ops():
    state = PartialState(cpu=True)
    W, r = state.num_processes, state.process_index
    t = torch.arange(3.0) + 3 * r
    assert gather(t).tolist() == list(range(3 * W))
    nested = {"a": torch.tensor([r, r]), "b": [torch.ones(2, 2) * r]}
    g = gather(nested)
    assert g["a"].tolist() == [i for i in range(W) for _ in range(2)]
    assert g["b"][0].shape == (2 * W, 2)
    assert gather_object([r]) == list(range(W))
    b = broadcast(torch.full((4,), float(r)), from_process=0)
    assert b.tolist() == [0.0] * 4
    s = reduce(torch.tensor([float(r + 1)]), reduction="sum")
    assert s.item() == W * (W + 1) / 2
    m = reduce({"x": torch.tensor([float(r)]), "y": torch.tensor([2.0 * r])}, reduction="mean")
    assert abs(m["x"].item() - (W - 1) / 2) < 1e-6 and abs(m["y"].item() - (W - 1)) < 1e-6
    p = pad_across_processes(torch.ones(r + 1, 2), dim=0)
    assert p.shape == (W, 2)
    with state.split_between_processes(list(range(2 * W + 1))) as part:
        assert len(part) in (2, 3)
    # debug-mode shape checker
    state.debug = True
    try:
        gather(torch.ones(r + 1))
        raised = False
    except DistributedOperationException:
        raised = True
    state.debug = False
    assert raised


def _global_batches(n_steps, bs_per_rank, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(bs_per_rank * W, 4, generator=g), torch.randn(bs_per_rank * W, generator=g)) for _ in range(n_steps)]


def check_ddp_matches_single(grad_accum: int = 1):
    acc = Accelerator(cpu=True, gradient_accumulation_steps=grad_accum)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    bs = 4
    batches = _global_batches(4 * grad_accum, bs, W)
    for step, (x, y) in enumerate(batches):
        with acc.accumulate(model):
            xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
            loss = F.mse_loss(model(xl), yl)
            acc.backward(loss)
            opt.step()
            opt.zero_grad()
        # baseline on the global batch
        bl = F.mse_loss(base(x), y) / grad_accum
        bl.backward()
        if (step + 1) % grad_accum == 0:
            base_opt.step()
            base_opt.zero_grad()
    inner = acc.unwrap_model(model)
    for (n, p), (_, q) in zip(inner.named_parameters(), base.named_parameters()):
        assert torch.allclose(p, q, atol=1e-5), (n, (p - q).abs().max())


def check_fsdp_matches_single(reshard: bool = True, state_dict_type: str = "SHARDED_STATE_DICT", force_sharded: bool = False,
                              cpu_offload: bool = False):
    if force_sharded:  # world size 1 running the multi-rank code (RcclKwargs.fsdp_force_sharded)
        os.environ["ACCELERATE_FSDP_FORCE_SHARDED"] = "1"
    plugin = FullyShardedDataParallelPlugin(
        fsdp_version=2,
        auto_wrap_policy="transformer_based_wrap",
        transformer_cls_names_to_wrap=["Block"],
        reshard_after_forward=reshard,
        state_dict_type=state_dict_type,
        cpu_offload=cpu_offload,
    )
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2, weight_decay=0.01)
    model, opt = acc.prepare(model, opt)
    assert model.engine.sharded == (W > 1 or force_sharded)
    assert model.engine.offload == cpu_offload
    if cpu_offload:  # host optimizer step: the native OpenMP AdamW (csrc/runtime/cpu_adam.cpp)
        from accelerate_hpc_test_amd.ops.multi_tensor import CpuFusedAdamStep

        assert isinstance(opt._maybe_fused(), CpuFusedAdamStep)
    bs = 4
    for x, y in _global_batches(3, bs, W):
        xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
        loss = F.mse_loss(model(xl), yl)
        acc.backward(loss)
        n1 = acc.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
        opt.zero_grad()
        bl = F.mse_loss(base(x), y)
        bl.backward()
        n2 = torch.nn.utils.clip_grad_norm_(base.parameters(), 0.5)
        assert torch.allclose(n1.reshape(()), n2, rtol=1e-4), (n1, n2)
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (n, (full[n] - q).abs().max())

    # checkpoint round trip: perturb, reload, compare
    d = tempfile.mkdtemp() if r == 0 else None
    d = gather_object([d])[0]
    acc.save_state(d)
    if state_dict_type == "SHARDED_STATE_DICT" and r == 0:
        # `accelerate merge-weights`: the per-rank shard files merge into the full state dict (reference
        # tests/test_merge_weights.py strategy)
        from safetensors.torch import load_file

        from accelerate_hpc_test_amd.utils import merge_fsdp_weights

        merged = load_file(merge_fsdp_weights(os.path.join(d, "pytorch_model_fsdp_0"), os.path.join(d, "merged")))
        assert set(merged) == set(full), (sorted(merged), sorted(full))
        for n in full:
            assert torch.equal(merged[n], full[n]), n
    acc.wait_for_everyone()
    for p in model.parameters():
        p.data.add_(1.0)
    acc.load_state(d)
    full2 = acc.get_state_dict(model)
    for n in full:
        assert torch.allclose(full[n], full2[n]), n
    # training continues identically after reload (optimizer state restored)
    x, y = _global_batches(1, bs, W, seed=5)[0]
    xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
    acc.backward(F.mse_loss(model(xl), yl))
    opt.step()
    opt.zero_grad()
    F.mse_loss(base(x), y).backward()
    base_opt.step()
    full3 = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full3[n], q, atol=1e-5), (n, (full3[n] - q).abs().max())


def check_fsdp_checkpoint_io(phase: str, ckpt_dir: str, state_dict_type: str = "SHARDED_STATE_DICT"):
    """Per-rank-bounded checkpoint IO (reference: DCP planned reads / rank-0 broadcast,
    /root/reference/src/accelerate/utils/fsdp_utils.py:161-230,281-335,467-554).

    phase "save": tiny Llama, 2 AdamW steps, `save_state`; rank 0 also writes the full model + optimizer state as the
    oracle. phase "load" (any world size): fresh model, `load_state`, then every rank's bytes of tensor data read from
    the checkpoint must be <= 1/W of it plus boundary pieces (SHARDED), or zero off rank 0 (FULL); the full model and
    optimizer state must equal the oracle."""
    from accelerate_hpc_test_amd.models.llama import LlamaForCausalLM
    from accelerate_hpc_test_amd.utils import fsdp_utils

    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"], state_dict_type=state_dict_type)
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(0 if phase == "save" else 1)
    cfg = _tiny_llama_cfg()
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    model, opt = acc.prepare(model, opt)
    eng = model.engine
    if phase == "save":
        g = torch.Generator().manual_seed(3)
        for _ in range(2):
            ids = torch.randint(0, cfg.vocab_size, (2 * W, 16), generator=g)[2 * r : 2 * r + 2]
            acc.backward(model(ids, labels=ids).loss)
            opt.step()
            opt.zero_grad()
        acc.save_state(ckpt_dir)
        full = acc.get_state_dict(model)
        optim = fsdp_utils._optim_full_state(eng, opt)
        if r == 0:
            torch.save({"model": full, "optim": optim["state"]}, os.path.join(ckpt_dir, "oracle.pt"))
        acc.wait_for_everyone()
        return
    fsdp_utils.IO_STATS["bytes_read"] = 0
    acc.load_state(ckpt_dir)
    mine = fsdp_utils.IO_STATS["bytes_read"]
    reads = gather_object([mine])
    oracle = torch.load(os.path.join(ckpt_dir, "oracle.pt"), weights_only=True)
    total = sum(t.numel() * 4 for t in oracle["model"].values())
    total += sum(t.numel() * 4 for st in oracle["optim"].values() for t in st.values())
    if r == 0:
        print(f"[checkpoint io] {state_dict_type} W={W}: bytes read per rank {reads}, checkpoint tensors {total}", flush=True)
    if state_dict_type == "SHARDED_STATE_DICT":
        # a rank's slice of every unit (padding included) + the pieces of parameters cut by a saved-rank boundary
        bound = total / W * 1.05 + 64 * 1024
        assert max(reads) <= bound, (reads, total, W)
        assert sum(reads) >= total * 0.99, (reads, total)  # and together the ranks read everything once
    else:
        assert all(b == 0 for b in reads[1:]) and reads[0] >= total * 0.99, (reads, total)
    full = acc.get_state_dict(model)
    for n, t in oracle["model"].items():
        assert torch.equal(full[n].float(), t.float()), n
    optim = fsdp_utils._optim_full_state(eng, opt)
    if r == 0:
        for fqn, st in oracle["optim"].items():
            for k, t in st.items():
                assert torch.equal(optim["state"][fqn][k], t), (fqn, k)
    acc.wait_for_everyone()


def check_fsdp_optimizer_overlap(grad_accum: int = 1):
    """`RcclKwargs(fsdp_optimizer_overlap=True)`: the per-unit updates applied during backward must give exactly the
    single-process AdamW trajectory (with a LR schedule and gradient accumulation), and clipping must refuse."""
    from accelerate_hpc_test_amd.utils import RcclKwargs

    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap", transformer_cls_names_to_wrap=["Block"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin, gradient_accumulation_steps=grad_accum,
                      kwargs_handlers=[RcclKwargs(fsdp_optimizer_overlap=True)])
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 1.0 / (1 + s))
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2, weight_decay=0.01)
    base_sched = torch.optim.lr_scheduler.LambdaLR(base_opt, lambda s: 1.0 / (1 + s))
    model, opt, sched = acc.prepare(model, opt, sched)
    assert getattr(opt, "_overlap_engine", None) is not None
    bs = 4
    batches = _global_batches(3 * grad_accum, bs, W)
    for i, (x, y) in enumerate(batches):
        xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
        with acc.accumulate(model):
            acc.backward(F.mse_loss(model(xl), yl))
            if acc.sync_gradients:
                try:
                    acc.clip_grad_norm_(model.parameters(), 1.0)
                    raise AssertionError("clip_grad_norm_ must refuse after overlapped updates")
                except RuntimeError:
                    pass
            opt.step()
            sched.step()
            opt.zero_grad()
        (F.mse_loss(base(x), y) / grad_accum).backward()
        if (i + 1) % grad_accum == 0:
            base_opt.step()
            for _ in range(W):  # AcceleratedScheduler steps num_processes times (split_batches=False)
                base_sched.step()
            base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (n, (full[n] - q).abs().max())


def check_fsdp_no_sync_accumulation():
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap", transformer_cls_names_to_wrap=["Block"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin, gradient_accumulation_steps=2)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    bs = 2
    for step, (x, y) in enumerate(_global_batches(4, bs, W)):
        with acc.accumulate(model):
            xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
            acc.backward(F.mse_loss(model(xl), yl))
            opt.step()
            opt.zero_grad()
        (F.mse_loss(base(x), y) / 2).backward()
        if step % 2 == 1:
            base_opt.step()
            base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (n, (full[n] - q).abs().max())


def check_dataloader_sharding():
    acc = Accelerator(cpu=True)
    W, r = acc.num_processes, acc.process_index
    dl = torch.utils.data.DataLoader(list(range(10)), batch_size=2)
    dl = acc.prepare(dl)
    seen = []
    for b in dl:
        seen.append(acc.gather_for_metrics(b))
    allv = torch.cat(seen).tolist()
    assert sorted(allv) == list(range(10)), allv


def _tiny_llama_cfg():
    from accelerate_hpc_test_amd.models.llama import LlamaConfig

    return LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)


def check_tp_matches_single(sequence_parallel: bool = False, dp_shard: int = 1, steps: int = 2, dp_replicate: int = 1,
                            norm_type: float = 2.0, max_norm: float = 1e9, adamw: bool = False):
    """TP (optionally sequence-parallel, optionally x FSDP over dp_shard, optionally x HSDP replicas) must train
    exactly like one process on the global batch: same loss, same global gradient norm, same full weights after
    `steps` steps. The norm is the reference's DTensor-aware `clip_grad_norm_` over the whole mesh
    (/root/reference/src/accelerate/accelerator.py:2943-2953): tp-sharded squares summed over tp and dp_shard,
    tp-replicated ones counted once, HSDP replicas not at all. `max_norm` below the norm exercises the clip scale
    itself (every rank must scale its shards by the same global factor); `adamw` trains with AdamW instead of SGD."""
    from accelerate_hpc_test_amd import ParallelismConfig
    from accelerate_hpc_test_amd.models.llama import LlamaForCausalLM
    from accelerate_hpc_test_amd.utils.dataclasses import TorchTensorParallelConfig

    W = int(os.environ["WORLD_SIZE"])
    dp = dp_shard * dp_replicate
    tp = W // dp
    pc = ParallelismConfig(tp_size=tp, dp_shard_size=dp_shard, dp_replicate_size=dp_replicate,
                           tp_handler=TorchTensorParallelConfig(sequence_parallel=sequence_parallel))
    plugin = None
    if dp > 1:
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(cpu=True, parallelism_config=pc, fsdp_plugin=plugin)
    set_seed(0)
    cfg = _tiny_llama_cfg()
    base = LlamaForCausalLM(cfg)
    base.init_weights()
    model = copy.deepcopy(base)
    if adamw:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
        base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2, weight_decay=0.01)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=0.5, momentum=0.9)
        base_opt = torch.optim.SGD(base.parameters(), lr=0.5, momentum=0.9)
    model, opt = acc.prepare(model, opt)
    dp_rank = acc.process_index // tp  # mesh order: dp_replicate, dp_shard outer, tp inner
    g = torch.Generator().manual_seed(3)
    bs, S = 2, 16
    for _ in range(steps):
        ids = torch.randint(0, cfg.vocab_size, (bs * dp, S), generator=g)
        local = ids[dp_rank * bs : (dp_rank + 1) * bs]
        out = model(local, labels=local)
        acc.backward(out.loss)
        # the global gradient norm: tp-sharded squares summed over the group, replicated ones counted once
        gn = acc.clip_grad_norm_(model.parameters(), max_norm, norm_type=norm_type)
        opt.step()
        opt.zero_grad()
        ref = base(ids, labels=ids)
        ref.loss.backward()
        gn_ref = torch.nn.utils.clip_grad_norm_(base.parameters(), max_norm, norm_type=norm_type)
        assert torch.allclose(gn.float(), gn_ref.float(), rtol=1e-4), (gn, gn_ref)
        if max_norm < 1e9:
            assert gn_ref.item() > max_norm, "the clip must be active for this check"
        base_opt.step()
        base_opt.zero_grad()
        lg = acc.reduce(out.loss.detach().reshape(1), reduction="mean")
        assert torch.allclose(lg, ref.loss.detach().reshape(1), atol=2e-5), (lg, ref.loss)
    full = acc.get_state_dict(model)
    # AdamW normalises each element's step, so float rounding in a near-zero gradient can move a weight by a sizeable
    # fraction of lr (1e-2): 2 % of one step; SGD stays at the rounding level
    atol = 2e-4 if adamw else 2e-5
    for n, q in base.state_dict().items():
        assert full[n].shape == q.shape, (n, full[n].shape, q.shape)
        assert torch.allclose(full[n].float(), q.float(), atol=atol), (n, (full[n] - q).abs().max())


def check_tp_fsdp_sharded_merge():
    """dp_shard 2 x tp 2, SHARDED_STATE_DICT: every (dp, tp) rank writes its TP-local FSDP shard; `merge_fsdp_weights`
    must rebuild the FULL weights (TP slices concatenated along each parameter's shard dim, fused q/k/v and gate/up
    segments re-interleaved) equal to `get_state_dict`; `load_state` round-trips exactly in the same layout, and a
    checkpoint whose tp size differs from the loading job's is refused."""
    from safetensors.torch import load_file

    from accelerate_hpc_test_amd import ParallelismConfig
    from accelerate_hpc_test_amd.models.llama import LlamaForCausalLM
    from accelerate_hpc_test_amd.utils import fsdp_utils, merge_fsdp_weights

    pc = ParallelismConfig(tp_size=2, dp_shard_size=2)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"],
                                            state_dict_type="SHARDED_STATE_DICT")
    acc = Accelerator(cpu=True, parallelism_config=pc, fsdp_plugin=plugin)
    r = acc.process_index
    set_seed(0)
    cfg = _tiny_llama_cfg()
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    model, opt = acc.prepare(model, opt)
    ids = torch.randint(0, cfg.vocab_size, (2, 16), generator=torch.Generator().manual_seed(1))
    acc.backward(model(ids, labels=ids).loss)
    opt.step()
    opt.zero_grad()
    full = acc.get_state_dict(model)
    d = gather_object([tempfile.mkdtemp() if r == 0 else None])[0]
    acc.save_state(d)
    if r == 0:
        merged = load_file(merge_fsdp_weights(os.path.join(d, "pytorch_model_fsdp_0"), os.path.join(d, "merged")))
        assert set(merged) == set(full), set(merged) ^ set(full)
        for k, v in full.items():
            assert merged[k].shape == v.shape, (k, merged[k].shape, v.shape)
            assert torch.equal(merged[k].float(), v.float()), (k, (merged[k].float() - v.float()).abs().max())
    acc.wait_for_everyone()
    with torch.no_grad():
        for q in model.parameters():
            q.add_(1.0)
    acc.load_state(d)
    back = acc.get_state_dict(model)
    for k, v in full.items():
        assert torch.equal(back[k], v), k
    metas = fsdp_utils._saved_metas(os.path.join(d, "pytorch_model_fsdp_0"))
    fake = [(path, dict(m, tp_size=4)) for path, m in metas]
    try:
        fsdp_utils._check_tp_layout(fake, model.engine, "probe")
        raise AssertionError("a tp-size mismatch must be refused")
    except ValueError as exc:
        assert "tensor-parallel size" in str(exc)


def check_dtensor_clip_norm_2d_mesh(norm_type: float = 2.0):
    """DTensor gradients on a 2 x 2 mesh sharded on dim 0 only, dim 1 only, both dims, or replicated: the global norm
    of `Accelerator._clip_grad_norm_dtensor` equals the norm of the full gradients (each partial is reduced over its
    own sharded dims only), and the clip scales every local shard by the same factor."""
    import torch.distributed as dist
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import Replicate, Shard, distribute_tensor

    acc = Accelerator(cpu=True)
    assert acc.num_processes == 4
    mesh = init_device_mesh("cpu", (2, 2))
    g = torch.Generator().manual_seed(0)
    fulls = [torch.randn(8, 6, generator=g) for _ in range(4)]
    grads = [torch.randn(8, 6, generator=g) for _ in range(4)]
    layouts = [[Shard(0), Replicate()], [Replicate(), Shard(1)], [Shard(0), Shard(1)], [Replicate(), Replicate()]]
    params = []
    for w, gr, pl in zip(fulls, grads, layouts):
        p = torch.nn.Parameter(distribute_tensor(w.clone(), mesh, pl))
        p.grad = distribute_tensor(gr.clone(), mesh, pl)
        params.append(p)
    want = torch.stack([x.abs().max() for x in grads]).max() if norm_type == float("inf") else \
        torch.sqrt(sum((x ** 2).sum() for x in grads))
    total = Accelerator._clip_grad_norm_dtensor(params, 1e9, norm_type)
    assert torch.allclose(total, want, rtol=1e-5), (total, want)
    clip = float(want) / 4
    total = Accelerator._clip_grad_norm_dtensor(params, clip, norm_type)
    for p, gr in zip(params, grads):
        got = p.grad.full_tensor()
        assert torch.allclose(got, gr * (clip / (float(want) + 1e-6)), rtol=1e-4, atol=1e-6)
    dist.barrier()


def check_tp_dtensor_model(steps: int = 3, norm_type: float = 2.0):
    """A model already sharded as DTensors (torch `parallelize_module`, the layout transformers' `tp_plan="auto"`
    produces in the reference's nd-parallel flow) goes through `prepare` unchanged; AdamW runs torch's DTensor-aware
    step (not the fused HIP kernel) and `clip_grad_norm_` reduces the sharded placements over the mesh: losses, norms
    and full weights == one process."""
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor import DTensor
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel
    from torch.distributed.tensor.parallel import parallelize_module as torch_parallelize

    from accelerate_hpc_test_amd import ParallelismConfig

    W = int(os.environ["WORLD_SIZE"])
    acc = Accelerator(cpu=True, parallelism_config=ParallelismConfig(tp_size=W))
    torch.manual_seed(0)
    base = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    model = copy.deepcopy(base)
    mesh = init_device_mesh("cpu", (W,))
    torch_parallelize(model, mesh, {"0": ColwiseParallel(), "2": RowwiseParallel()})
    assert any(isinstance(p, DTensor) for p in model.parameters())
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2)
    model, opt = acc.prepare(model, opt)
    assert opt._maybe_fused() is False, "DTensor parameters must not take the fused HIP AdamW"
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        x, y = torch.randn(6, 8, generator=g), torch.randn(6, 4, generator=g)
        loss = F.mse_loss(model(x), y)
        acc.backward(loss)
        gn = acc.clip_grad_norm_(model.parameters(), 0.05, norm_type=norm_type)
        opt.step()
        opt.zero_grad()
        ref = F.mse_loss(base(x), y)
        ref.backward()
        gn_ref = torch.nn.utils.clip_grad_norm_(base.parameters(), 0.05, norm_type=norm_type)
        base_opt.step()
        base_opt.zero_grad()
        assert torch.allclose(loss.detach(), ref.detach(), atol=1e-6), (loss, ref)
        assert torch.allclose(gn.float(), gn_ref.float(), rtol=1e-5), (gn, gn_ref)
    for (n, p), q in zip(model.named_parameters(), base.parameters()):
        full = p.full_tensor() if isinstance(p, DTensor) else p
        assert torch.allclose(full.detach(), q.detach(), atol=1e-6), (n, (full - q).abs().max())


def check_ring_attention(strategy: str = "allgather"):
    """Zig-zag ring attention (fwd + bwd) on a cp group == full causal attention on one process."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.ops.fused import attention_reference
    from accelerate_hpc_test_amd.parallel.context_parallel import ring_attention, zigzag_shard

    PartialState(cpu=True)
    W, r = dist.get_world_size(), dist.get_rank()
    g = torch.Generator().manual_seed(0)
    B, S, Hq, Hkv, D = 2, 8 * W, 4, 2, 16
    q = torch.randn(B, S, Hq, D, generator=g)
    k = torch.randn(B, S, Hkv, D, generator=g)
    v = torch.randn(B, S, Hkv, D, generator=g)
    w = torch.randn(B, S, Hq, D, generator=g)
    # reference
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    (attention_reference(qr, kr, vr, causal=True) * w).sum().backward()
    # ring
    ql, kl, vl = (zigzag_shard(t, 1, W, r).requires_grad_() for t in (q, k, v))
    o = ring_attention(ql, kl, vl, None, strategy=strategy)
    ref_o = zigzag_shard(attention_reference(q, k, v, causal=True), 1, W, r)
    assert torch.allclose(o, ref_o, atol=1e-5), (o - ref_o).abs().max()
    (o * zigzag_shard(w, 1, W, r)).sum().backward()
    for name, got, ref in (("dq", ql.grad, qr.grad), ("dk", kl.grad, kr.grad), ("dv", vl.grad, vr.grad)):
        exp = zigzag_shard(ref, 1, W, r)
        assert torch.allclose(got, exp, atol=1e-4), (name, (got - exp).abs().max())


def check_cp_llama_matches_single(strategy: str = "allgather", steps: int = 2, dp_shard: int = 1):
    """Llama trained under `maybe_context_parallel` (cp = world / dp_shard, FSDP over dp_shard x cp) == one process
    on the global batch: same loss, same global gradient norm, same weights."""
    from accelerate_hpc_test_amd import ParallelismConfig
    from accelerate_hpc_test_amd.models.llama import LlamaForCausalLM
    from accelerate_hpc_test_amd.utils.dataclasses import TorchContextParallelConfig

    W = int(os.environ["WORLD_SIZE"])
    cp = W // dp_shard
    pc = ParallelismConfig(dp_shard_size=dp_shard, cp_size=cp,
                           cp_handler=TorchContextParallelConfig(cp_comm_strategy=strategy))
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(cpu=True, parallelism_config=pc, fsdp_plugin=plugin)
    set_seed(0)
    base = LlamaForCausalLM(_tiny_llama_cfg())
    base.init_weights()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.5, momentum=0.9)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.5, momentum=0.9)
    model, opt = acc.prepare(model, opt)
    dp_rank = acc.process_index // cp  # mesh order: dp_shard outer, cp inner
    g = torch.Generator().manual_seed(7)
    B, S = 2, 8 * cp
    for _ in range(steps):
        ids = torch.randint(0, 128, (B * dp_shard, S), generator=g)
        shift = torch.randint(0, 128, (B * dp_shard, S), generator=g)  # every position valid: equal token counts
        ref = base(ids, shift_labels=shift)
        ref.loss.backward()
        gn_ref = torch.nn.utils.clip_grad_norm_(base.parameters(), 1e9)
        base_opt.step()
        base_opt.zero_grad()
        rows = slice(dp_rank * B, (dp_rank + 1) * B)
        ids_l, shift_l = ids[rows].clone(), shift[rows].clone()
        with acc.maybe_context_parallel(buffers=[ids_l, shift_l], buffer_seq_dims=[1, 1], no_restore_buffers={ids_l, shift_l}):
            assert ids_l.shape[1] == S // cp
            out = model(ids_l, shift_labels=shift_l)
            acc.backward(out.loss)
        gn = acc.clip_grad_norm_(model.parameters(), 1e9)
        assert torch.allclose(gn.float(), gn_ref.float(), rtol=1e-4), (gn, gn_ref)
        opt.step()
        opt.zero_grad()
        lg = acc.reduce(out.loss.detach().reshape(1), reduction="mean")
        assert torch.allclose(lg, ref.loss.detach().reshape(1), atol=2e-5), (lg, ref.loss)
    full = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        assert torch.allclose(full[n].float(), q.float(), atol=5e-5), (n, (full[n] - q).abs().max())


def check_ulysses_attention():
    """All-to-all (Ulysses) attention on contiguous sequence slices == full causal attention (fwd + bwd)."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.ops.fused import attention_reference
    from accelerate_hpc_test_amd.parallel.ulysses import ulysses_attention

    PartialState(cpu=True)
    W, r = dist.get_world_size(), dist.get_rank()
    g = torch.Generator().manual_seed(0)
    B, S, Hq, Hkv, D = 2, 4 * W, 4, 2, 8
    q, k, v, w = (torch.randn(B, S, h, D, generator=g) for h in (Hq, Hkv, Hkv, Hq))
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = attention_reference(qr, kr, vr, causal=True)
    (ref * w).sum().backward()
    L = S // W
    sl = slice(r * L, (r + 1) * L)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    o = ulysses_attention(ql, kl, vl, None)
    assert torch.allclose(o, ref[:, sl].detach(), atol=1e-5), (o - ref[:, sl]).abs().max()
    (o * w[:, sl]).sum().backward()
    for name, got, exp in (("dq", ql.grad, qr.grad), ("dk", kl.grad, kr.grad), ("dv", vl.grad, vr.grad)):
        assert torch.allclose(got, exp[:, sl], atol=1e-4), (name, (got - exp[:, sl]).abs().max())


def check_ulysses_llama_matches_single(steps: int = 2):
    """Llama with Ulysses SP (sp = world) fed through the prepared data loader == one process on full batches."""
    from accelerate_hpc_test_amd import ParallelismConfig
    from accelerate_hpc_test_amd.models.llama import LlamaForCausalLM

    W = int(os.environ["WORLD_SIZE"])
    pc = ParallelismConfig(sp_size=W)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(cpu=True, parallelism_config=pc, fsdp_plugin=plugin)
    set_seed(0)
    base = LlamaForCausalLM(_tiny_llama_cfg())
    base.init_weights()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.5, momentum=0.9)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.5, momentum=0.9)
    g = torch.Generator().manual_seed(11)
    B, S = 2, 8 * W
    data = [{"input_ids": torch.randint(0, 128, (S,), generator=g), "shift_labels": torch.randint(0, 128, (S,), generator=g)}
            for _ in range(steps * B)]
    dl = torch.utils.data.DataLoader(data, batch_size=B)
    model, opt, dl = acc.prepare(model, opt, dl)
    for i, batch in enumerate(dl):
        assert batch["input_ids"].shape == (B, S // W) and "position_ids" in batch
        out = model(batch["input_ids"], shift_labels=batch["shift_labels"], position_ids=batch["position_ids"])
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
        full = data[i * B : (i + 1) * B]
        ids = torch.stack([d["input_ids"] for d in full])
        sl = torch.stack([d["shift_labels"] for d in full])
        ref = base(ids, shift_labels=sl)
        ref.loss.backward()
        base_opt.step()
        base_opt.zero_grad()
        lg = acc.reduce(out.loss.detach().reshape(1), reduction="mean")
        assert torch.allclose(lg, ref.loss.detach().reshape(1), atol=2e-5), (lg, ref.loss)
    sd = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        assert torch.allclose(sd[n].float(), q.float(), atol=5e-5), (n, (sd[n] - q).abs().max())


def check_local_sgd(k: int = 2, steps: int = 4, chunk_bytes: int = 256 << 20):
    """LocalSGD == every rank trains alone for k steps, then parameters are averaged (simulated locally). With a
    small `chunk_bytes` the averaging must stay in packed buffers of at most that size (or one parameter alone):
    no whole-model transient (the reference averages per parameter, local_sgd.py:98-106)."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.local_sgd import LocalSGD

    sizes = []
    real_all_reduce = dist.all_reduce

    def recording_all_reduce(t, *a, **kw):
        sizes.append(t.numel() * t.element_size())
        return real_all_reduce(t, *a, **kw)

    acc = Accelerator(cpu=True)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    sims = [copy.deepcopy(base) for _ in range(W)]
    sim_opts = [torch.optim.SGD(m.parameters(), lr=0.1) for m in sims]
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    bs = 4
    batches = _global_batches(steps, bs, W)
    dist.all_reduce = recording_all_reduce
    try:
        _local_sgd_loop(acc, model, opt, sims, sim_opts, batches, W, r, bs, k, chunk_bytes)
    finally:
        dist.all_reduce = real_all_reduce
    largest = max(p.numel() * p.element_size() for p in sims[0].parameters())
    assert sizes and max(sizes) <= max(chunk_bytes, largest), (sizes, chunk_bytes, largest)
    inner = acc.unwrap_model(model)
    for (n, p), q in zip(inner.named_parameters(), sims[0].parameters()):
        assert torch.allclose(p, q, atol=1e-6), (n, (p - q).abs().max())


def check_local_sgd_integer_params():
    """Non-float parameters (e.g. an integer step counter registered as a frozen Parameter) are averaged too, in
    their own buckets: integers as sum then floor division (the reference's per-parameter `reduce(param, "mean")`
    cannot divide an integer tensor in place), bool flags by majority vote (ties True), identical on every rank."""
    from accelerate_hpc_test_amd.local_sgd import LocalSGD

    acc = Accelerator(cpu=True)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    model = TinyMLP()
    model.counter = torch.nn.Parameter(torch.zeros(2, dtype=torch.int64), requires_grad=False)
    model.small = torch.nn.Parameter(torch.zeros(3, dtype=torch.int8), requires_grad=False)
    model.flags = torch.nn.Parameter(torch.zeros(4, dtype=torch.bool), requires_grad=False)
    opt = torch.optim.SGD([p for p in model.parameters() if p.is_floating_point()], lr=0.1)
    model, opt = acc.prepare(model, opt)
    inner = acc.unwrap_model(model)
    inner.counter.data.copy_(torch.tensor([10 * (r + 1), 3 * r]))  # diverged after DDP's broadcast
    inner.small.data.copy_(torch.tensor([r, -r, 7], dtype=torch.int8))
    # flag 0 set on every rank, flag 1 on rank 0 only, flag 2 on ranks < W / 2 (a tie at even W), flag 3 on none
    inner.flags.data.copy_(torch.tensor([True, r == 0, r < W / 2, False]))
    with LocalSGD(acc, model, local_sgd_steps=1) as local_sgd:
        local_sgd.step()
    want = torch.tensor([sum(10 * (j + 1) for j in range(W)) // W, sum(3 * j for j in range(W)) // W])
    assert inner.counter.dtype == torch.int64 and torch.equal(inner.counter.data, want), (inner.counter, want)
    want8 = torch.tensor([sum(range(W)) // W, -sum(range(W)) // W, 7], dtype=torch.int8)
    assert inner.small.dtype == torch.int8 and torch.equal(inner.small.data, want8), (inner.small, want8)
    votes = [W, 1, sum(1 for j in range(W) if j < W / 2), 0]
    want_b = torch.tensor([2 * v >= W for v in votes])
    assert inner.flags.dtype == torch.bool and torch.equal(inner.flags.data, want_b), (inner.flags, want_b)


def _local_sgd_loop(acc, model, opt, sims, sim_opts, batches, W, r, bs, k, chunk_bytes):
    from accelerate_hpc_test_amd.local_sgd import LocalSGD

    with LocalSGD(acc, model, local_sgd_steps=k, chunk_bytes=chunk_bytes) as local_sgd:
        for step, (x, y) in enumerate(batches):
            acc.backward(F.mse_loss(model(x[r * bs : (r + 1) * bs]), y[r * bs : (r + 1) * bs]))
            opt.step()
            opt.zero_grad()
            local_sgd.step()
            for j, (m, o) in enumerate(zip(sims, sim_opts)):
                F.mse_loss(m(x[j * bs : (j + 1) * bs]), y[j * bs : (j + 1) * bs]).backward()
                o.step()
                o.zero_grad()
            if (step + 1) % k == 0:
                with torch.no_grad():
                    for ps in zip(*[m.parameters() for m in sims]):
                        avg = sum(p.detach() for p in ps) / W
                        for p in ps:
                            p.copy_(avg)


def check_pipeline_inference(gather_output: bool = True, split="auto"):
    """prepare_pippy: the staged model's logits (micro-batched) == the full model's logits on one process."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.inference import prepare_pippy
    from accelerate_hpc_test_amd.models.llama import LlamaConfig, LlamaForCausalLM

    state = PartialState(cpu=True)
    W, r = state.num_processes, state.process_index
    cfg = LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2 * W,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
    set_seed(0)
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    ids = torch.randint(0, 128, (4, 16), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = model(ids).logits
    splits = split if split == "auto" else [f"layers.{2 * i}" for i in range(1, W)]
    model = prepare_pippy(model, split_points=splits, gather_output=gather_output, num_chunks=2)
    assert len(model.hf_split_points) == W - 1
    # this rank only materialised its own stage
    n_real = sum(p.numel() for p in model.parameters() if p.device.type != "meta")
    n_all = sum(p.numel() for p in model.parameters())
    assert n_real < n_all
    out = model(ids)
    if gather_output or r == W - 1:
        assert torch.allclose(out.logits, ref, atol=1e-5), (out.logits - ref).abs().max()
    else:
        assert out is None
    dist.barrier()


def check_expert_parallel_mixtral(steps: int = 2, skew: float = 0.0):
    """Mixtral with experts sharded over the FSDP group (ep = world) == one process on the global batch, incl. the
    clipped grad norm and a sharded checkpoint round trip. `skew` > 0 biases every router towards expert 0 and away
    from the last expert (uneven loads: one rank receives most rows, an expert may receive none)."""
    from accelerate_hpc_test_amd import ParallelismConfig
    from accelerate_hpc_test_amd.models.mixtral import MixtralConfig, MixtralForCausalLM

    W = int(os.environ["WORLD_SIZE"])
    r = int(os.environ["RANK"])
    pc = ParallelismConfig(dp_shard_size=W, ep_size=W)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["MixtralDecoderLayer"], state_dict_type="SHARDED_STATE_DICT")
    acc = Accelerator(cpu=True, parallelism_config=pc, fsdp_plugin=plugin)
    cfg = MixtralConfig(vocab_size=128, hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, head_dim=8, num_local_experts=2 * W, num_experts_per_tok=2, max_position_embeddings=64)
    set_seed(0)
    base = MixtralForCausalLM(cfg)
    base.init_weights()
    if skew:  # selection bias: expert 0 favoured, the last expert almost never chosen
        E = cfg.num_local_experts
        for layer in base.layers:
            layer.block_sparse_moe.router_bias = torch.linspace(skew, -skew, E) * (torch.arange(E) % 2 == 0) + \
                torch.tensor([skew] + [0.0] * (E - 2) + [-skew])
    model = copy.deepcopy(base)
    captured = {}
    base.layers[0].block_sparse_moe.gate.register_forward_hook(lambda m, i, o: captured.__setitem__("logits", o.detach()))
    opt = torch.optim.SGD(model.parameters(), lr=0.2, momentum=0.9)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.2, momentum=0.9)
    model, opt = acc.prepare(model, opt)
    g = torch.Generator().manual_seed(5)
    bs, S = 2, 8
    for _ in range(steps):
        ids = torch.randint(0, 128, (bs * W, S), generator=g)
        local = ids[r * bs : (r + 1) * bs]
        out = model(local, labels=local)
        acc.backward(out.loss)
        n1 = acc.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
        opt.zero_grad()
        ref = base(ids, labels=ids)
        if skew:  # the routing really is uneven: per-expert loads of the global batch differ a lot
            sel = torch.softmax(captured["logits"].float(), -1) + base.layers[0].block_sparse_moe.router_bias
            loads = torch.bincount(torch.topk(sel, 2, -1)[1].reshape(-1), minlength=cfg.num_local_experts)
            assert loads.max() >= 4 * max(int(loads.min()), 1), loads
            captured["loads"] = loads
        ref.loss.backward()
        n2 = torch.nn.utils.clip_grad_norm_(base.parameters(), 0.5)
        base_opt.step()
        base_opt.zero_grad()
        assert torch.allclose(n1.reshape(()), n2, rtol=1e-4), (n1, n2)
    full = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        assert full[n].shape == q.shape, (n, full[n].shape, q.shape)
        assert torch.allclose(full[n].float(), q.float(), atol=5e-5), (n, (full[n] - q).abs().max())
    # sharded checkpoint round trip (expert shards are saved per rank and restored)
    d = tempfile.mkdtemp() if r == 0 else None
    d = gather_object([d])[0]
    acc.save_state(d)
    with torch.no_grad():
        for p in model.parameters():  # shard params + expert shards
            p.add_(1.0)
    acc.load_state(d)
    full2 = acc.get_state_dict(model)
    for n in full:
        assert torch.allclose(full[n], full2[n]), n


def check_fsdp_mixtral_expert_slots(steps: int = 2):
    """Mixtral under FSDP without expert parallelism: the stacked expert weights are FSDP-sharded and their grouped
    weight-gradient GEMMs write straight into the engine's gradient slots (models/moe.py) == one process."""
    from accelerate_hpc_test_amd.models.mixtral import MixtralConfig, MixtralForCausalLM

    W = int(os.environ["WORLD_SIZE"])
    r = int(os.environ["RANK"])
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["MixtralDecoderLayer"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    cfg = MixtralConfig(vocab_size=128, hidden_size=32, intermediate_size=48, num_hidden_layers=2, num_attention_heads=4,
                        num_key_value_heads=2, head_dim=8, num_local_experts=4, num_experts_per_tok=2, max_position_embeddings=64)
    set_seed(0)
    base = MixtralForCausalLM(cfg)
    base.init_weights()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.2, momentum=0.9)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.2, momentum=0.9)
    model, opt = acc.prepare(model, opt)
    eng = model.engine
    fused = sorted(i.fqn for u in eng.units for i in u.infos if i.fused and "experts" in i.fqn)
    assert fused == sorted(f"layers.{l}.block_sparse_moe.experts.{n}" for l in range(2) for n in ("w_gate_up", "w_down")), fused
    g = torch.Generator().manual_seed(5)
    bs, S = 2, 8
    for _ in range(steps):
        ids = torch.randint(0, 128, (bs * W, S), generator=g)
        local = ids[r * bs : (r + 1) * bs]
        out = model(local, labels=local)
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
        ref = base(ids, labels=ids)
        ref.loss.backward()
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        assert torch.allclose(full[n].float(), q.float(), atol=5e-5), (n, (full[n] - q).abs().max())


def check_dispatch_batches_matches_upstream():
    """`prepare_data_loader(dispatch_batches=True)` (rank 0 reads, broadcasts, every rank slices) yields exactly the
    batches of the upstream accelerate installed in the image, for map-style and iterable datasets, split / whole
    batches, drop_last on/off and sizes that do not divide evenly; also the remainder bookkeeping."""
    try:
        import accelerate.data_loader as up_dl
        from accelerate.state import PartialState as UpState
    except ImportError:
        return
    from torch.utils.data import DataLoader, IterableDataset

    from accelerate_hpc_test_amd.data_loader import prepare_data_loader
    from accelerate_hpc_test_amd.state import PartialState

    PartialState(cpu=True)
    UpState._reset_state()  # a parent process may have left a single-process upstream state behind (forked Borg dict)
    UpState(cpu=True)
    assert UpState().num_processes == PartialState().num_processes

    class It(IterableDataset):
        def __init__(self, n):
            self.n = n

        def __iter__(self):
            return iter(torch.arange(self.n, dtype=torch.float32))

    compared = 0
    for iterable in (False, True):
        for n in (7, 16, 19):
            for bs in (2, 4):
                for split in (False, True):
                    for drop_last in (False, True):
                        ds = It(n) if iterable else torch.arange(n, dtype=torch.float32)
                        res = []
                        for prep in (prepare_data_loader, up_dl.prepare_data_loader):
                            dl = prep(DataLoader(ds, batch_size=bs, drop_last=drop_last), device=torch.device("cpu"),
                                      put_on_device=True, dispatch_batches=True, split_batches=split)
                            try:
                                got = [b.tolist() for b in dl]
                            except TypeError as exc:  # upstream broadcasts None for an empty final step here
                                if prep is prepare_data_loader:
                                    raise
                                res.append(("upstream-error", str(exc)[:40]))
                                continue
                            res.append((got, dl.remainder))
                        if res[1][0] == "upstream-error":
                            continue  # no oracle for this configuration (ours must merely run, checked above)
                        assert res[0][0] == res[1][0], (iterable, n, bs, split, drop_last, res)
                        assert res[0][1] == res[1][1], ("remainder", iterable, n, bs, split, drop_last, res[0][1], res[1][1])
                        compared += 1
    assert compared >= 40, compared  # of 48 configurations


def check_join_uneven_inputs():
    """Rank r gets 2 + r batches; with `join_uneven_inputs` the short rank shadows the long rank's all-reduces.
    Oracle: grads of each step = sum over active ranks / W (divide_by_initial_world_size)."""
    acc = Accelerator(cpu=True)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    bs = 4
    n_steps = [2 + j for j in range(W)]
    data = {j: _global_batches(n_steps[j], bs, 1, seed=10 + j) for j in range(W)}
    with acc.join_uneven_inputs([model]):
        for x, y in data[r]:
            acc.backward(F.mse_loss(model(x), y))
            opt.step()
            opt.zero_grad()
    # oracle
    for step in range(max(n_steps)):
        active = [j for j in range(W) if step < n_steps[j]]
        for j in active:
            x, y = data[j][step]
            (F.mse_loss(base(x), y) / W).backward()
        base_opt.step()
        base_opt.zero_grad()
    inner = acc.unwrap_model(model)
    for (n, p), q in zip(inner.named_parameters(), base.parameters()):
        assert torch.allclose(p, q, atol=1e-5), (n, (p - q).abs().max())


class _TwoExperts(torch.nn.Module):
    """Each rank routes through a different same-shaped expert: with find_unused_parameters the ranks leave different
    parameters unused, so their buckets become ready in different orders."""

    def __init__(self):
        super().__init__()
        self.inp = torch.nn.Linear(4, 8)
        self.experts = torch.nn.ModuleList([torch.nn.Linear(8, 8) for _ in range(3)])
        self.out = torch.nn.Linear(8, 1)

    def forward(self, x, expert: int):
        return self.out(torch.relu(self.experts[expert](torch.relu(self.inp(x))))).squeeze(-1)


def check_ddp_unused_params_differ_by_rank():
    """Advisor finding: buckets must be all-reduced in the same order on every rank. Tiny buckets (one parameter
    each) and rank-dependent unused experts; the result must equal the single-process average of the per-rank grads."""
    from accelerate_hpc_test_amd.utils import DistributedDataParallelKwargs

    acc = Accelerator(cpu=True, kwargs_handlers=[DistributedDataParallelKwargs(find_unused_parameters=True, bucket_cap_mb=1e-5)])
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = _TwoExperts()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    assert len(acc.unwrap_model(model).__class__.__name__) and len(model.buckets) == len(list(base.parameters()))
    bs = 4
    for step, (x, y) in enumerate(_global_batches(3, bs, W)):
        e = (r + step) % 3
        loss = F.mse_loss(model(x[r * bs : (r + 1) * bs], e), y[r * bs : (r + 1) * bs])
        acc.backward(loss)
        opt.step()
        opt.zero_grad()
        for q in range(W):  # oracle: mean over ranks of each rank's loss on its own expert
            bl = F.mse_loss(base(x[q * bs : (q + 1) * bs], (q + step) % 3), y[q * bs : (q + 1) * bs]) / W
            bl.backward()
        base_opt.step()
        base_opt.zero_grad()
    for (n, p), (_, q) in zip(acc.unwrap_model(model).named_parameters(), base.named_parameters()):
        assert torch.allclose(p, q, atol=1e-6), (n, (p - q).abs().max())


def check_fsdp_cpu_ram_efficient_loading():
    """cpu_ram_efficient_loading: rank 0 holds the pretrained weights, every other rank builds the model on the meta
    device; after prepare every rank's shards hold rank 0's values and training matches the single-process run."""
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["Block"], cpu_ram_efficient_loading=True)
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    with torch.no_grad():  # "pretrained": values no init_fn would produce
        for i, p in enumerate(base.parameters()):
            p.copy_(torch.linspace(-1, 1, p.numel()).view_as(p) * (i + 1) * 0.1)
    if r == 0:
        model = copy.deepcopy(base)
    else:
        with torch.device("meta"):
            model = TinyMLP()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2)
    model, opt = acc.prepare(model, opt)
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.equal(full[n], q.detach()), n
    bs = 4
    for x, y in _global_batches(2, bs, W):
        acc.backward(F.mse_loss(model(x[r * bs : (r + 1) * bs]), y[r * bs : (r + 1) * bs]))
        opt.step()
        opt.zero_grad()
        F.mse_loss(base(x), y).backward()
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (n, (full[n] - q).abs().max())


def check_broadcast_from_rank0_loading():
    """load_checkpoint_in_model(broadcast_from_rank0=True): only rank 0 reads the (sharded safetensors) checkpoint;
    every rank ends with its weights — a plain model gets full tensors, an FSDP-engine model its shards."""
    import json as _json

    from safetensors.torch import save_file

    from accelerate_hpc_test_amd.utils.checkpoint_io import load_checkpoint_in_model

    acc = Accelerator(cpu=True)
    r = acc.process_index
    torch.manual_seed(123)
    src = TinyMLP()
    d = tempfile.mkdtemp() if r == 0 else None
    d = gather_object([d])[0]
    if r == 0:
        sd = {k: v.contiguous() for k, v in src.state_dict().items()}
        keys = sorted(sd)
        wm = {}
        for i in range(2):
            part = {k: sd[k] for k in keys[i::2]}
            save_file(part, os.path.join(d, f"m-{i}.safetensors"), metadata={"format": "pt"})
            wm.update({k: f"m-{i}.safetensors" for k in part})
        _json.dump({"weight_map": wm}, open(os.path.join(d, "model.safetensors.index.json"), "w"))
    acc.wait_for_everyone()
    ck = d if r == 0 else "/nonexistent-on-other-ranks"
    torch.manual_seed(r + 7)
    plain = TinyMLP()
    load_checkpoint_in_model(plain, ck, broadcast_from_rank0=True)
    for k, v in src.state_dict().items():
        assert torch.equal(plain.state_dict()[k], v), (r, k)
    # FSDP engine: the broadcast lands in each rank's shard
    from accelerate_hpc_test_amd.state import AcceleratorState

    AcceleratorState._reset_state(True)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap", transformer_cls_names_to_wrap=["Block"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    torch.manual_seed(r + 11)
    model = acc.prepare(TinyMLP())
    load_checkpoint_in_model(model, ck, broadcast_from_rank0=True)
    full = acc.get_state_dict(model)
    for k, v in src.state_dict().items():
        assert torch.equal(full[k], v), (r, k)


def check_fsdp_full_load_missing_keys():
    """FULL_STATE_DICT rank-0 broadcast load (`FSDPEngine.load_full_state_dict_broadcast`) with a key missing from the
    checkpoint: strict -> KeyError on EVERY rank before anything is copied (the model is untouched); non-strict -> the
    missing parameter keeps its current values on every rank (no zero placeholder), the others are loaded."""
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["Block"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    r = acc.process_index
    torch.manual_seed(5)
    model = acc.prepare(TinyMLP())
    eng = model.engine
    before = acc.get_state_dict(model)
    drop = sorted(before)[0]
    sd = None
    if r == 0:
        sd = {k: v + 1.0 for k, v in before.items() if k != drop}
    try:
        eng.load_full_state_dict_broadcast(sd)
        raise AssertionError("strict load with a missing key must raise")
    except KeyError as exc:
        assert drop in str(exc), exc
    after = acc.get_state_dict(model)
    for k, v in before.items():
        assert torch.equal(after[k], v), (r, k)
    missing = eng.load_full_state_dict_broadcast(sd, strict=False)
    assert missing == [drop], missing
    after = acc.get_state_dict(model)
    for k, v in before.items():
        want = v if k == drop else v + 1.0
        assert torch.allclose(after[k], want), (r, k, (after[k] - want).abs().max())


class _F8Block(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.norm = torch.nn.LayerNorm(128)
        self.fc1 = torch.nn.Linear(128, 256)
        self.fc2 = torch.nn.Linear(256, 128)

    def forward(self, x):
        return x + self.fc2(torch.relu(self.fc1(self.norm(x))))


class _F8Net(torch.nn.Module):
    """128-wide blocks so every inner linear takes the fp8 GEMM path (M % 128, N % 128, K % 64)."""

    def __init__(self):
        super().__init__()
        self.inp = torch.nn.Linear(128, 128)
        self.blocks = torch.nn.ModuleList([_F8Block() for _ in range(2)])
        self.out = torch.nn.Linear(128, 1)

    def forward(self, x):
        x = self.inp(x)
        for b in self.blocks:
            x = b(x)
        return self.out(x).squeeze(-1)


def check_fsdp_fp8_all_gather(force_sharded: bool = False):
    """AORecipeKwargs(enable_fsdp_float8_all_gather=True): the fp8 GEMM weights travel as e4m3 shards quantised with
    the all-reduced global amax. That is the same quantisation as casting the gathered bf16 weight, so losses and
    weights must equal the bf16-all-gather run exactly."""
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState
    from accelerate_hpc_test_amd.utils import AORecipeKwargs

    if force_sharded:
        os.environ["ACCELERATE_FSDP_FORCE_SHARDED"] = "1"
    results = {}
    for ag in (False, True):
        AcceleratorState._reset_state(True)
        GradientState._reset_state()
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["_F8Block"])
        acc = Accelerator(cpu=True, mixed_precision="fp8", fsdp_plugin=plugin,
                          kwargs_handlers=[AORecipeKwargs(enable_fsdp_float8_all_gather=ag)])
        W, r = acc.num_processes, acc.process_index
        torch.manual_seed(0)
        model = _F8Net()
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        model, opt = acc.prepare(model, opt)
        eng = model.engine
        assert bool(eng.f8_units) == ag and eng.fp8_all_gather == ag
        if ag:
            f8_names = sorted(i.fqn for u in eng.f8_units for i in u.f8_infos)
            assert f8_names == sorted(f"blocks.{b}.{n}.weight" for b in range(2) for n in ("fc1", "fc2")), f8_names
        losses = []
        g = torch.Generator().manual_seed(1)
        for _ in range(3):
            x = torch.randn(128 * W, 128, generator=g)
            y = torch.randn(128 * W, generator=g)
            loss = F.mse_loss(model(x[r * 128 : (r + 1) * 128]).float(), y[r * 128 : (r + 1) * 128])
            acc.backward(loss)
            opt.step()
            opt.zero_grad()
            losses.append(loss.item())
        results[ag] = (losses, acc.get_state_dict(model))
    if W <= 2:
        # two-rank sums are order-free, so the two layouts must agree bit for bit
        assert results[False][0] == results[True][0], (results[False][0], results[True][0])
        for n, t in results[False][1].items():
            assert torch.equal(t, results[True][1][n]), n
    else:
        # W >= 3: the fp8 region changes the flat layout, so an element's ring reduce-scatter sums its W terms in a
        # different order in the two runs (fp32 rounding differences only). The first step's forward uses the
        # initial weights, so the gathered fp8 weights themselves must still match exactly; later steps see the
        # rounding through the next per-tensor fp8 scale (the toy run climbs steeply at lr 1e-2, amplifying it)
        assert results[False][0][0] == results[True][0][0], (results[False][0], results[True][0])
        for a, b in zip(results[False][0], results[True][0]):
            assert abs(a - b) <= 1e-2 * abs(a), (results[False][0], results[True][0])
        for n, t in results[False][1].items():
            d = (t.float() - results[True][1][n].float()).abs()
            # Adam moves a near-zero-gradient element by up to lr per step whatever the rounding, so bound the
            # worst element by 3 steps x lr and the average by a small fraction of the weights' size
            assert float(d.max()) <= 3e-2 and float(d.mean()) <= 2e-2 * float(t.float().abs().mean()) + 1e-5, (n, float(d.max()), float(d.mean()), float(t.float().abs().mean()))


def check_ddp_powersgd():
    """PowerSGD hook: with start_powerSGD_iter=0 training still converges and ranks stay in sync."""
    from accelerate_hpc_test_amd.utils import DDPCommunicationHookType, DistributedDataParallelKwargs

    kw = DistributedDataParallelKwargs(comm_hook=DDPCommunicationHookType.POWER_SGD,
                                       comm_state_option={"start_powerSGD_iter": 0, "matrix_approximation_rank": 2, "min_compression_rate": 0.0})
    acc = Accelerator(cpu=True, kwargs_handlers=[kw])
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    model = TinyMLP()
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    model, opt = acc.prepare(model, opt)
    losses = []
    for x, y in _global_batches(30, 8, W, seed=3):
        loss = F.mse_loss(model(x[r * 8 : (r + 1) * 8]), y[r * 8 : (r + 1) * 8])
        acc.backward(loss)
        opt.step()
        opt.zero_grad()
        losses.append(acc.reduce(loss.detach().reshape(1), "mean").item())
    assert sum(losses[-5:]) < sum(losses[:5]), losses
    flat = torch.cat([p.detach().reshape(-1) for p in acc.unwrap_model(model).parameters()])
    g = gather(flat.unsqueeze(0))
    assert torch.allclose(g[0], g[-1], atol=1e-6)


def _grads_equal(a, b, **kw):
    return all(torch.allclose(p.grad, q.grad, **kw) for p, q in zip(a.parameters(), b.parameters()) if p.requires_grad)


def check_grad_sync(mode: str = "no_sync", sync_each_batch: bool = False):
    """The reference's `test_sync.py` oracle on our DDP reducer: after each backward, the data-parallel model's local
    grads equal a single-process model's grads on the gathered global batch exactly when a sync was due.

    modes: `no_sync` (odd iterations sync), `accumulate` (GradientAccumulationPlugin(num_steps=2, sync_each_batch)),
    `trigger` (three no_sync forwards, backwards with the last one under `trigger_sync_in_backward`)."""
    from accelerate_hpc_test_amd.utils import GradientAccumulationPlugin

    plugin = GradientAccumulationPlugin(num_steps=2, sync_each_batch=sync_each_batch) if mode == "accumulate" else None
    acc = Accelerator(cpu=True, gradient_accumulation_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(42)
    base = TinyMLP()
    model = acc.prepare(copy.deepcopy(base))
    bs = 4
    batches = _global_batches(4, bs, W, seed=1)
    ga = acc.gradient_accumulation_steps

    def base_step(x, y):
        (F.mse_loss(base(x), y) / ga).backward()

    def local(x, y):
        return x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]

    if mode == "trigger":
        losses = []
        for x, y in batches[:3]:
            base_step(x, y)
            with acc.no_sync(model):
                xl, yl = local(x, y)
                losses.append(F.mse_loss(model(xl), yl))
        for i, loss in enumerate(losses):
            if i < len(losses) - 1:
                acc.backward(loss)
                assert not _grads_equal(base, acc.unwrap_model(model), atol=1e-6), f"synced early at backward {i}"
            else:
                with acc.trigger_sync_in_backward(model):
                    acc.backward(loss)
                assert _grads_equal(base, acc.unwrap_model(model), atol=1e-6), "not synced after triggered backward"
        return
    for it, (x, y) in enumerate(batches):
        base_step(x, y)
        xl, yl = local(x, y)
        if mode == "no_sync":
            synced = it % 2 == 1
            ctx = acc.no_sync(model) if not synced else __import__("contextlib").nullcontext()
            with ctx:
                acc.backward(F.mse_loss(model(xl), yl))
        else:
            synced = (it + 1) % 2 == 0 or sync_each_batch
            with acc.accumulate(model):
                acc.backward(F.mse_loss(model(xl), yl))
        same = _grads_equal(base, acc.unwrap_model(model), atol=1e-6)
        if mode == "accumulate" and sync_each_batch:
            # every batch synced, but the reference grads accumulate over 2 steps exactly like ours
            assert same, f"iteration {it}: grads not in sync"
        else:
            assert same == synced, f"iteration {it}: in sync={same}, expected {synced}"
        if mode == "no_sync" and synced or mode == "accumulate" and (it + 1) % 2 == 0:
            base.zero_grad()
            acc.unwrap_model(model).zero_grad()
            for p in acc.unwrap_model(model).parameters():
                p.grad = None


def check_collective_sequence(mismatch: bool = False):
    """Debug-mode collective-order check: identical sequences pass; an extra collective on one rank is named."""
    from accelerate_hpc_test_amd.utils.fault_tolerance import CollectiveLog, check_collective_sequence as check

    state = PartialState(cpu=True)
    CollectiveLog.get().reset()
    reduce(torch.ones(3), reduction="sum")
    gather(torch.ones(2))
    if mismatch and state.process_index == 1:
        CollectiveLog.get().record("all_reduce", state.num_processes, torch.float32, 7)  # a collective rank 0 never issued
    try:
        check()
        raised = False
    except DistributedOperationException as e:
        raised = True
        assert "rank 1" in str(e)
    assert raised == mismatch


def main():
    check_ops()
    check_dataloader_sharding()
    check_ddp_matches_single()


if __name__ == "__main__":
    main()


def check_ddp_forced_single_rank():
    """RcclKwargs(ddp_force=True) at world size 1: the model goes through the DDP reducer (buckets, hooks, a one-rank
    all-reduce) and trains exactly like the unwrapped model."""
    import torch.nn as nn

    from accelerate_hpc_test_amd import Accelerator
    from accelerate_hpc_test_amd.parallel.ddp import DistributedDataParallel
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState
    from accelerate_hpc_test_amd.utils import RcclKwargs

    assert torch.distributed.is_initialized() and torch.distributed.get_world_size() == 1
    res = {}
    for force in (False, True):
        AcceleratorState._reset_state(True)
        GradientState._reset_state()
        acc = Accelerator(cpu=True, kwargs_handlers=[RcclKwargs(ddp_force=force)])
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 1))
        opt = torch.optim.AdamW(m.parameters(), lr=1e-2)
        m, opt = acc.prepare(m, opt)
        assert isinstance(m, DistributedDataParallel) == force, type(m)
        g = torch.Generator().manual_seed(1)
        losses = []
        for _ in range(3):
            x, y = torch.randn(8, 16, generator=g), torch.randn(8, 1, generator=g)
            loss = ((m(x) - y) ** 2).mean()
            acc.backward(loss)
            opt.step()
            opt.zero_grad()
            losses.append(loss.item())
        res[force] = (losses, {k: v.clone() for k, v in acc.unwrap_model(m).state_dict().items()})
    assert res[False][0] == res[True][0], (res[False][0], res[True][0])
    for k, v in res[False][1].items():
        assert torch.equal(v, res[True][1][k]), k


class _SkipBlock(torch.nn.Module):
    def __init__(self, d=16):
        super().__init__()
        self.fc1 = torch.nn.Linear(d, d)
        self.side = torch.nn.Linear(d, d)  # used only on even steps

    def forward(self, h, use_side: bool):
        h = h + self.fc1(h)
        return h + self.side(h) if use_side else h


class _SkipNet(torch.nn.Module):
    def __init__(self, d=16):
        super().__init__()
        self.inp = torch.nn.Linear(4, d)
        self.blocks = torch.nn.ModuleList([_SkipBlock(d) for _ in range(2)])
        self.out = torch.nn.Linear(d, 1)

    def forward(self, x, use_side: bool = True):
        h = self.inp(x)
        for b in self.blocks:
            h = b(h, use_side)
        return self.out(h).squeeze(-1)


def check_fsdp_skipped_fused_weight():
    """A Linear skipped on alternate steps: its fused weight-gradient slot is not written in those backwards and must
    not replay the previous step's gradient (SGD without momentum: a zero gradient == no update == torch skipping a
    param whose grad is None). Against the single-process model on the global batch."""
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["_SkipBlock"])
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    torch.manual_seed(0)
    base = _SkipNet()
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    assert any(i.fused for u in model.engine.units for i in u.infos if i.fqn.endswith("side.weight"))
    bs = 4
    for step, (x, y) in enumerate(_global_batches(4, bs, W)):
        use = step % 2 == 0
        xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
        acc.backward(F.mse_loss(model(xl, use), yl))
        opt.step()
        opt.zero_grad()
        F.mse_loss(base(x, use), y).backward()
        for p in base.parameters():  # torch leaves an unused param's grad None; SGD skips it
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (n, (full[n] - q).abs().max())


def check_fsdp_fp8_all_gather_ragged_batch():
    """fp8 all-gather with a per-rank batch the fp8 GEMM cannot tile (M % 128 != 0): the Fp8Linear falls back to a
    linear on the dequantised e4m3 weight, and the weight gradient must still reach its FSDP slot. The update of every
    fp8-gathered weight must follow the bf16-all-gather run (same fallback on the unquantised weight)."""
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState
    from accelerate_hpc_test_amd.utils import AORecipeKwargs

    results = {}
    for ag in (False, True):
        AcceleratorState._reset_state(True)
        GradientState._reset_state()
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["_F8Block"])
        acc = Accelerator(cpu=True, mixed_precision="fp8", fsdp_plugin=plugin,
                          kwargs_handlers=[AORecipeKwargs(enable_fsdp_float8_all_gather=ag)])
        W, r = acc.num_processes, acc.process_index
        torch.manual_seed(0)
        model = _F8Net()
        init = {n: p.detach().clone() for n, p in model.named_parameters()}
        opt = torch.optim.SGD(model.parameters(), lr=1e-2)
        model, opt = acc.prepare(model, opt)
        assert bool(model.engine.f8_units) == ag
        g = torch.Generator().manual_seed(1)
        m = 96  # not a multiple of 128
        for _ in range(2):
            x = torch.randn(m * W, 128, generator=g)
            y = torch.randn(m * W, generator=g)
            acc.backward(F.mse_loss(model(x[r * m : (r + 1) * m]).float(), y[r * m : (r + 1) * m]))
            opt.step()
            opt.zero_grad()
        full = acc.get_state_dict(model)
        results[ag] = {n: full[n].float() - init[n].float() for n in init}
    for b in range(2):
        for n in ("fc1", "fc2"):
            k = f"blocks.{b}.{n}.weight"
            d0, d1 = results[False][k].flatten(), results[True][k].flatten()
            assert d1.abs().max() > 0, f"{k}: no update with the fp8 all-gather"
            cos = float(torch.dot(d0, d1) / (d0.norm() * d1.norm()))
            assert cos > 0.98 and abs(float(d1.norm() / d0.norm()) - 1) < 0.05, (k, cos, float(d1.norm() / d0.norm()))


def check_fsdp1_strategy(strategy: str, backward_prefetch=None, forward_prefetch: bool = False, local_world: int = 2):
    """FSDP1 `sharding_strategy` semantics on the native engine (reference accelerator.py:1909-1925; mapping of
    commands/to_fsdp2.py:50-66): NO_SHARD = unsharded units + a replicate all-reduce over the world; HYBRID_SHARD(_ZERO2)
    = shard within LOCAL_WORLD_SIZE ranks, replicate across; SHARD_GRAD_OP keeps params gathered after forward. Shard
    sizes, groups and prefetch mode are asserted, then training (with clipping) and a sharded checkpoint round trip are
    compared with the single-process model."""
    os.environ["LOCAL_WORLD_SIZE"] = str(local_world)
    plugin = FullyShardedDataParallelPlugin(
        fsdp_version=1, sharding_strategy=strategy, auto_wrap_policy="transformer_based_wrap",
        transformer_cls_names_to_wrap=["Block"], backward_prefetch=backward_prefetch, forward_prefetch=forward_prefetch,
        state_dict_type="SHARDED_STATE_DICT")
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP()
    model = copy.deepcopy(base)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-2, weight_decay=0.01)
    model, opt = acc.prepare(model, opt)
    eng = model.engine
    shard, reps = {"NO_SHARD": (1, W), "FULL_SHARD": (W, 1), "SHARD_GRAD_OP": (W, 1)}.get(strategy, (local_world, W // local_world))
    assert (eng.world_size, eng.replicate_size) == (shard, reps), (strategy, eng.world_size, eng.replicate_size)
    assert eng.sharded == (shard > 1)
    assert eng.reshard_after_forward == (strategy in ("FULL_SHARD", "HYBRID_SHARD") and shard > 1)
    for u in eng.units:
        assert u.shard_numel * shard == u.padded, (u.shard_numel, u.padded)
    assert eng.bwd_prefetch == backward_prefetch and eng.fwd_prefetch_depth == (eng.prefetch_depth if forward_prefetch else 0)
    bs = 4
    for x, y in _global_batches(3, bs, W):
        xl, yl = x[r * bs : (r + 1) * bs], y[r * bs : (r + 1) * bs]
        acc.backward(F.mse_loss(model(xl), yl))
        n1 = acc.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
        opt.zero_grad()
        F.mse_loss(base(x), y).backward()
        n2 = torch.nn.utils.clip_grad_norm_(base.parameters(), 0.5)
        assert torch.allclose(n1.reshape(()), n2, rtol=1e-4), (n1, n2)
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.named_parameters():
        assert torch.allclose(full[n], q, atol=1e-5), (strategy, n, (full[n] - q).abs().max())
    d = tempfile.mkdtemp() if r == 0 else None
    d = gather_object([d])[0]
    acc.save_state(d)
    if r == 0:  # replicas do not duplicate shard files
        files = sorted(f for f in os.listdir(os.path.join(d, "pytorch_model_fsdp_0")) if f.startswith("shard_"))
        assert files == [f"shard_{i}.safetensors" for i in range(shard)], files
    acc.wait_for_everyone()
    with torch.no_grad():
        for p in model.parameters():
            p.add_(1.0)
    acc.load_state(d)
    back = acc.get_state_dict(model)
    for n in full:
        assert torch.allclose(full[n], back[n]), n


def check_fsdp_split_root_units(steps: int = 2):
    """Large root leaves (token embedding, lm_head) become FSDP units of their own (ACCELERATE_FSDP_SPLIT_ROOT; the
    threshold is lowered so llama-tiny's qualify): the unit layout has them, training equals one process, and the
    sharded checkpoint round-trips."""
    os.environ["ACCELERATE_FSDP_SPLIT_ROOT_MIN_PARAMS"] = "1000"
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM

    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"],
                                            state_dict_type="SHARDED_STATE_DICT")
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    torch.manual_seed(0)
    base = LlamaForCausalLM(LLAMA_PRESETS["llama-tiny"])
    base.init_weights()
    model = copy.deepcopy(base)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    base_opt = torch.optim.AdamW(base.parameters(), lr=1e-3)
    model, opt = acc.prepare(model, opt)
    eng = model.engine
    unit_names = [sorted(i.fqn for i in u.infos) for u in eng.units]
    assert ["embed_tokens.weight"] in unit_names and ["lm_head.weight"] in unit_names, unit_names
    assert [i.fqn for i in eng.root.infos] == ["norm.weight"], [i.fqn for i in eng.root.infos]
    g = torch.Generator().manual_seed(3)
    bs = 2
    for _ in range(steps):
        ids = torch.randint(0, 512, (bs * W, 64), generator=g)
        local = ids[r * bs : (r + 1) * bs]
        out = model(local, labels=local)
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
        base(ids, labels=ids).loss.backward()
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        # Adam turns fp32 summation-order noise in a near-zero gradient (rows of tokens seen on one rank) into up to
        # +-lr per step; everything else agrees to fp32 rounding
        d = (full[n].float() - q.float()).abs()
        assert d.max() <= 2 * 1e-3 * steps and d.mean() <= 1e-5, (n, d.max(), d.mean())
    d = tempfile.mkdtemp() if r == 0 else None
    d = gather_object([d])[0]
    acc.save_state(d)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(1.0)
    acc.load_state(d)
    back = acc.get_state_dict(model)
    for n in full:
        assert torch.equal(full[n], back[n]), n


def check_fsdp_bert_accuracy_lower_bound(version: int, strategy: str = "FULL_SHARD", wrap: str = "transformer_based_wrap",
                                        steps: int = 60, bound: float = 0.82):
    """The reference's FSDP `test_performance` (tests/fsdp/test_fsdp.py:484-566: BERT trained under FSDP1 / FSDP2 x
    sharding strategy x wrap policy must reach accuracy >= 0.82) without the Hub: a tiny random-init transformers
    BertForSequenceClassification learns a synthetic pair task (label 1 iff the marker token 4 occurs in the sequence,
    the evaluation set held out) on 2 gloo ranks; evaluation goes through gather_for_metrics."""
    import transformers as tf

    plugin = FullyShardedDataParallelPlugin(fsdp_version=version, sharding_strategy=strategy if version == 1 else None,
                                            reshard_after_forward=(strategy == "FULL_SHARD") if version == 2 else None,
                                            auto_wrap_policy=wrap, transformer_cls_names_to_wrap=["BertLayer"],
                                            min_num_params=2000 if wrap == "size_based_wrap" else None)
    acc = Accelerator(cpu=True, fsdp_plugin=plugin)
    W, r = acc.num_processes, acc.process_index
    set_seed(0)
    cfg = tf.BertConfig(vocab_size=64, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                        max_position_embeddings=64, num_labels=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    model = tf.BertForSequenceClassification(cfg)

    def make(n, seed):
        g = torch.Generator().manual_seed(seed)
        ids = torch.randint(5, 64, (n, 24), generator=g)
        ids[:, 0] = 2  # [CLS]-like
        y = (torch.rand(n, generator=g) < 0.5).long()
        pos = torch.randint(1, 24, (n,), generator=g)
        ids[y == 1, pos[y == 1]] = 4
        return ids, y

    xtr, ytr = make(steps * 16 * W, 1)
    xev, yev = make(256, 2)
    opt = torch.optim.AdamW(model.parameters(), lr=2e-3)
    model, opt = acc.prepare(model, opt)
    model.train()
    bs = 16
    for i in range(steps):
        lo = (i * W + r) * bs
        out = model(input_ids=xtr[lo : lo + bs], labels=ytr[lo : lo + bs])
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
    model.eval()
    correct = total = 0
    per = len(xev) // W
    with torch.no_grad():
        for lo in range(r * per, (r + 1) * per, 32):
            hi = min(lo + 32, (r + 1) * per)
            pred = model(input_ids=xev[lo:hi]).logits.argmax(-1)
            pred, ref = acc.gather_for_metrics((pred, yev[lo:hi]))
            correct += int((pred == ref).sum())
            total += len(ref)
    accuracy = correct / total
    assert total == len(xev), total
    assert accuracy >= bound, (version, strategy, wrap, accuracy)
    return accuracy


def _tiny_hf_model(kind: str):
    """Tiny random-init transformers models of the families the reference's pippy examples run
    (`/root/reference/examples/inference/pippy/{llama,bert,gpt2,t5}.py`), and example inputs."""
    import transformers as tf

    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, 128, (4, 16), generator=g)
    if kind == "llama":
        cfg = tf.LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=4,
                             num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64)
        return tf.LlamaForCausalLM(cfg), {"input_ids": ids}
    if kind == "bert":
        cfg = tf.BertConfig(vocab_size=128, hidden_size=64, num_hidden_layers=4, num_attention_heads=4,
                            intermediate_size=96, max_position_embeddings=64)
        return tf.BertForMaskedLM(cfg), {"input_ids": ids, "attention_mask": torch.ones_like(ids)}
    if kind == "gpt2":
        cfg = tf.GPT2Config(vocab_size=128, n_embd=64, n_layer=4, n_head=4, n_positions=64, num_labels=3, pad_token_id=0)
        return tf.GPT2ForSequenceClassification(cfg), {"input_ids": ids}
    if kind == "t5":
        cfg = tf.T5Config(vocab_size=128, d_model=64, d_ff=96, d_kv=16, num_layers=2, num_decoder_layers=2, num_heads=4,
                          decoder_start_token_id=0, pad_token_id=0)
        dec = torch.randint(1, 128, (4, 8), generator=g)
        return tf.T5ForConditionalGeneration(cfg), {"input_ids": ids, "decoder_input_ids": dec}
    raise ValueError(kind)


def check_pipeline_hf(kind: str, split="auto"):
    """prepare_pippy on a transformers model (reference inference.py:75-123 traces any HF model): the last stage's
    logits (micro-batched, gathered to every rank) equal the unsplit model's on one process."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd.inference import prepare_pippy

    state = PartialState(cpu=True)
    set_seed(0)
    model, inputs = _tiny_hf_model(kind)
    model.eval()
    with torch.no_grad():
        ref = model(**inputs).logits
    model = prepare_pippy(model, split_points=split, gather_output=True, num_chunks=2)
    assert len(model.hf_split_points) == state.num_processes - 1
    out = model(**inputs)
    assert torch.allclose(out.logits, ref, atol=1e-5), (kind, (out.logits - ref).abs().max())
    dist.barrier()


def _tiny_hf_causal_lm(kind: str, kv_heads: int = 2):
    import transformers as tf

    if kind == "llama":
        cfg = tf.LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                             num_attention_heads=4, num_key_value_heads=kv_heads, max_position_embeddings=64)
        return tf.LlamaForCausalLM(cfg)
    if kind == "qwen3":  # per-head q/k norms: `replicated_with_grad_allreduce`
        cfg = tf.Qwen3Config(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                             num_attention_heads=4, num_key_value_heads=2, head_dim=16, max_position_embeddings=64)
        return tf.Qwen3ForCausalLM(cfg)
    if kind == "mixtral":  # 3-D expert weights: `packed_colwise` / `rowwise` parameter entries + `moe_tp_experts`
        cfg = tf.MixtralConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2,
                               num_attention_heads=4, num_key_value_heads=2, num_local_experts=4, num_experts_per_tok=2,
                               max_position_embeddings=64)
        return tf.MixtralForCausalLM(cfg)
    raise ValueError(kind)


def check_tp_hf(kind: str, steps: int = 2):
    """TP over a transformers model's own `tp_plan` (the reference's `_prepare_tp` path, accelerator.py:1579-1639,
    on models sharded by transformers `tp_plan="auto"`): loss and full weights after `steps` SGD steps equal one
    process's on the same batch."""
    from accelerate_hpc_test_amd import ParallelismConfig

    W = int(os.environ["WORLD_SIZE"])
    acc = Accelerator(cpu=True, parallelism_config=ParallelismConfig(tp_size=W))
    set_seed(0)
    base = _tiny_hf_causal_lm(kind, kv_heads=max(2, W))  # whole kv heads per rank
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.5, momentum=0.9)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.5, momentum=0.9)
    model, opt = acc.prepare(model, opt)
    assert any(getattr(p, "_tp_spec", None) is not None for p in model.parameters()), "nothing was sharded"
    g = torch.Generator().manual_seed(3)
    for _ in range(steps):
        ids = torch.randint(0, 128, (2, 16), generator=g)
        out = model(input_ids=ids, labels=ids)
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
        ref = base(input_ids=ids, labels=ids)
        ref.loss.backward()
        base_opt.step()
        base_opt.zero_grad()
        assert torch.allclose(out.loss.detach(), ref.loss.detach(), atol=2e-5), (kind, out.loss, ref.loss)
    full = acc.get_state_dict(model)
    for n, q in base.state_dict().items():
        assert full[n].shape == q.shape, (n, full[n].shape, q.shape)
        assert torch.allclose(full[n].float(), q.float(), atol=2e-5), (kind, n, (full[n] - q).abs().max())
