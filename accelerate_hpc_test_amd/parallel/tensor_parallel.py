"""Tensor parallelism (Megatron-style column/row sharding) over the `tp` mesh dimension.

Parity target: the reference delegates TP to 🤗 transformers `tp_plan="auto"` + DTensor
(`/root/reference/src/accelerate/accelerator.py:1579-1639` `_prepare_tp`, `examples/torch_native_parallelism/
nd_parallel.py:106-117`) and replicates the leftover parameters on the `tp` mesh. Here TP is native:

  * `colwise`  — weight rows sharded (out-features / tp). Input is replicated: fwd identity, bwd all-reduce.
                 Fused projections (qkv, gate|up) are sharded per *segment* so every rank keeps whole heads /
                 matching gate and up rows.
  * `rowwise`  — weight columns sharded (in-features / tp). Output partial sums: fwd all-reduce over xGMI
                 (or reduce-scatter along the sequence with `sequence_parallel=True`).
  * `colwise_rep` — colwise whose output is all-gathered (e.g. `lm_head` → full logits on every rank).
  * `replicate` — left whole; with sequence parallelism its grads are all-reduced over `tp`.

No DTensor dispatch in the hot path: parameters stay plain local tensors tagged with a `_tp_spec`, so the FSDP
engine flat-shards the TP-local shards over `dp_shard` unchanged (2-D TP × FSDP), and full state dicts are rebuilt by
`gather_tp_state_dict`. TP groups are the innermost mesh dim, i.e. ranks on the same node (xGMI only).
"""

from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable, Optional, Union

import torch
import torch.nn as nn

from . import comm


@dataclass
class TPSpec:
    """How a parameter is sharded across the tp group."""

    dim: int  # 0 = rows (colwise), 1 = cols (rowwise)
    segments: Optional[list] = None  # sizes along `dim` of fused sub-blocks, each split separately
    group: object = None
    size: int = 1

    def local_segments(self):
        return [s // self.size for s in self.segments] if self.segments else None


def _shard_tensor(full: torch.Tensor, spec: TPSpec, rank: int) -> torch.Tensor:
    segs = spec.segments or [full.shape[spec.dim]]
    parts, off = [], 0
    for s in segs:
        if s % spec.size:
            raise ValueError(f"TP: segment of size {s} along dim {spec.dim} not divisible by tp={spec.size}")
        blk = full.narrow(spec.dim, off, s)
        parts.append(blk.chunk(spec.size, dim=spec.dim)[rank])
        off += s
    return torch.cat(parts, dim=spec.dim) if len(parts) > 1 else parts[0]


def _unshard_tensor(local: torch.Tensor, spec: TPSpec) -> torch.Tensor:
    """All-gather the TP shards of `local` and re-interleave the segments."""
    gathered = comm.all_gather_dim(local.contiguous(), spec.dim, spec.group)  # [r0 | r1 | ...] along dim
    if not spec.segments or len(spec.segments) == 1:
        return gathered
    per_rank = gathered.chunk(spec.size, dim=spec.dim)
    lsegs = spec.local_segments()
    out = []
    for si, ls in enumerate(lsegs):
        off = sum(lsegs[:si])
        for r in range(spec.size):
            out.append(per_rank[r].narrow(spec.dim, off, ls))
    return torch.cat(out, dim=spec.dim)


_PARAM_MAP: dict = {}  # old Parameter -> TP-local Parameter, collected during one parallelize_module call


def _replace_param(module: nn.Module, name: str, new: torch.Tensor, spec: TPSpec):
    old = getattr(module, name)
    p = nn.Parameter(new, requires_grad=old.requires_grad)
    p._tp_spec = spec
    setattr(module, name, p)
    _PARAM_MAP[old] = p
    return p


# ------------------------------------------------------------------------------------------------ styles
# A style shards the parameters of the module (or the single parameter) a plan entry names and installs the
# forward hooks that move activations across the tp group. Every parameter keeps a `_tp_spec` (dim, segments) so the
# FSDP engine shards the TP-local tensors unchanged and `gather_tp_state_dict` rebuilds full ones.
class ParallelStyle:
    def apply(self, module: nn.Module, group, sequence_parallel: bool):
        raise NotImplementedError

    def shard_parameter(self, module: nn.Module, name: str, group):
        """A plan entry naming a parameter rather than a module (HF MoE: `...experts.gate_up_proj`): shard it only —
        the activation hooks belong to the owning module's own entry."""
        raise ValueError(f"TP style {type(self).__name__} cannot be applied to the parameter `{name}` alone")


def _norm_dim(dim: int, ndim: int) -> int:
    return dim % ndim


def _shard_named(module, name, dim, segments, group):
    p = getattr(module, name)
    W, r = comm.group_size(group), comm.group_rank(group)
    spec = TPSpec(_norm_dim(dim, p.dim()), segments, group, W)
    return _replace_param(module, name, _shard_param_data(p, spec, r), spec)


class ColwiseParallel(ParallelStyle):
    """Output features sharded (weight dim -2: rows of a Linear, the per-expert output rows of a 3-D expert weight;
    bias dim -1). Input replicated: fwd identity, bwd all-reduce. `segments` shards fused sub-blocks separately
    (qkv, gate|up: HF `packed_colwise` = two equal segments); `gather_output` all-gathers the output (HF
    `colwise_gather_output`, e.g. `lm_head` -> full logits)."""

    def __init__(self, segments: Optional[Union[list, Callable, int]] = None, gather_output: bool = False):
        self.segments = segments
        self.gather_output = gather_output

    def _segs(self, module, p):
        segs = self.segments(module) if callable(self.segments) else self.segments
        if isinstance(segs, int):  # `packed`: this many equal sub-blocks along the sharded dim
            n = p.shape[-2] if p.dim() > 1 else p.shape[-1]
            segs = [n // segs] * segs
        return segs

    def shard_parameter(self, module, name, group):
        p = getattr(module, name)
        _shard_named(module, name, -2 if p.dim() > 1 else -1, self._segs(module, p), group)

    def apply(self, module, group, sequence_parallel):
        segs = self._segs(module, module.weight)
        if isinstance(module, nn.Embedding):
            raise ValueError("colwise on an nn.Embedding: use `embedding_colwise` / `embedding_rowwise`")
        _shard_named(module, "weight", -2, segs, group)
        if getattr(module, "bias", None) is not None:
            _shard_named(module, "bias", -1, segs, group)
        if isinstance(module, nn.Linear):
            module.out_features = module.weight.shape[0]
        gather = self.gather_output

        def pre(mod, args):
            x = args[0]
            x = comm.gather_along(x, 1, group) if sequence_parallel else comm.copy_to_group(x, group)
            return (x,) + tuple(args[1:])

        def post(mod, args, out):
            if not gather:
                return out
            if segs and len(segs) > 1:  # gathered [r0 seg0 | r0 seg1 | r1 seg0 ...] -> [seg0 | seg1]
                full = comm.gather_along(out, -1, group, reduce_grad=False)
                per = full.chunk(comm.group_size(group), dim=-1)
                parts = [q.split([sg // comm.group_size(group) for sg in segs], dim=-1) for q in per]
                return torch.cat([parts[rk][si] for si in range(len(segs)) for rk in range(len(per))], dim=-1)
            return comm.gather_along(out, -1, group, reduce_grad=False)

        module.register_forward_pre_hook(pre)
        module.register_forward_hook(post)


class RowwiseParallel(ParallelStyle):
    """Input features sharded (weight dim -1). Output partial sums: fwd all-reduce over xGMI (or reduce-scatter along
    the sequence with `sequence_parallel=True`); the bias is added once, after the reduction. `split_input` (HF
    `rowwise_split_input`) keeps this rank's chunk of a replicated input first; `segments` as in ColwiseParallel (HF
    `packed_rowwise`)."""

    def __init__(self, split_input: bool = False, segments: Optional[Union[list, int]] = None):
        self.split_input = split_input
        self.segments = segments

    def _segs(self, p):
        segs = self.segments
        if isinstance(segs, int):
            segs = [p.shape[-1] // segs] * segs
        return segs

    def shard_parameter(self, module, name, group):
        p = getattr(module, name)
        if p.dim() > 1:
            _shard_named(module, name, -1, self._segs(p), group)

    def apply(self, module, group, sequence_parallel):
        _shard_named(module, "weight", -1, self._segs(module.weight), group)
        if isinstance(module, nn.Linear):
            module.in_features = module.weight.shape[1]
        bias = getattr(module, "bias", None)
        if bias is not None:
            # bias is added once, after the reduction
            module._tp_bias = bias
            module.bias = None
        split = self.split_input

        if split:
            module.register_forward_pre_hook(
                lambda mod, args: (comm.split_along(args[0], -1, group),) + tuple(args[1:]))

        def post(mod, args, out):
            out = comm.reduce_scatter_along(out, 1, group) if sequence_parallel else comm.reduce_from_group(out, group)
            if getattr(mod, "_tp_bias", None) is not None:
                out = out + mod._tp_bias
            return out

        module.register_forward_hook(post)


class VocabParallelEmbedding(ParallelStyle):
    """HF `embedding_rowwise`: the vocabulary (weight dim 0) is sharded; ids outside this rank's range look up row 0
    and are zeroed, and the partial embeddings are all-reduced."""

    def apply(self, module, group, sequence_parallel):
        if module.weight.shape[0] % comm.group_size(group):
            raise ValueError(f"embedding_rowwise: vocabulary {module.weight.shape[0]} not divisible by tp")
        _shard_named(module, "weight", 0, None, group)
        rank = comm.group_rank(group)

        def pre(mod, args):
            ids = args[0]
            n = mod.weight.shape[0]
            lo = rank * n
            mask = (ids < lo) | (ids >= lo + n)
            mod._tp_mask = mask
            return ((ids - lo).masked_fill(mask, 0),) + tuple(args[1:])

        def post(mod, args, out):
            out = out.masked_fill(mod._tp_mask.unsqueeze(-1), 0.0)
            del mod._tp_mask
            return comm.reduce_from_group(out, group)

        if hasattr(module, "num_embeddings"):
            module.num_embeddings = module.weight.shape[0]
        module.register_forward_pre_hook(pre)
        module.register_forward_hook(post)


class EmbeddingColwise(ParallelStyle):
    """HF `embedding_colwise`: the embedding dim (weight dim 1) is sharded; outputs are all-gathered."""

    def apply(self, module, group, sequence_parallel):
        _shard_named(module, "weight", 1, None, group)
        if hasattr(module, "embedding_dim"):
            module.embedding_dim = module.weight.shape[1]
        module.register_forward_hook(lambda mod, args, out: comm.gather_along(out, -1, group, reduce_grad=False))


class ReplicateParallel(ParallelStyle):
    def apply(self, module, group, sequence_parallel):
        pass

    def shard_parameter(self, module, name, group):
        pass


class ReplicatedGradAllReduce(ParallelStyle):
    """HF `replicated_with_grad_allreduce`: replicated parameters that sit between colwise and rowwise layers (per-head
    q/k norms) see only this rank's heads, so their gradients are summed over tp."""

    def apply(self, module, group, sequence_parallel):
        # marks the module at parallelize time (the hook itself is attached at the first forward): engines that write a
        # parameter's gradient straight into a buffer (FSDP gradient slots) must leave these parameters on autograd so
        # the tp all-reduce hook fires
        module._tp_grad_allreduce_group = group

        def attach(mod, args):  # lazily: engines may replace the Parameter objects after parallelize
            for p in mod.parameters(recurse=False):
                if p.requires_grad and not getattr(p, "_tp_grad_hooked", False):
                    p.register_hook(lambda g, _grp=group: comm.all_reduce_(g.contiguous().clone(), _grp))
                    p._tp_grad_hooked = True

        module.register_forward_pre_hook(attach)


class MoeExpertsParallel(ParallelStyle):
    """HF `moe_tp_experts`: the experts module of a TP-sharded MoE layer (its `gate_up_proj` / `down_proj` parameters
    carry their own packed_colwise / rowwise entries). Hidden states and routing weights enter replicated (bwd
    all-reduce: the colwise expert GEMMs and the per-rank partial outputs both feed their gradients); the partial
    expert outputs are all-reduced."""

    def apply(self, module, group, sequence_parallel):
        def pre(mod, args, kwargs):
            args = list(args)
            if args:
                args[0] = comm.copy_to_group(args[0], group)
            if len(args) > 2 and torch.is_tensor(args[2]) and args[2].is_floating_point():
                args[2] = comm.copy_to_group(args[2], group)
            for k in ("hidden_states", "top_k_weights", "routing_weights"):
                if k in kwargs and torch.is_tensor(kwargs[k]):
                    kwargs[k] = comm.copy_to_group(kwargs[k], group)
            return tuple(args), kwargs

        module.register_forward_pre_hook(pre, with_kwargs=True)
        module.register_forward_hook(lambda mod, args, out: comm.reduce_from_group(out, group))


class AllReduceOutput(ParallelStyle):
    """HF `all_reduce`: the module's forward output is a partial sum over tp."""

    def apply(self, module, group, sequence_parallel):
        module.register_forward_hook(lambda mod, args, out: comm.reduce_from_group(out, group))


class SequenceParallel(ParallelStyle):
    """Module runs on the local sequence shard (norms between rowwise → colwise pairs). Its replicated params
    only see 1/tp of the tokens, so their grads are summed over tp."""

    def apply(self, module, group, sequence_parallel):
        if not sequence_parallel:
            return
        ReplicatedGradAllReduce().apply(module, group, sequence_parallel)


class SplitSequenceOutput(ParallelStyle):
    """Sequence-parallel entry point (token embeddings): the output keeps this rank's sequence chunk."""

    def apply(self, module, group, sequence_parallel):
        if not sequence_parallel:
            return
        module.register_forward_hook(lambda mod, args, out: comm.split_along(out, 1, group))


class _Unsupported(ParallelStyle):
    def __init__(self, name, why):
        self.name, self.why = name, why

    def apply(self, module, group, sequence_parallel):
        raise ValueError(f"TP style `{self.name}` is not supported here: {self.why}")

    shard_parameter = apply


def _shard_param_data(p: torch.Tensor, spec: TPSpec, rank: int) -> torch.Tensor:
    if p.device.type == "meta":
        shape = list(p.shape)
        shape[spec.dim] //= spec.size
        return torch.empty(shape, dtype=p.dtype, device="meta")
    return _shard_tensor(p.data, spec, rank).clone()


_EP = ("expert parallelism is configured with ParallelismConfig(ep_size=...) (models/moe.py), not through the tp "
       "plan")
_STYLE_BY_NAME = {
    # this framework's names
    "colwise_rep": lambda: ColwiseParallel(gather_output=True),
    "rowwise_rep": lambda: RowwiseParallel(),
    "replicate": lambda: ReplicateParallel(),
    "sequence_parallel": lambda: SequenceParallel(),
    "seq_split": lambda: SplitSequenceOutput(),
    # transformers tp_plan names (transformers/integrations/tensor_parallel.py ParallelInterface)
    "colwise": lambda: ColwiseParallel(),
    "colwise_gather_output": lambda: ColwiseParallel(gather_output=True),
    "packed_colwise": lambda: ColwiseParallel(segments=2),
    "rowwise": lambda: RowwiseParallel(),
    "rowwise_split_input": lambda: RowwiseParallel(split_input=True),
    "packed_rowwise": lambda: RowwiseParallel(segments=2),
    "embedding_rowwise": lambda: VocabParallelEmbedding(),
    "embedding_colwise": lambda: EmbeddingColwise(),
    "replicated_with_grad_allreduce": lambda: ReplicatedGradAllReduce(),
    "moe_tp_experts": lambda: MoeExpertsParallel(),
    "all_reduce": lambda: AllReduceOutput(),
    "local": lambda: ReplicateParallel(),
    "local_colwise": lambda: ColwiseParallel(),
    "local_rowwise": lambda: RowwiseParallel(),
    "gather": lambda: ReplicateParallel(),
    "grouped_gemm": lambda: _Unsupported("grouped_gemm", _EP),
    "ep_router": lambda: _Unsupported("ep_router", _EP),
    "moe_identity_expert": lambda: _Unsupported("moe_identity_expert", "zero / identity experts"),
    "mla_kv_a_proj": lambda: _Unsupported("mla_kv_a_proj", "MLA (DeepSeek-V2-style) attention"),
}


def _resolve_style(s) -> ParallelStyle:
    if isinstance(s, ParallelStyle):
        return s
    if s not in _STYLE_BY_NAME:
        raise ValueError(f"Unknown TP style `{s}`; choose from {sorted(_STYLE_BY_NAME)} or pass a ParallelStyle.")
    return _STYLE_BY_NAME[s]()


def _match(name: str, pattern: str) -> bool:
    """HF plan keys: `*` stands for one path component (a layer index)."""
    return re.fullmatch(re.escape(pattern).replace(r"\*", r"[^.]+"), name) is not None


def get_tp_plan(model: nn.Module, sequence_parallel: bool = False) -> Optional[dict]:
    """Model-provided plan: our models' `tp_plan()`, or a transformers `_tp_plan` / `config.base_model_tp_plan`."""
    if hasattr(model, "tp_plan") and callable(model.tp_plan):
        return model.tp_plan(sequence_parallel=sequence_parallel)
    plan = {}
    if sequence_parallel:
        raise ValueError("sequence-parallel TP needs a plan with sequence-parallel entries (this framework's models' "
                         "`tp_plan(sequence_parallel=True)`); a transformers tp_plan has none — pass `plan=`")
    base = getattr(getattr(model, "config", None), "base_model_tp_plan", None)
    if base:
        prefix = getattr(model, "base_model_prefix", "")
        inner = getattr(model, prefix, None) if prefix else None
        plan.update({(f"{prefix}.{k}" if inner is not None else k): v for k, v in base.items()})
    for k, v in (getattr(model, "_tp_plan", None) or {}).items():
        plan[k] = v
    return plan or None


def parallelize_module(model: nn.Module, group, plan: Optional[dict] = None, sequence_parallel: bool = False) -> nn.Module:
    """Apply `plan` ({module-name glob: style}) to `model` over the `group` tensor-parallel process group.

    After sharding, modules exposing `shard_heads(tp_size)` (attention) adapt their local head counts. With
    `sequence_parallel`, gradients of replicated parameters are all-reduced across tp (they see different
    sequence shards)."""
    W = comm.group_size(group)
    if W == 1:
        return model
    try:
        from torch.distributed.tensor import DTensor
    except ImportError:  # pragma: no cover
        DTensor = ()
    if any(isinstance(p, DTensor) for p in model.parameters()):
        # already sharded by transformers (`from_pretrained(tp_plan="auto", device_mesh=...)`, the reference's flow) or
        # torch's `parallelize_module`: keep its DTensor layout. The optimizer then runs torch's DTensor-aware AdamW
        # (the fused HIP kernel needs plain storage, optimizer._fused_adam_eligible) and the gradient norm sums the
        # sharded placements over their mesh (Accelerator._clip_grad_norm_dtensor).
        model._tp_group, model._tp_size, model._tp_sequence_parallel = group, W, False
        model._tp_dtensor = True
        return model
    plan = plan if plan is not None else get_tp_plan(model, sequence_parallel)
    if plan is None:
        raise ValueError("No tensor-parallel plan: pass `plan=` or give the model a `tp_plan()` / transformers `_tp_plan`.")
    _PARAM_MAP.clear()
    matched = set()
    for name, module in list(model.named_modules()):
        for pattern, style in plan.items():
            if _match(name, pattern):
                _resolve_style(style).apply(module, group, sequence_parallel)
                matched.add(pattern)
                break
    # entries that name a parameter (HF MoE experts' 3-D `gate_up_proj` / `down_proj`)
    for pname, _ in list(model.named_parameters()):
        for pattern, style in plan.items():
            if _match(pname, pattern):
                mod_name, _, leaf = pname.rpartition(".")
                owner = model.get_submodule(mod_name) if mod_name else model
                if getattr(getattr(owner, leaf), "_tp_spec", None) is None:
                    _resolve_style(style).shard_parameter(owner, leaf, group)
                matched.add(pattern)
                break
    for m in model.modules():
        if hasattr(m, "shard_heads"):
            m.shard_heads(W)
        hd = getattr(m, "head_dim", None)
        if isinstance(hd, int) and hd > 0:  # HF attention: every rank must keep whole heads of q / k / v
            for proj in ("q_proj", "k_proj", "v_proj"):
                lin = getattr(m, proj, None)
                w = getattr(lin, "weight", None)
                if w is not None and getattr(w, "_tp_spec", None) is not None and w.shape[0] % hd:
                    raise ValueError(f"TP={W}: `{proj}` keeps {w.shape[0]} output features per rank, not a whole "
                                     f"number of heads of {hd} (its head count must be divisible by tp)")
    model._tp_param_map = dict(_PARAM_MAP)  # lets an optimizer built on the unsharded model be re-pointed
    _PARAM_MAP.clear()
    model._tp_group = group
    model._tp_size = W
    model._tp_sequence_parallel = sequence_parallel
    return model


def gather_tp_state_dict(state_dict: dict, model: nn.Module) -> dict:
    """Replace TP-local tensors in `state_dict` by their full (unsharded) values. Collective over tp."""
    specs = {n: p._tp_spec for n, p in model.named_parameters() if getattr(p, "_tp_spec", None) is not None}
    if not specs:
        return state_dict
    out = dict(state_dict)
    for name, spec in specs.items():
        key = name if name in out else next((k for k in out if k.endswith(name)), None)
        if key is None:
            continue
        t = out[key]
        dev = t.device
        src = t.to(comm_device(spec.group)) if dev.type == "cpu" and not comm._is_gloo(spec.group) else t
        out[key] = _unshard_tensor(src, spec).to(dev)
    return out


def shard_tp_state_dict(state_dict: dict, model: nn.Module) -> dict:
    """Inverse of `gather_tp_state_dict`: slice full tensors for this TP rank (used when loading)."""
    out = dict(state_dict)
    for name, p in model.named_parameters():
        spec = getattr(p, "_tp_spec", None)
        if spec is not None and name in out and out[name].shape != p.shape:
            out[name] = _shard_tensor(out[name], spec, comm.group_rank(spec.group)).contiguous()
    return out


def comm_device(group):
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
