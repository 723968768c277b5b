"""Native fully-sharded data parallel engine (FSDP2-equivalent) for MI355X.

Parity: the reference wraps `torch.distributed.fsdp.fully_shard` (`/root/reference/src/accelerate/accelerator.py:1656-1746`,
`utils/fsdp_utils.py:621-737`). Here the engine is our own:

* **Units.** The wrap policy (transformer classes / min params / none) selects modules; each selected module's
  parameters (plus the leftovers, in a root unit) are flattened into ONE buffer per unit, padded to a multiple of
  the shard world size. Rank r owns the contiguous slice r of that buffer.
* **Precision.** Each unit keeps an fp32 master shard (what the optimizer updates), an fp32 gradient shard, and a
  `param_dtype` (bf16) shard that is the all-gather input. The fused HIP AdamW writes the bf16 shard in the same
  pass as the fp32 update (`_acc_bf16_shadow`), so there is no separate cast pass. The reference's fp32 "upcast"
  loop is a no-op (`utils/fsdp_utils.py:723-736`); here master weights are explicitly fp32.
* **Unshard.** The original `nn.Parameter` objects stay registered in their modules; their `.data` are views into
  the unit's full bf16 buffer, whose storage is resized 0 ↔ full. Before a unit runs, RCCL `all_gather_into_tensor`
  fills it on a dedicated HIP stream; the next unit in execution order is prefetched (depth configurable) so the
  gather of block i+1 overlaps block i's compute. After forward (`reshard_after_forward`) the storage is freed and
  re-gathered before the unit's backward (triggered by a gradient hook on the unit's outputs).
* **Reduce.** Parameter grads accumulate in place into a flat bf16 gradient buffer (pre-assigned `.grad` views).
  For plain `nn.Linear` weights the weight-gradient GEMM itself targets the buffer (gradient-accumulation fusion:
  `mm(dyᵀ, x, out=slot)` on first touch, `addmm_` after), so no separate grad tensor, add or zero fill exists.
  When every parameter of the unit has accumulated (post-accumulate-grad hooks), ONE `reduce_scatter_tensor` runs on
  the reduce stream; its output is scaled by 1/W and accumulated into the fp32 gradient shard. HSDP adds an
  all-reduce across the replicate group. `no_sync` (`set_requires_gradient_sync(False)`) keeps the flat grads.
* **World size 1** degenerates to zero collectives: the bf16 shard IS the full buffer (no copies).
* **CPU offload** (`plugin.cpu_offload`, reference `fsdp_utils.py:648` offload_policy): the fp32 master shard, the fp32
  gradient shard and the optimizer state live in pinned host memory and the optimizer step runs on the host (native
  OpenMP AdamW, `csrc/runtime/cpu_adam.cpp`, which also writes the bf16 upload copy). Only the bf16 all-gather
  source (2 B/param/W) stays in HBM: on a 288 GB MI355X that is the cheap part, and keeping it resident avoids an H2D
  per all-gather. Reduced gradients go D2H from the reduce stream; the host waits for them at the end of backward.

Messages are one transformer block each (≈436 MB bf16 for Llama-3-8B), large enough for RCCL to spread over all 7
xGMI links; streams and events order everything on the device — the host never blocks.
"""

from __future__ import annotations

import json
import math
import os
import weakref
from collections import OrderedDict
from contextlib import contextmanager
from typing import Callable, Iterable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.dataclasses import FullyShardedDataParallelPlugin, MixedPrecisionPolicy
from ..utils.fault_tolerance import record_collective
from ..utils.tracing import trace_range
from ..ops._ext import ext, native_enabled
from ..ops.fp8 import Fp8Linear
from ..ops import fused as fused_ops
from ..ops.fused import linear_dgrad, linear_fwd, wgrad_into
from . import small_allreduce

_ALIGN = 64  # elements; keeps every rank's shard 128-B aligned for bf16 / 256-B for fp32
# opt-in: on MI355X the searched algorithms measured 0.3-0.6 % slower end to end than torch's default pick (interleaved A/B,
# profiles/r1_session3_benches.json), so the torch path stays the default
_WGRAD_XT = os.environ.get("ACCELERATE_FSDP_WGRAD_XT", "1") != "0"


def _round_up(x, m):
    return (x + m - 1) // m * m


class _ParamInfo:
    __slots__ = ("fqn", "module", "attr", "param", "orig_param", "offset", "numel", "shape", "shard_param", "local_lo", "local_hi",
                 "param_lo", "fused", "fused_written", "region", "f8_index", "f8_t")

    def __init__(self, fqn, module, attr, param, offset):
        self.fqn = fqn
        self.module = module
        self.attr = attr
        self.param = param
        self.orig_param = param
        self.offset = offset
        self.numel = param.numel()
        self.shape = tuple(param.shape)
        self.shard_param = None
        self.local_lo = self.local_hi = self.param_lo = 0
        self.fused = False  # weight-gradient GEMM writes straight into the flat grad buffer (see _WgradSlot)
        self.fused_written = False
        self.region = None
        self.f8_index = -1
        self.f8_t = None  # world-size-1 fp8 weights: the stored K-major e4m3 copy (FSDPEngine._init_fp8_all_gather)


class _Region:
    """A contiguous span [base, base + length) of a unit's flat buffer, sharded on its own: rank r owns
    [base + r * shard_len, base + (r + 1) * shard_len), stored at [shard_base, shard_base + shard_len) of its shard."""

    __slots__ = ("base", "length", "shard_len", "shard_base", "fp8")

    def __init__(self, base, length, world, shard_base, fp8=False):
        self.base, self.length, self.fp8 = base, length, fp8
        self.shard_len = length // world
        self.shard_base = shard_base

    def slice_of(self, rank):
        lo = self.base + rank * self.shard_len
        return lo, lo + self.shard_len


class FlatUnit:
    """One sharding unit (e.g. a decoder layer).

    Its parameters are laid out in one flat buffer made of one or two `_Region`s. Normally a single region; with the
    fp8 all-gather the unit's fp8 GEMM weights form region 0 (all-gathered as e4m3 bytes) and everything else
    region 1 (all-gathered in bf16). Each rank's shard is the concatenation of its slice of every region."""

    def __init__(self, engine: "FSDPEngine", idx: int, module: nn.Module, infos: list[_ParamInfo], fp8_count: int = 0):
        self.engine = engine
        self.idx = idx
        self.module = module
        W = engine.world_size
        quantum = W * _ALIGN
        groups = [infos[:fp8_count], infos[fp8_count:]] if fp8_count else [infos]
        self.infos, self.regions = [], []
        base = shard_base = 0
        for gi, group in enumerate(groups):
            off = base
            for info in group:  # pack the group's parameters from the region base
                info.offset = off
                off += info.numel
                self.infos.append(info)
            length = _round_up(max(off - base, 1), quantum)
            region = _Region(base, length, W, shard_base, fp8=bool(fp8_count) and gi == 0)
            self.regions.append(region)
            base += length
            shard_base += region.shard_len
        for info in self.infos:
            info.region = next(r for r in self.regions if r.base <= info.offset < r.base + r.length) if info.numel else self.regions[-1]
        self.numel = sum(i.numel for i in infos)
        self.padded = base
        self.shard_numel = shard_base
        self.f8 = self.regions[0] if fp8_count else None
        self.f8_infos = [i for i in self.infos if self.f8 is not None and i.region is self.f8]
        # bf16 compute buffer covers the non-fp8 regions only
        self.bf_base = self.regions[1].base if fp8_count else 0
        self.f8_shard = self.f8_full = self.f8_amax = None
        self.is_root = False
        self.state = "sharded"  # or "unsharding" / "unsharded"
        self.ag_event: Optional[torch.cuda.Event] = None
        self.full: Optional[torch.Tensor] = None
        self.full_grad: Optional[torch.Tensor] = None
        self.pending_grads = 0
        self.grad_ready = False
        self.reduced = False
        self.bwd_prefetched = False
        self.in_backward = False

    # --- layout -------------------------------------------------------------------------------------------
    def local_of_full(self, full: torch.Tensor) -> torch.Tensor:
        """This rank's shard (region slices concatenated) cut out of a full-layout tensor."""
        r = self.engine.rank
        parts = [full[slice(*reg.slice_of(r))] for reg in self.regions]
        return parts[0].clone() if len(parts) == 1 else torch.cat(parts)

    def local_range(self, info):
        """(local_lo, local_hi, param_lo) of `info`'s piece in this rank's shard."""
        reg = info.region
        lo, hi = reg.slice_of(self.engine.rank)
        a, b = max(info.offset, lo), min(info.offset + info.numel, hi)
        if b <= a:
            a = b = max(min(info.offset, hi), lo)
        return reg.shard_base + (a - lo), reg.shard_base + (b - lo), a - info.offset


class FSDPEngine:
    def __init__(
        self,
        model: nn.Module,
        plugin: FullyShardedDataParallelPlugin,
        device: torch.device,
        process_group=None,
        replicate_group=None,
        init_fn: Optional[Callable[[nn.Module], None]] = None,
        seed: int = 0,
        prefetch_depth: int = 1,
        force_sharded: bool = False,
        fp8_all_gather: bool = False,
    ):
        self.model = model
        self.fp8_all_gather = bool(fp8_all_gather)
        self.f8_units: list = []
        self.plugin = plugin
        self.device = device
        self.group = process_group
        self.replicate_group = replicate_group
        if dist.is_available() and dist.is_initialized():
            self.world_size = dist.get_world_size(process_group)
            self.rank = dist.get_rank(process_group)
        else:
            self.world_size, self.rank = 1, 0
        self.replicate_size = dist.get_world_size(replicate_group) if replicate_group is not None else 1
        self.replicate_rank = dist.get_rank(replicate_group) if replicate_group is not None else 0
        # `sharded`: the unit buffers are sharded and every collective of the W>1 path runs. At world size 1 this is the
        # degenerate no-collective path unless `force_sharded` (RcclKwargs.fsdp_force_sharded): then the one GPU runs
        # exactly the multi-GPU code (separate full buffer resized 0 <-> full, RCCL all-gather / reduce-scatter with
        # nranks=1, bf16 flat grads reduced into the fp32 shard, reshard-after-forward and prefetch).
        self.sharded = self.world_size > 1 or (bool(force_sharded) and dist.is_available() and dist.is_initialized())
        if self.sharded or self.replicate_size > 1:
            fused_ops.set_dgrad_concurrent(True)  # collectives beside the backward: dgrad without the transpose kernel
        mp = plugin.mixed_precision_policy or MixedPrecisionPolicy()
        self.param_dtype = mp.param_dtype or torch.float32
        self.reduce_dtype = mp.reduce_dtype or self.param_dtype
        self.output_dtype = mp.output_dtype
        self.reshard_after_forward = bool(plugin.reshard_after_forward) and self.sharded
        self.prefetch_depth = max(0, prefetch_depth)
        # FSDP1 prefetch flags (reference accelerator.py:1909-1925 passes them to torch FSDP1). FSDP2 has neither
        # flag: the forward prefetches `prefetch_depth` units ahead and the backward prefetches before each unit's
        # gradient computation. With fsdp_version=1:
        #   forward_prefetch=False -> no explicit forward prefetch (the next all-gather is issued by the next unit's
        #     pre-forward hook, which still overlaps the GPU when the host runs ahead); True -> `prefetch_depth` ahead;
        #   backward_prefetch None (NO_PREFETCH) / BACKWARD_PRE (before this unit's gradient computation) /
        #     BACKWARD_POST (after this unit's gradients are reduced);
        #   limit_all_gathers=False -> at least 2 units of forward prefetch (True: the engine's inherent bound of
        #     prefetch_depth + 1 gathered units, as each unit's buffer is freed in stream order after its use).
        self.fsdp1 = getattr(plugin, "fsdp_version", 2) == 1
        if self.fsdp1:
            self.fwd_prefetch_depth = self.prefetch_depth if plugin.forward_prefetch else 0
            if plugin.forward_prefetch and plugin.limit_all_gathers is False:
                self.fwd_prefetch_depth = max(self.fwd_prefetch_depth, 2)
            self.bwd_prefetch = plugin.backward_prefetch  # None, "BACKWARD_PRE" or "BACKWARD_POST"
        else:
            self.fwd_prefetch_depth = self.prefetch_depth
            self.bwd_prefetch = "BACKWARD_PRE"
        self.requires_grad_sync = True
        self.is_cuda = device.type == "cuda"
        # host ranks on gloo run the same all_gather_into_tensor / reduce_scatter_tensor calls as RCCL ranks (the CPU
        # tests then cover the exact shard offsets and buffers); only HIP tensors on a gloo group (several ranks
        # sharing one GPU in the one-GPU rehearsal) need the list / all-reduce forms, gloo's tensor forms being host-only
        self._uses_gloo = self.is_cuda and (dist.is_available() and dist.is_initialized()
                                            and dist.get_backend(process_group) == "gloo")
        self.offload = plugin.cpu_offload not in (None, False)
        self._pin = self.offload and torch.cuda.is_available() and getattr(plugin.cpu_offload, "pin_memory", True)
        self._d2h_pending = []
        if self.is_cuda:
            self.ag_stream = torch.cuda.Stream(device=device, priority=-1)
            # ACCELERATE_FSDP_RS_PRIORITY: 0 = the reduce-scatter / gradient-shard update stream at normal priority (its
            # work is needed only at the end of backward), -1 = high like the all-gather stream
            self.rs_stream = torch.cuda.Stream(device=device, priority=int(os.environ.get("ACCELERATE_FSDP_RS_PRIORITY", "-1")))
        else:
            self.ag_stream = self.rs_stream = None
        # All-gather and reduce-scatter get communicators of their own (same ranks as `group`): ProcessGroupNCCL runs
        # all collectives of one group on that group's single internal stream (event-fenced against the issuing
        # stream), so only separate groups let the backward prefetch AG(i-1) overlap RS(i+1) (comm.duplicate_group).
        self.ag_group = self.rs_group = process_group
        if self.sharded and self.is_cuda and dist.get_backend(process_group) != "gloo":
            from .comm import duplicate_group

            self.ag_group = duplicate_group(process_group)
            self.rs_group = duplicate_group(process_group)
        self.units: list[FlatUnit] = []
        self.exec_order: list[FlatUnit] = []
        self._recording_order = True
        self._final_cb_queued = False
        self._pending_frees = []
        self._build_units(init_fn, seed)

    # =========================================================================================== build
    def _wrap_fn(self):
        fn = getattr(self.plugin, "_wrap_fn", None)
        if fn is None and self.plugin.auto_wrap_policy not in (None, "NO_WRAP"):
            fn = self.plugin.set_auto_wrap_policy(self.model)
        return fn

    def _build_units(self, init_fn, seed):
        wrap = self._wrap_fn()
        owned: set[int] = set()
        ignored = set()
        if self.plugin.ignored_modules is not None and not isinstance(self.plugin.ignored_modules, str):
            for m in self.plugin.ignored_modules:
                for p in m.parameters():
                    ignored.add(id(p))
        unit_modules = []
        if wrap is not None:
            # post-order: inner matches become units before their parents
            def visit(m):
                for c in m.children():
                    visit(c)
                if m is not self.model and wrap(m):
                    unit_modules.append(m)

            visit(self.model)
        name_of = {id(m): n for n, m in self.model.named_modules()}
        if wrap is not None:
            unit_modules += self._large_root_leaves(unit_modules, ignored)
        assigned_units = []
        for m in unit_modules:
            infos = self._collect(m, name_of[id(m)], owned, ignored)
            if infos:
                assigned_units.append((m, infos))
        root_infos = self._collect(self.model, "", owned, ignored)
        # Units are created in module order; the root goes first so its index is 0.
        all_units = [(self.model, root_infos, True)] + [(m, infos, False) for m, infos in assigned_units]
        refs = {}
        if self.fp8_all_gather:
            for mod in self.model.modules():
                for p in mod._parameters.values():
                    if p is not None:
                        refs[id(p)] = refs.get(id(p), 0) + 1
        for idx, (m, infos, is_root) in enumerate(all_units):
            f8 = [i for i in infos if self._fp8_gathered(i, refs)]
            f8_ids = {id(i) for i in f8}
            unit = FlatUnit(self, idx, m, f8 + [i for i in infos if id(i) not in f8_ids], fp8_count=len(f8))
            unit.is_root = is_root
            self._materialize(unit, init_fn, seed)
            self.units.append(unit)
        self.root = self.units[0]
        self._init_fp8_all_gather()
        self._init_expert_amax()
        # parameters the engine does not own (ignored modules, expert-parallel experts): kept as plain device
        # tensors; they still take part in the global grad-norm (see clip_grad_norm_)
        self.extra_names = [n for n, p in self.model.named_parameters() if id(p) in ignored]
        self.extra_params = [p for p in self.model.parameters() if id(p) in ignored]
        for p in self.extra_params:
            if p.device.type != "meta" and p.device != self.device:
                p.data = p.data.to(self.device)
        for unit in self.units[1:]:
            unit.module.register_forward_pre_hook(self._make_pre_forward(unit), with_kwargs=True)
            unit.module.register_forward_hook(self._make_post_forward(unit), with_kwargs=True)
        for unit in self.units:
            for info in unit.infos:
                if info.param.requires_grad:
                    info.param.register_post_accumulate_grad_hook(self._make_grad_hook(unit))
        if os.environ.get("ACCELERATE_FSDP_FUSED_WGRAD", "1") != "0":
            self._install_fused_wgrad()

    def _large_root_leaves(self, unit_modules, ignored) -> list:
        """Large leaf modules the wrap policy left in the root (Llama's token embedding and lm_head: 525 M params each,
        1.05 GB bf16): each becomes a unit of its own. In the root they would be all-gathered before the first block
        (not overlapped with anything) and reduce-scattered after the last gradient of the step (2.1 GB each way,
        ~6 ms per direction over 7 xGMI links at 8 GPUs); as units, the lm_head's gather is prefetched under the last
        blocks' forward and its reduce-scatter overlaps the blocks' backward, leaving only the embedding's exposed.
        Only modules whose parameters no other module shares (tied embeddings stay in the root).
        `ACCELERATE_FSDP_SPLIT_ROOT=0` keeps everything in the root (reference FSDP2 wrap behaviour)."""
        if os.environ.get("ACCELERATE_FSDP_SPLIT_ROOT", "1") == "0":
            return []
        min_params = int(os.environ.get("ACCELERATE_FSDP_SPLIT_ROOT_MIN_PARAMS", 16 << 20))
        inside = set()
        for m in unit_modules:
            inside.update(id(x) for x in m.modules())
        refs = {}
        for m in self.model.modules():
            for q in m._parameters.values():
                if q is not None:
                    refs[id(q)] = refs.get(id(q), 0) + 1
        out = []
        for m in self.model.modules():
            if m is self.model or id(m) in inside or next(m.children(), None) is not None:
                continue
            params = [q for q in m._parameters.values() if q is not None]
            if not params or any(refs.get(id(q), 0) != 1 or id(q) in ignored for q in params):
                continue
            if sum(q.numel() for q in params) >= min_params:
                out.append(m)
        return out

    # =========================================================================================== fp8 all-gather
    def _fp8_gathered(self, info: _ParamInfo, refs: dict) -> bool:
        """Whether `info` is an fp8 GEMM weight that travels as e4m3 in the all-gather (torchao
        `enable_fsdp_float8_all_gather` semantics: dynamic per-tensor scaling from the global amax)."""
        if not self.fp8_all_gather or self.param_dtype != torch.bfloat16 or self.offload:
            return False
        if os.environ.get("ACCELERATE_FSDP_FUSED_WGRAD", "1") == "0":
            # an e4m3 parameter cannot take an autograd gradient: its weight gradient must go to the fused slot
            return False
        m = info.module
        rec = getattr(m, "fp8_recipe", None)
        return (isinstance(m, Fp8Linear) and info.attr == "weight" and info.param.requires_grad and len(info.shape) == 2
                and refs.get(id(info.param), 0) == 1 and getattr(info.param, "_tp_spec", None) is None
                and rec is not None and not rec.delayed and not rec.mx and not rec.fwd_e5m2())

    def _init_fp8_all_gather(self):
        """Index the fp8-gathered weights (one amax slot each, in one engine-wide buffer so the global amax is ONE
        all-reduce per step) and quantise the initial shards."""
        self.f8_units = [u for u in self.units if u.f8 is not None]
        if not self.f8_units:
            return
        n = 0
        for u in self.f8_units:
            lo, hi = [], []
            for info in u.f8_infos:
                info.f8_index = n
                n += 1
                lo.append(info.local_lo)
                hi.append(info.local_hi)
                info.param._acc_fp8_ag = (u, info)  # read by Fp8Linear.forward
            assert max(hi, default=0) <= u.f8.shard_len and min(lo, default=0) >= 0, "fp8 segment outside the fp8 region"
            u.f8_seg = (torch.tensor(lo, dtype=torch.long, device=self.device), torch.tensor(hi, dtype=torch.long, device=self.device),
                        max((b - a for a, b in zip(lo, hi)), default=0), n - len(lo))
        self.f8_amax_all = torch.zeros(n, dtype=torch.float32, device=self.device)
        for u in self.f8_units:
            first = u.f8_seg[3]
            u.f8_amax = self.f8_amax_all[first : first + len(u.f8_infos)]
            # the fused AdamW writes these weights' bf16 shards and can max-reduce them into the amax slots on the way
            # (ops/multi_tensor.py FusedAdamStep); refresh_fp8 then skips its own amax pass for the unit
            u.f8_amax_fresh = False
            u.f8_param_ids = {id(info.shard_param) for info in u.f8_infos}
            for k, info in enumerate(u.f8_infos):
                info.shard_param._acc_fp8_amax = (self, u, u.f8_amax[k : k + 1])
        # World size 1 (no all-gather), opt-in with ACCELERATE_FP8_PRETRANSPOSE=1: the e4m3 weights are persistent, so
        # their K-major copies for the dgrad GEMM can be kept too and written by the same per-step cast (one read of the
        # bf16 weight writes both layouts) instead of a byte transpose of every weight in every backward. Measured on
        # Llama-3-8B: 23.49k / 23.58k tok/s on vs 23.55k / 23.53k off (same box), +6.4 GiB, so it stays off.
        from ..ops._ext import use_native

        self.f8_pretransposed = (not self.sharded and os.environ.get("ACCELERATE_FP8_PRETRANSPOSE", "0") == "1"
                                 and all(use_native(u.shard_lp) for u in self.f8_units))
        for u in self.f8_units:
            for info in u.f8_infos:
                info.f8_t = (torch.empty((info.shape[1], info.shape[0]), dtype=torch.float8_e4m3fn, device=self.device)
                             if self.f8_pretransposed else None)
        self.refresh_fp8()

    def _init_expert_amax(self):
        """World size 1 (the shard is the whole stack): give every fp8 MoE expert stack [E, N, K] a per-expert amax
        that the fused AdamW max-reduces from the bf16 values it writes (one kernel row per expert), so the expert
        forward (models/moe.py `_expert_weight_fp8`) skips its amax pass over the stack."""
        self.expert_amax = []
        if self.sharded or self.offload or self.param_dtype != torch.bfloat16:
            return
        from ..models.moe import MoEExperts  # lazy: models import parallel.comm

        for unit in self.units:
            for info in unit.infos:
                m, sp = info.module, info.shard_param
                rec = getattr(m, "fp8_recipe", None)
                if (not isinstance(m, MoEExperts) or rec is None or getattr(rec, "mx", False) or len(info.shape) != 3
                        or sp is None or sp.numel() != info.numel or getattr(sp, "_acc_bf16_shadow", None) is None):
                    continue
                holder = _ExpertAmax(torch.zeros(info.shape[0], dtype=torch.float32, device=self.device),
                                     info.numel // info.shape[0])
                info.param._acc_fp8_expert_amax = holder
                sp._acc_fp8_amax_segs = holder
                self.expert_amax.append(holder)

    def fp8_amax_from_optimizer(self, unit: FlatUnit, updated_ids: set):
        """Called by the fused AdamW after it max-reduced |bf16(update)| into `unit.f8_amax` (zeroed first): the amax is
        current only if every fp8 weight of the unit was updated by that launch."""
        unit.f8_amax_fresh = updated_ids >= unit.f8_param_ids

    @torch.no_grad()
    def refresh_fp8(self, optimizer_amax: bool = False):
        """Re-quantise the fp8-gathered weights from the bf16 shards: per-weight amax of the local pieces, ONE
        all-reduce(MAX) over the shard group for every weight of the model (torchao's
        `precompute_float8_dynamic_scale_for_fsdp`, reference accelerator.py:2061-2066), then the per-weight scaled
        cast of each shard into its e4m3 all-gather source. Runs after every optimizer step."""
        if not optimizer_amax:
            for h in getattr(self, "expert_amax", ()):
                h.fresh = False  # weights changed by something other than the fused AdamW: recompute in forward
        if not self.f8_units:
            return
        from ..ops._ext import use_native

        for u in self.f8_units:
            fresh, u.f8_amax_fresh = u.f8_amax_fresh, False
            if optimizer_amax and fresh:
                continue  # the fused AdamW already reduced this unit's amax from the values it wrote
            lo, hi, max_len, _ = u.f8_seg
            src = u.shard_lp[: u.f8.shard_len]
            if use_native(src):
                ext().fp8_segment_amax(src, lo, hi, u.f8_amax, max_len)
            else:
                for k, info in enumerate(u.f8_infos):
                    piece = src[info.local_lo : info.local_hi]
                    u.f8_amax[k] = piece.abs().max().float() if piece.numel() else 0.0
        if self.sharded and self.world_size > 1:
            small_allreduce.all_reduce_(self.f8_amax_all, op=dist.ReduceOp.MAX, group=self.group)
        for u in self.f8_units:
            lo, hi, max_len, _ = u.f8_seg
            src = u.shard_lp[: u.f8.shard_len]
            if self.f8_pretransposed:
                for k, info in enumerate(u.f8_infos):
                    a, b = info.local_lo, info.local_hi
                    ext().fp8_cast_into(src[a:b].view(info.shape), u.f8_amax[k : k + 1], 448.0, True, False,
                                        u.f8_shard[a:b].view(info.shape), info.f8_t)
            elif use_native(src):
                ext().fp8_segment_cast(src, lo, hi, u.f8_amax, 448.0, u.f8_shard, max_len)
            else:
                for k, info in enumerate(u.f8_infos):
                    s = 448.0 / u.f8_amax[k].clamp_min(1e-12)
                    piece = (src[info.local_lo : info.local_hi].float() * s).clamp(-448.0, 448.0)
                    u.f8_shard[info.local_lo : info.local_hi] = piece.to(torch.float8_e4m3fn)

    def fp8_weight_t(self, unit: FlatUnit, info: _ParamInfo):
        """The stored K-major e4m3 copy of an fp8-gathered weight (world size 1), or None (made in backward)."""
        return info.f8_t

    def fp8_weight_scale(self, unit: FlatUnit, info: _ParamInfo) -> torch.Tensor:
        """The amax (fp32 [1], device) whose scale 448 / amax quantised this gathered weight."""
        return unit.f8_amax[info.f8_index - unit.f8_seg[3] : info.f8_index - unit.f8_seg[3] + 1]

    def _install_fused_wgrad(self):
        """Route the weight gradient of every plain `nn.Linear` whose weight this engine owns (and that no other module
        shares) through `_FusedWgradLinearFn`; Fp8Linear weights, MoE expert stacks and RMSNorm weights get a slot their
        own backward writes into."""
        from ..models.llama import RMSNorm  # lazy: models import parallel.comm
        from ..models.moe import MoEExperts
        refs = {}
        for m in self.model.modules():
            for p in m._parameters.values():
                if p is not None:
                    refs[id(p)] = refs.get(id(p), 0) + 1
        for unit in self.units:
            for info in unit.infos:
                m = info.module
                plain = type(m) is nn.Linear
                experts = isinstance(m, MoEExperts) and info.attr in ("w_gate_up", "w_down")
                norm = type(m) is RMSNorm and info.attr == "weight"
                # embeddings only where the slot is the fp32 grad shard (world size 1): the backward scatters the token
                # rows into it instead of a dense bf16 [V, H] gradient that is then added and converted
                emb = (type(m) is nn.Embedding and info.attr == "weight" and self._direct_grads() and m.padding_idx is None
                       and m.max_norm is None and not m.scale_grad_by_freq and not m.sparse)
                # parameters whose gradient a TP hook all-reduces (sequence-parallel norms, per-head q/k norms:
                # tensor_parallel.ReplicatedGradAllReduce) keep the autograd gradient: a slot would bypass the hook
                tp_hooked = getattr(m, "_tp_grad_allreduce_group", None) is not None or getattr(info.param, "_tp_grad_hooked", False)
                if (((plain or isinstance(m, Fp8Linear) or norm or emb) and info.attr == "weight") or experts) and info.param.requires_grad \
                        and refs.get(id(info.param), 0) == 1 and getattr(info.param, "_tp_spec", None) is None and not tp_hooked:
                    info.fused = True
                    info.param._acc_wgrad_slot = _WgradSlot(self, unit, info)
                    # Fp8Linear routes its fp8 weight-gradient GEMM to the slot itself (ops/fp8.py), MoEExperts its
                    # grouped weight-gradient GEMMs (models/moe.py), RMSNorm its dweight column sum (ops/fused.py; on a
                    # path without the HIP kernel the plain autograd gradient is absorbed into the slot instead)
                    if plain:
                        m.__class__ = _FusedWgradLinear
                    elif emb:
                        m.__class__ = _FusedSlotEmbedding

    def _replace_param(self, info: _ParamInfo, new: nn.Parameter):
        """Swap a (meta) Parameter object for `new` in every module that registers it (tied weights included)."""
        if not hasattr(self, "_holders"):
            self._holders = {}
            for m in self.model.modules():
                for attr, p in m._parameters.items():
                    if p is not None:
                        self._holders.setdefault(id(p), []).append((m, attr))
        old = info.param
        for tag in ("_tp_spec", "_ep_spec"):  # sharding metadata of TP / EP parameters survives materialisation
            if hasattr(old, tag):
                setattr(new, tag, getattr(old, tag))
        for m, attr in self._holders.get(id(old), []):
            m._parameters[attr] = new
        self._holders[id(new)] = self._holders.pop(id(old), [])
        info.orig_param = old
        info.param = new

    def _collect(self, module, prefix, owned, ignored):
        infos, offset = [], 0
        for name, p in module.named_parameters(recurse=True, remove_duplicate=True):
            if id(p) in owned or id(p) in ignored:
                continue
            owned.add(id(p))
            sub_name, _, attr = name.rpartition(".")
            sub = module.get_submodule(sub_name) if sub_name else module
            fqn = f"{prefix}.{name}" if prefix else name
            infos.append(_ParamInfo(fqn, sub, attr, p, offset))
            offset += p.numel()
        return infos

    @torch.no_grad()
    def _materialize(self, unit: FlatUnit, init_fn, seed):
        dev, W, r = self.device, self.world_size, self.rank
        full32 = torch.zeros(unit.padded, dtype=torch.float32, device=dev)
        on_meta = any(i.param.is_meta for i in unit.infos)
        # cpu_ram_efficient_loading (reference fsdp_utils.py:467-554,664-719): only rank 0 holds the real (pretrained)
        # weights — the other ranks built the model on the meta device — and rank 0's unit is broadcast over the
        # shard group straight into HBM, one unit at a time (one RCCL broadcast per block instead of one per tensor).
        R = self.replicate_size
        ram_efficient = bool(getattr(self.plugin, "cpu_ram_efficient_loading", False)) and (W > 1 or R > 1)
        holds_weights = (dist.get_rank() == 0) if dist.is_available() and dist.is_initialized() else True
        if ram_efficient and not holds_weights:
            for info in unit.infos:
                if info.param.is_meta:
                    view = full32[info.offset : info.offset + info.numel].view(info.shape)
                    self._replace_param(info, nn.Parameter(view, requires_grad=info.param.requires_grad))
        elif on_meta:
            # Materialise the whole unit on the GPU with a per-unit seed: every rank generates the identical unit
            # (deterministic regardless of world size) and keeps its slice.
            if init_fn is None:
                raise ValueError("Meta-device parameters need an `init_fn` (e.g. model.init_weights).")
            for info in unit.infos:
                view = full32[info.offset : info.offset + info.numel].view(info.shape)
                self._replace_param(info, nn.Parameter(view, requires_grad=info.param.requires_grad))
            gen_state = torch.cuda.get_rng_state(dev) if dev.type == "cuda" else torch.get_rng_state()
            torch.manual_seed(seed * 100003 + unit.idx)
            if dev.type == "cuda":
                torch.cuda.manual_seed(seed * 100003 + unit.idx)
            # init in module-registration order, not the (fp8-first) flat layout order: the values each module draws
            # from the seeded stream must not depend on the layout
            mods = {id(i.module): i.module for i in unit.infos}
            order = {id(m): k for k, m in enumerate(unit.module.modules())}
            for m in sorted(mods.values(), key=lambda m: order.get(id(m), -1)):
                init_fn(m)
            if dev.type == "cuda":
                torch.cuda.set_rng_state(gen_state, dev)
            else:
                torch.set_rng_state(gen_state)
        else:
            for info in unit.infos:
                full32[info.offset : info.offset + info.numel].copy_(info.param.detach().reshape(-1).to(dev, torch.float32))
        sync = ram_efficient or (self.plugin.sync_module_states and not on_meta)
        if W > 1 and sync:
            dist.broadcast(full32, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0, group=self.group)
        if R > 1 and sync:  # HSDP / NO_SHARD replicas: then from replica 0 to the same shard position of every replica
            dist.broadcast(full32, src=dist.get_global_rank(self.replicate_group, 0), group=self.replicate_group)
        local32 = unit.local_of_full(full32)  # this rank's slice of every region, concatenated
        if self.offload:
            unit.master = self._host(local32)
            unit.grad_shard = self._host(torch.zeros(unit.shard_numel, dtype=torch.float32))
            unit.shard_lp = local32.to(self.param_dtype, copy=True)  # HBM-resident all-gather source
            # what the host optimizer writes for upload (bf16), or None: upload the fp32 master and cast on the GPU
            unit.shadow_host = self._host(torch.empty(unit.shard_numel, dtype=self.param_dtype)) if self.param_dtype != torch.float32 else None
        else:
            unit.master = local32
            unit.grad_shard = torch.zeros_like(unit.master)
            unit.shard_lp = unit.master.to(self.param_dtype) if self.param_dtype != torch.float32 else unit.master
        unit.grad_valid = False
        del full32, local32
        if not self.sharded:
            # degenerate: no collective, the shard is the full buffer (its bf16 regions start at bf_base)
            unit.full = unit.shard_lp[unit.bf_base :]
        else:
            unit.full = torch.empty(unit.padded - unit.bf_base, dtype=self.param_dtype, device=dev)
        if unit.f8 is not None:
            unit.f8_shard = torch.zeros(unit.f8.shard_len, dtype=torch.float8_e4m3fn, device=dev)
            unit.f8_full = unit.f8_shard if not self.sharded else torch.zeros(unit.f8.length, dtype=torch.float8_e4m3fn, device=dev)
        # Point every original parameter at its slice of the full buffer (views survive storage resizes): fp8
        # all-gathered weights at their e4m3 copy, everything else at the compute-dtype buffer.
        for info in unit.infos:
            info.param.data = self._full_view(unit, info)
            # per-parameter views of the local shard, exposed to the optimizer
            info.local_lo, info.local_hi, info.param_lo = unit.local_range(info)
            sp = nn.Parameter(unit.master[info.local_lo : info.local_hi], requires_grad=info.param.requires_grad)
            if self.offload:
                sp._acc_offloaded = True
                if unit.shadow_host is not None:
                    sp._acc_bf16_shadow_host = unit.shadow_host[info.local_lo : info.local_hi]
            elif self.param_dtype != torch.float32:
                sp._acc_bf16_shadow = unit.shard_lp[info.local_lo : info.local_hi]
            sp._acc_fsdp_fqn = info.fqn
            sp._acc_fsdp_full_shape = info.shape
            sp._acc_fsdp_param_lo = info.param_lo
            info.shard_param = sp
        if self.sharded:
            unit.state = "unsharded"
            self._free_full(unit)
        else:
            unit.state = "unsharded"

    def _full_view(self, unit: FlatUnit, info: _ParamInfo) -> torch.Tensor:
        if unit.f8 is not None and info.region is unit.f8:
            return unit.f8_full[info.offset : info.offset + info.numel].view(info.shape)
        o = info.offset - unit.bf_base
        return unit.full[o : o + info.numel].view(info.shape)

    def _bf_regions(self, unit: FlatUnit):
        return [reg for reg in unit.regions if not reg.fp8]

    def gather_full(self, unit: FlatUnit, local: torch.Tensor) -> torch.Tensor:
        """A full-layout tensor assembled from every rank's shard-layout `local` (one all-gather per region)."""
        if not self.sharded:
            return local
        full = torch.empty(unit.padded, dtype=local.dtype, device=local.device)
        for reg in unit.regions:
            dst, src = full[reg.base : reg.base + reg.length], local[reg.shard_base : reg.shard_base + reg.shard_len]
            if self._uses_gloo and self._gloo():
                dist.all_gather(list(dst.chunk(self.world_size)), src, group=self.group)
            else:
                dist.all_gather_into_tensor(dst, src, group=self.group)
        return full

    def _host(self, t: torch.Tensor) -> torch.Tensor:
        """A host copy of `t` (pinned when offloading to a GPU run, so D2H/H2D are true async DMA)."""
        h = t.detach().to("cpu", copy=True)
        return h.pin_memory() if self._pin else h

    # =========================================================================================== storage
    def _free_full(self, unit: FlatUnit):
        if not self.sharded or unit.state == "sharded":
            return
        unit.full.untyped_storage().resize_(0)
        if unit.f8 is not None:
            unit.f8_full.untyped_storage().resize_(0)
        unit.state = "sharded"
        unit.ag_event = None

    def _unshard(self, unit: FlatUnit):
        """Issue the all-gather of `unit` on the AG stream (no host wait). Idempotent."""
        if not self.sharded or unit.state != "sharded":
            return
        unit.full.untyped_storage().resize_(unit.full.numel() * unit.full.element_size())
        if unit.f8 is not None:
            unit.f8_full.untyped_storage().resize_(unit.f8_full.numel())
        if self.is_cuda:
            cur = torch.cuda.current_stream(self.device)
            self.ag_stream.wait_stream(cur)
            record_collective("fsdp_all_gather", unit.shard_lp, self.group)
            with torch.cuda.stream(self.ag_stream), trace_range(f"fsdp.all_gather[{unit.idx}]"):
                self._all_gather_unit(unit, self.ag_group)
                ev = torch.cuda.Event()
                ev.record(self.ag_stream)
            unit.ag_event = ev
        else:
            self._all_gather_unit(unit, self.group)
            unit.ag_event = None
        unit.state = "unsharding"

    def _all_gather_unit(self, unit: FlatUnit, group):
        """bf16 regions into `unit.full`; the fp8 region (e4m3 bytes, half the traffic) into `unit.f8_full`."""
        gloo = self._uses_gloo and self._gloo()
        pairs = [(unit.full[reg.base - unit.bf_base : reg.base - unit.bf_base + reg.length],
                  unit.shard_lp[reg.shard_base : reg.shard_base + reg.shard_len]) for reg in self._bf_regions(unit)]
        if unit.f8 is not None:
            pairs.append((unit.f8_full.view(torch.uint8), unit.f8_shard.view(torch.uint8)))
        for dst, src in pairs:
            if gloo:
                dist.all_gather(list(dst.chunk(self.world_size)), src, group=group)
            else:
                dist.all_gather_into_tensor(dst, src, group=group)

    def _gloo(self):
        return dist.get_backend(self.group) == "gloo"

    def _wait_unsharded(self, unit: FlatUnit):
        if unit.state == "sharded":
            self._unshard(unit)
        if unit.state == "unsharding":
            if unit.ag_event is not None:
                torch.cuda.current_stream(self.device).wait_event(unit.ag_event)
            unit.state = "unsharded"

    # =========================================================================================== hooks
    def _in_backward(self):
        return torch._C._current_graph_task_id() != -1

    def _make_pre_forward(self, unit: FlatUnit):
        def hook(module, args, kwargs):
            self._wait_unsharded(unit)
            if self._in_backward():
                return None  # activation-checkpoint recompute: params are already gathered for backward
            if self._recording_order:
                if unit not in self.exec_order:
                    self.exec_order.append(unit)
            else:
                self._prefetch_forward(unit)
            return None

        return hook

    def _prefetch_forward(self, unit):
        if not self.sharded or self.fwd_prefetch_depth == 0:
            return
        try:
            i = self.exec_order.index(unit)
        except ValueError:
            return
        for nxt in self.exec_order[i + 1 : i + 1 + self.fwd_prefetch_depth]:
            self._unshard(nxt)

    def _make_post_forward(self, unit: FlatUnit):
        def hook(module, args, kwargs, output):
            if self._in_backward():
                return output
            if torch.is_grad_enabled():
                self._register_pre_backward(unit, output)
            if self.reshard_after_forward:
                self._free_full(unit)
            return output

        return hook

    def _register_pre_backward(self, unit, output):
        tensors = [t for t in _flatten_tensors(output) if t.requires_grad]
        if not tensors:
            return
        unit.bwd_prefetched = False

        def pre_backward(grad):
            if not unit.in_backward:
                unit.in_backward = True
                self._queue_final_callback()
                self._wait_unsharded(unit)
                if self.bwd_prefetch == "BACKWARD_PRE":
                    self._prefetch_backward(unit)
                self._prepare_grad_buffer(unit)
            return grad

        for t in tensors:
            t.register_hook(pre_backward)

    def _prefetch_backward(self, unit):
        if not self.sharded or self.prefetch_depth == 0:
            return
        try:
            i = self.exec_order.index(unit)
        except ValueError:
            return
        for j in range(i - 1, max(-1, i - 1 - self.prefetch_depth), -1):
            self._unshard(self.exec_order[j])

    def _queue_final_callback(self):
        if not self._final_cb_queued:
            self._final_cb_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)

    def _prepare_grad_buffer(self, unit: FlatUnit):
        """Point every param's `.grad` at its slice of a zeroed flat grad buffer (accumulated in place)."""
        if unit.full_grad is None:
            unit.full_grad = self._new_grad_buffer(unit)
            for info in unit.infos:
                if info.param.requires_grad and not info.fused:
                    info.param.grad = unit.full_grad[info.offset : info.offset + info.numel].view(info.shape)
        unit.pending_grads = sum(1 for i in unit.infos if i.param.requires_grad)
        unit.reduced = False

    def _new_grad_buffer(self, unit: FlatUnit):
        """Flat grad buffer; only the slots that are accumulated into (non-fused params, padding) are zeroed — a
        fused slot is overwritten by its first weight-gradient GEMM.

        The buffer is allocated once per unit and reused every backward (it is free again once the compute stream
        has waited for the reduce-scatter stream at the end of backward). A fresh buffer per backward, released with
        reduce-scatter stream uses recorded on it, cannot be recycled by the caching allocator until the GPU catches
        up with the host, which runs a step ahead: on Llama-3-8B at one forced-sharded GPU the reserved pool reached
        285 of 288 GiB, the allocator fell back to freeing its cache (hipFree + sync) and the step took 1.3 s instead
        of 0.46 s. Without sharding (world size 1 shortcut: fused weight grads go to the fp32 shard, this buffer only
        carries the few non-fused slots and is never handed to another stream) it stays transient: keeping 32 of them
        would hold 14 GB of Llama-3-8B for nothing."""
        buf = getattr(unit, "_grad_buf", None)
        if buf is not None and self.is_cuda and getattr(unit, "_rs_done", None) is not None:
            # reused: writes on the compute stream must follow the last reduce-scatter that read it (normally long
            # done; this only matters if the unit is re-gradded within the backward that reduced it)
            torch.cuda.current_stream(self.device).wait_event(unit._rs_done)
        if buf is None or buf.numel() != unit.padded or buf.dtype != self.param_dtype:
            buf = torch.empty(unit.padded, dtype=self.param_dtype, device=self.device)
            if self.sharded:
                unit._grad_buf = buf
        if not any(i.fused for i in unit.infos):
            return buf.zero_()
        pos = 0
        for info in sorted(unit.infos, key=lambda i: i.offset):
            if info.fused:
                if info.offset > pos:
                    buf[pos : info.offset].zero_()
                pos = info.offset + info.numel
                info.fused_written = False
        if pos < unit.padded:
            buf[pos:].zero_()
        return buf

    def _direct_grads(self):
        """World size 1 (no replicas): fused weight grads go straight to the fp32 grad shard (the GEMM writes fp32)."""
        return not self.sharded and not self.offload and self.replicate_size == 1 and os.environ.get("ACCELERATE_FSDP_WGRAD_FP32", "1") != "0"

    def _fused_dest(self, unit, info):
        """(destination view, accumulate?) for a fused weight gradient."""
        if self._direct_grads():
            # torch semantics: accumulate unless the grad was set to None (zero_grad). The grad is exposed at once, so a
            # second use in this pass or the next no_sync micro-batch accumulates.
            sp = info.shard_param
            flat = unit.grad_shard[info.local_lo : info.local_hi]
            acc = sp.grad is not None
            sp.grad = flat
            info.fused_written = True
            return flat.view(info.shape), acc
        if unit.full_grad is None:
            self._prepare_grad_buffer(unit)
        dest = unit.full_grad[info.offset : info.offset + info.numel].view(info.shape)
        acc = info.fused_written
        info.fused_written = True
        return dest, acc

    def _fused_slot_dest(self, slot: "_WgradSlot"):
        """(destination view, accumulate?) for a weight-gradient GEMM that writes its result in place (the bf16 path
        below, and the fp8 GEMM of ops/fp8.py)."""
        unit = slot.unit
        if unit.full_grad is None:
            self._prepare_grad_buffer(unit)
        return self._fused_dest(unit, slot.info)

    def _fused_slot_done(self, slot: "_WgradSlot"):
        """The slot's gradient for this backward is written: counts as the parameter's grad-ready event."""
        unit = slot.unit
        slot.uses -= 1
        if slot.uses <= 0:
            slot.uses = 0
            unit.pending_grads -= 1
            if unit.pending_grads == 0 and self.requires_grad_sync:
                self._reduce_unit(unit)

    def _fused_wgrad(self, slot: "_WgradSlot", dy2: torch.Tensor, x2: torch.Tensor):
        """dW = dy2ᵀ · x2 written into the unit's flat grad buffer (or fp32 grad shard at world size 1); counts as the
        parameter's grad-ready event."""
        dest, acc = self._fused_slot_dest(slot)
        wgrad_into(dest, dy2, x2, acc)
        self._fused_slot_done(slot)

    def _make_grad_hook(self, unit: FlatUnit):
        # The hook lives in the parameter's C++ autograd metadata, which the Python cycle collector cannot traverse:
        # a strong reference to the engine here would keep every shard, optimizer-visible master and buffer of the
        # model alive after the user drops it (measured: 33 GiB of an 8-layer Llama-3-8B-width model). It therefore
        # holds the engine weakly and finds the unit by index.
        eng_ref, idx = weakref.ref(self), unit.idx

        def hook(param):
            eng = eng_ref()
            if eng is not None:
                eng._on_grad_ready(eng.units[idx], param)

        return hook

    def _on_grad_ready(self, unit: FlatUnit, param):
        if param.grad is None and getattr(param, "_acc_wgrad_slot", None) is not None:
            return  # fused weight: its Linear backward already wrote the slot and counted it
        if unit.full_grad is None or param.grad is None or param.grad.data_ptr() != self._grad_slot_ptr(unit, param):
            self._absorb_foreign_grad(unit, param)
        unit.pending_grads -= 1
        if unit.pending_grads == 0 and self.requires_grad_sync:
            self._reduce_unit(unit)

    def _grad_slot_ptr(self, unit, param):
        for info in unit.infos:
            if info.param is param:
                return unit.full_grad[info.offset : info.offset + info.numel].data_ptr()
        return -1

    def _absorb_foreign_grad(self, unit, param):
        """A grad not living in our flat buffer (first use before a pre-backward hook, e.g. root params):
        copy/accumulate it into the flat buffer and re-point `.grad`."""
        if unit.full_grad is None:
            unit.full_grad = self._new_grad_buffer(unit)
            unit.pending_grads = sum(1 for i in unit.infos if i.param.requires_grad)
            for info in unit.infos:
                if info.param.requires_grad and not info.fused and info.param is not param and info.param.grad is None:
                    info.param.grad = unit.full_grad[info.offset : info.offset + info.numel].view(info.shape)
        for info in unit.infos:
            if info.param is param:
                view = unit.full_grad[info.offset : info.offset + info.numel].view(info.shape)
                if info.fused:  # fused weight that took the plain autograd path (autocast / dtype mismatch)
                    if param.grad is not None:
                        dest, acc = self._fused_dest(unit, info)
                        dest.add_(param.grad.to(dest.dtype)) if acc else dest.copy_(param.grad)
                    param.grad = None
                    return
                if param.grad is not None and param.grad.data_ptr() != view.data_ptr():
                    view.add_(param.grad.to(view.dtype))
                param.grad = view
                return

    # =========================================================================================== reduction
    @torch.no_grad()
    def _reduce_unit(self, unit: FlatUnit):
        if unit.reduced or unit.full_grad is None:
            return
        unit.reduced = True
        W = self.world_size
        self._zero_unwritten_fused(unit)
        # torch semantics: grads accumulate until the optimizer (or user) sets them to None.
        first = (not unit.grad_valid) or all(i.shard_param.grad is None for i in unit.infos if i.shard_param.requires_grad)
        if not self.sharded and self.replicate_size == 1:
            if any(i.fused for i in unit.infos) and self._direct_grads():
                for info in unit.infos:  # fused weights are already in the fp32 shard
                    if info.fused or not info.param.requires_grad:
                        continue
                    g = unit.full_grad[info.offset : info.offset + info.numel]
                    d = unit.grad_shard[info.local_lo : info.local_hi]
                    d.copy_(g) if info.shard_param.grad is None else d.add_(g)
            else:
                self._deliver_grad(unit, unit.full_grad[: unit.shard_numel], 1.0, first)
            unit.grad_valid = True
            self._release_grad(unit)
            self._expose_unit_grads(unit)
            self._overlap_step(unit, torch.cuda.current_stream(self.device) if self.is_cuda else None)
            return
        src = unit.full_grad if unit.full_grad.dtype == self.reduce_dtype else unit.full_grad.to(self.reduce_dtype)
        out = self._reduce_out(unit)
        if self.is_cuda:
            cur = torch.cuda.current_stream(self.device)
            self.rs_stream.wait_stream(cur)
            with torch.cuda.stream(self.rs_stream), trace_range(f"fsdp.reduce_scatter[{unit.idx}]"):
                self._rs_and_accumulate(unit, src, out, first)
                unit._rs_done = torch.cuda.Event()
                unit._rs_done.record(self.rs_stream)
            if src is not unit.full_grad:
                src.record_stream(self.rs_stream)
        else:
            self._rs_and_accumulate(unit, src, out, first)
        unit.grad_valid = True
        self._release_grad(unit)
        self._expose_unit_grads(unit)
        self._overlap_step(unit, self.rs_stream)
        if not unit.is_root and self.sharded:
            self._free_full(unit)  # block done with backward: drop its gathered params
        if self.bwd_prefetch == "BACKWARD_POST" and unit.in_backward:
            self._prefetch_backward(unit)

    def _reduce_out(self, unit: FlatUnit) -> torch.Tensor:
        """The reduce-scatter output for `unit`: a view of ONE persistent engine-wide buffer (the largest shard). Every
        reduce-scatter and the grad-shard update that consumes its output run in order on the reduce stream, so unit
        i+1's reduce-scatter starts after unit i's update has read the buffer. A fresh buffer per unit per step would
        be released with reduce-stream uses recorded on it while the host runs a step ahead of the GPU, which is how
        the caching allocator piled up blocks before (round-2 forced-sharded blow-up to 285 of 288 GiB)."""
        buf = getattr(self, "_rs_out_buf", None)
        if buf is None or buf.dtype != self.reduce_dtype or buf.numel() < unit.shard_numel:
            n = max(u.shard_numel for u in self.units)
            buf = self._rs_out_buf = torch.empty(n, dtype=self.reduce_dtype, device=self.device)
        return buf[: unit.shard_numel]

    def _zero_unwritten_fused(self, unit: FlatUnit):
        """A fused weight whose Linear did not run in this backward (a skipped branch, an unused head) never wrote its
        gradient slot, which `_new_grad_buffer` leaves unzeroed (and, at world size 1, the fp32 grad shard still holds
        the previous step's gradient): zero it so the reduction never carries a stale gradient."""
        direct = self._direct_grads()
        for info in unit.infos:
            if not (info.fused and info.param.requires_grad) or info.fused_written:
                continue
            if direct:
                if info.shard_param.grad is None:  # accumulating micro-batches keep their sum
                    unit.grad_shard[info.local_lo : info.local_hi].zero_()
            elif unit.full_grad is not None:
                unit.full_grad[info.offset : info.offset + info.numel].zero_()

    # =========================================================================================== optimizer overlap
    def attach_overlapped_optimizer(self, step_fn: Callable[[list], None]):
        """Overlap the optimizer with the backward (`RcclKwargs.fsdp_optimizer_overlap`): `step_fn(shard_params)`
        updates the given shard parameters and is called for each unit as soon as its gradient shard is final — on a
        side HIP stream ordered after the stream that produced the gradient (reduce-scatter stream, or the compute
        stream at world size 1). The update is memory-bound (fp32 master, grad, Adam moments, bf16 shadow) and the
        backward GEMM/attention kernels are compute-bound, so the two share the CUs. A unit's weights are not read
        again in this backward once its gradient is final, and the next all-gather / forward runs after
        `take_overlapped()` has ordered the compute stream behind the side stream."""
        if self.offload:
            raise ValueError("fsdp_optimizer_overlap cannot be combined with FSDP CPU offload (the step runs on the host).")
        self._overlap_fn = step_fn
        self._overlap_done: set[int] = set()
        if self.is_cuda and getattr(self, "opt_stream", None) is None:
            self.opt_stream = torch.cuda.Stream(device=self.device)

    def _overlap_step(self, unit: FlatUnit, src_stream):
        fn = getattr(self, "_overlap_fn", None)
        if fn is None or not self.requires_grad_sync:
            return
        params = [i.shard_param for i in unit.infos if i.shard_param.requires_grad and i.shard_param.grad is not None
                  and id(i.shard_param) not in self._overlap_done]
        if not params:
            return
        if self.is_cuda:
            self.opt_stream.wait_stream(src_stream)
            with torch.cuda.stream(self.opt_stream), trace_range(f"fsdp.optimizer_overlap[{unit.idx}]"):
                fn(params)
        else:
            fn(params)
        self._overlap_done.update(id(p) for p in params)

    def take_overlapped(self) -> set:
        """ids of the shard params already updated during this backward; orders the current stream after them."""
        done = getattr(self, "_overlap_done", None)
        if not done:
            return set()
        self._overlap_done = set()
        if self.is_cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.opt_stream)
        return done

    def _rs_and_accumulate(self, unit, src, out, first):
        W = self.world_size
        if self.sharded:
            record_collective("fsdp_reduce_scatter", src, self.group)
            for reg in unit.regions:  # one reduce-scatter per region (a single one in the plain layout)
                o = out[reg.shard_base : reg.shard_base + reg.shard_len]
                i = src[reg.base : reg.base + reg.length]
                if self._uses_gloo and self._gloo():
                    self._gloo_rs(o, i)
                else:
                    dist.reduce_scatter_tensor(o, i, group=self.rs_group)
        else:
            out.copy_(src[: unit.shard_numel])
        if self.replicate_group is not None and self.replicate_size > 1:
            dist.all_reduce(out, group=self.replicate_group)
        scale = 1.0 / (W * self.replicate_size)
        self._deliver_grad(unit, out, scale, first)

    def _deliver_grad(self, unit, src, scale, first):
        """grad shard (=|+=) scale * src. Offloaded: scale into a transient fp32 HBM buffer, then DMA it to the pinned
        host shard (or a staging buffer that the host adds at the end of backward when accumulating)."""
        if not (self.offload and self.is_cuda):
            _grad_update(unit.grad_shard, src, scale, accumulate=not first)
            return
        g32 = torch.empty(unit.shard_numel, dtype=torch.float32, device=self.device)
        _grad_update(g32, src, scale, accumulate=False)
        stage = unit.grad_shard if first else torch.empty(unit.shard_numel, dtype=torch.float32, pin_memory=self._pin)
        stage.copy_(g32, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._d2h_pending.append((ev, unit, None if first else stage, g32))

    def _drain_d2h(self):
        for ev, unit, stage, _ in self._d2h_pending:
            ev.synchronize()
            if stage is not None:
                unit.grad_shard.add_(stage)
        self._d2h_pending.clear()

    def _gloo_rs(self, out, src):
        # HIP tensors on a gloo group (one-GPU rehearsal): all-reduce then slice
        tmp = src.clone()
        dist.all_reduce(tmp, group=self.group)
        out.copy_(tmp[self.rank * out.numel() : (self.rank + 1) * out.numel()])

    def _release_grad(self, unit):
        for info in unit.infos:
            info.param.grad = None
        unit.full_grad = None

    def _finalize_backward(self):
        """End of backward: flush units whose hooks did not all fire, order the compute stream after the reduce
        stream, reshard, and expose the fp32 grad shards to the optimizer."""
        self._final_cb_queued = False
        if self._recording_order:
            self._recording_order = False
        for unit in self.units:
            unit.in_backward = False
            for info in unit.infos:
                if info.fused:
                    info.param._acc_wgrad_slot.uses = 0  # forwards whose outputs never reached this backward
            if self.requires_grad_sync and unit.full_grad is not None and not unit.reduced:
                self._reduce_unit(unit)
        if self.is_cuda and (self.sharded or self.replicate_size > 1):
            torch.cuda.current_stream(self.device).wait_stream(self.rs_stream)
        if self._d2h_pending:
            self._drain_d2h()  # offload: the host optimizer reads the gradient shards next
        for unit in self.units:
            if self.reshard_after_forward or not unit.is_root:
                if self.sharded and self.reshard_after_forward:
                    self._free_full(unit)
        if self.requires_grad_sync:
            self._expose_grads()

    def _expose_grads(self):
        for unit in self.units:
            self._expose_unit_grads(unit)

    def _expose_unit_grads(self, unit):
        if not unit.grad_valid:
            return
        for info in unit.infos:
            sp = info.shard_param
            if sp.requires_grad:
                sp.grad = unit.grad_shard[info.local_lo : info.local_hi]

    # =========================================================================================== public API
    def shard_parameters(self):
        for unit in self.units:
            for info in unit.infos:
                yield info.shard_param
        for _, p in self._extras():
            yield p

    def named_shard_parameters(self):
        for unit in self.units:
            for info in unit.infos:
                yield info.fqn, info.shard_param
        yield from self._extras()

    def param_map(self) -> dict:
        """original nn.Parameter -> shard nn.Parameter (used to remap optimizers created before prepare)."""
        return {info.orig_param: info.shard_param for unit in self.units for info in unit.infos}

    def pre_root_forward(self):
        """Called by the wrapper before the model's forward: gather the root unit (+ prefetch the first block)."""
        self._wait_unsharded(self.root)
        if not self._recording_order and self.exec_order:
            for u in self.exec_order[: self.fwd_prefetch_depth]:
                self._unshard(u)

    def post_root_forward(self, output):
        if self.exec_order:
            self._recording_order = False
        if torch.is_grad_enabled():
            tensors = [t for t in _flatten_tensors(output) if t.requires_grad]

            def hook(grad):
                self._queue_final_callback()
                if self.root.full_grad is None:
                    self._prepare_grad_buffer(self.root)
                return grad

            for t in tensors:
                t.register_hook(hook)
        return output

    def on_zero_grad(self):
        for unit in self.units:
            if all(info.shard_param.grad is None for info in unit.infos):
                unit.grad_valid = False

    @torch.no_grad()
    def on_optimizer_step(self, fused_wrote_shadow: bool):
        """Refresh the bf16 all-gather source from the fp32 master when the optimizer did not write it, and drop any
        gathered copies (they are stale now; the next forward re-gathers)."""
        if self.offload:
            for unit in self.units:  # upload the updated shard into the HBM all-gather source
                if fused_wrote_shadow and unit.shadow_host is not None:
                    unit.shard_lp.copy_(unit.shadow_host, non_blocking=True)
                else:
                    unit.shard_lp.copy_(unit.master.to(unit.shard_lp.device, non_blocking=True))
        elif self.param_dtype != torch.float32 and not fused_wrote_shadow:
            for unit in self.units:
                unit.shard_lp.copy_(unit.master)
        # the bf16 shards are current: re-quantise the fp8 all-gather sources (amax from the fused AdamW when it wrote them)
        self.refresh_fp8(optimizer_amax=fused_wrote_shadow and not self.offload)
        if self.sharded:
            for unit in self.units:
                if unit.state == "unsharding" and unit.ag_event is not None and self.is_cuda:
                    torch.cuda.current_stream(self.device).wait_event(unit.ag_event)
                unit.state = "unsharded" if unit.state == "unsharding" else unit.state
                self._free_full(unit)

    def set_requires_gradient_sync(self, flag: bool):
        self.requires_grad_sync = flag

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float, norm_type: float = 2.0) -> torch.Tensor:
        """Global gradient norm over all shards (HIP multi-tensor sum of squares + one all-reduce), then device-side
        scaling. Returns the total norm (device tensor, no host sync)."""
        from ..ops.multi_tensor import clip_grads_by_total_sq, grad_sq_norm

        if norm_type != 2.0:
            raise NotImplementedError("Only the L2 norm is supported by the FSDP engine.")
        if getattr(self, "_overlap_done", None):
            raise RuntimeError(
                "clip_grad_norm_ needs every gradient before any update, but `fsdp_optimizer_overlap` already applied the "
                "optimizer to some units during backward. Disable RcclKwargs(fsdp_optimizer_overlap) to clip gradients."
            )
        flat_params = []
        for unit in self.units:
            if unit.grad_valid:
                holder = _GradHolder(unit.grad_shard)
                flat_params.append(holder)
        total = torch.zeros(1, dtype=torch.float32, device=self.device)
        tp_group, tp = self._tp_group()
        if tp > 1:
            # 2-D FSDP x TP: a TP-sharded parameter's shard holds a disjoint 1/tp of its gradient on each tp rank (its
            # squares are summed over tp as well as dp_shard), a TP-replicated one the same values on every tp rank
            # (pre-divided by tp so the tp all-reduce counts it once). Reference: DTensor-aware clip_grad_norm_ over
            # the whole mesh, /root/reference/src/accelerate/accelerator.py:2943-2953.
            shard_pieces, rep_pieces = [], []
            for unit in self.units:
                if not unit.grad_valid:
                    continue
                for info in unit.infos:
                    if info.local_hi <= info.local_lo:
                        continue
                    piece = _GradHolder(unit.grad_shard[info.local_lo : info.local_hi])
                    spec = getattr(info.param, "_tp_spec", None)
                    (shard_pieces if spec is not None and spec.size > 1 else rep_pieces).append(piece)
            if shard_pieces:
                grad_sq_norm(shard_pieces, out=total)
            if rep_pieces:
                rep = grad_sq_norm(rep_pieces).to(total.device)
                total += rep / tp
        elif flat_params:
            grad_sq_norm(flat_params, out=total)
        # non-engine params: expert-parallel shards are disjoint across the group (summed by the all-reduce);
        # replicated ones are pre-divided by W (and by tp under a tp all-reduce) so the all-reduces count them once
        extra = [p for p in getattr(self, "extra_params", []) if p.grad is not None]
        for p in extra:
            sq = p.grad.detach().float().pow(2).sum()
            if getattr(getattr(p, "_tp_spec", None), "size", 1) > 1:
                total += sq / self.world_size
            else:
                total += (sq if getattr(p, "_ep_spec", None) is not None else sq / self.world_size) / tp
        if self.sharded:
            small_allreduce.all_reduce_(total, group=self.group)  # 4 bytes: IPC one-shot kernel, not an RCCL ring
        if tp > 1:
            torch.distributed.all_reduce(total, group=tp_group)
        clip_grads_by_total_sq(flat_params + extra, total, max_norm)
        return total.sqrt().reshape(())

    def _tp_group(self):
        """(tp process group, tp size) of the tensor-parallel parameters this engine shards; (None, 1) without TP."""
        if not hasattr(self, "_tp_cache"):
            self._tp_cache = (None, 1)
            params = [info.param for unit in self.units for info in unit.infos]
            params += list(getattr(self, "extra_params", []))
            for p in params:
                spec = getattr(p, "_tp_spec", None)
                if spec is not None and spec.size > 1:
                    self._tp_cache = (spec.group, spec.size)
                    break
        return self._tp_cache

    # --- state dicts --------------------------------------------------------------------------------------
    @torch.no_grad()
    def full_state_dict(self, rank0_only: bool = True, cpu: bool = True, dtype=None) -> dict:
        """Gather the fp32 master weights unit by unit (one all-gather per unit) → {fqn: full tensor}."""
        out = OrderedDict()
        for unit in self.units:
            master = unit.master.to(self.device) if self.offload else unit.master
            full = self.gather_full(unit, master)
            if rank0_only and self.rank != 0:
                continue
            for info in unit.infos:
                t = full[info.offset : info.offset + info.numel].view(info.shape)
                if dtype is not None:
                    t = t.to(dtype)
                out[info.fqn] = t.cpu().clone() if cpu else t.clone()
        for name, p in self._extras():
            t = self._gather_ep(p) if getattr(p, "_ep_spec", None) is not None else p.detach().float()
            if rank0_only and self.rank != 0:
                continue
            t = t.to(dtype) if dtype is not None else t
            out[name] = t.cpu().clone() if cpu else t.clone()
        return out

    def sharded_state_dict(self, to_cpu: bool = True) -> dict:
        """This rank's master shards: {fqn: local 1-D slice} plus layout metadata for resharding. `to_cpu=False`
        returns device views of the live shards (the non-blocking writer snapshots them on the device)."""
        tensors, meta = OrderedDict(), {"world_size": self.world_size, "rank": self.rank, "params": {}, "extra": {}}
        for unit in self.units:
            for info in unit.infos:
                piece = unit.master[info.local_lo : info.local_hi].detach()
                tensors[info.fqn] = piece.cpu().clone() if to_cpu else piece
                meta["params"][info.fqn] = {"shape": list(info.shape), "param_lo": info.param_lo, "numel": info.local_hi - info.local_lo}
                spec = getattr(info.param, "_tp_spec", None)
                if spec is not None and spec.size > 1:  # TP-local shape: how merge_fsdp_weights reassembles the full one
                    meta["params"][info.fqn]["tp"] = {"dim": spec.dim, "segments": list(spec.segments) if spec.segments else None}
        for name, p in self._extras():
            tensors[name] = p.detach().float().cpu().clone() if to_cpu else p.detach().float()
            meta["extra"][name] = {"ep": getattr(p, "_ep_spec", None) is not None, "rank": self.rank}
        return {"tensors": tensors, "meta": meta}

    # --- non-engine (ignored / expert-parallel) parameters -------------------------------------------------
    def _extras(self):
        for name in getattr(self, "extra_names", []):
            yield name, self.model.get_parameter(name)

    def _gather_ep(self, p):
        group, W = p._ep_spec
        t = p.detach().float().contiguous()
        out = torch.empty((W * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        if t.is_cuda and dist.get_backend(group) == "gloo":
            dist.all_gather(list(out.chunk(W)), t, group=group)
        else:
            dist.all_gather_into_tensor(out, t, group=group)
        return out

    @torch.no_grad()
    def _load_extra(self, name, full):
        p = self.model.get_parameter(name)
        spec = getattr(p, "_ep_spec", None)
        if spec is not None:
            group, W = spec
            n = full.shape[0] // W
            r = dist.get_rank(group)
            full = full[r * n : (r + 1) * n]
        p.copy_(full.to(p.device, p.dtype))

    @torch.no_grad()
    def load_full_state_dict(self, sd: dict, strict: bool = True):
        missing = []
        for unit in self.units:
            for info in unit.infos:
                if info.fqn not in sd:
                    missing.append(info.fqn)
                    continue
                full = sd[info.fqn].reshape(-1)
                piece = full[info.param_lo : info.param_lo + (info.local_hi - info.local_lo)]
                unit.master[info.local_lo : info.local_hi].copy_(piece.to(unit.master.device, torch.float32))
            if unit.shard_lp is not unit.master:
                unit.shard_lp.copy_(unit.master.to(unit.shard_lp.device))
        self.refresh_fp8()
        for name, _ in self._extras():
            if name in sd:
                self._load_extra(name, sd[name])
            else:
                missing.append(name)
        if strict and missing:
            raise KeyError(f"Missing keys in state dict: {missing[:5]}...")
        return missing

    @torch.no_grad()
    def broadcast_full(self, full: torch.Tensor):
        """Broadcast a full-layout unit buffer from global rank 0: over the shard group, then from replica 0 over the
        replicate group (HSDP), as `_materialize` does for cpu_ram_efficient_loading."""
        if self.world_size > 1:
            dist.broadcast(full, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0, group=self.group)
        if self.replicate_size > 1:
            dist.broadcast(full, src=dist.get_global_rank(self.replicate_group, 0), group=self.replicate_group)

    @torch.no_grad()
    def load_full_state_dict_broadcast(self, sd: Optional[dict], strict: bool = True):
        """FULL_STATE_DICT load where only global rank 0 holds `sd` (None elsewhere): one broadcast of each unit's
        flat fp32 buffer, every rank keeps its slice (reference fsdp2_load_full_state_dict,
        /root/reference/src/accelerate/utils/fsdp_utils.py:467-554). Host memory: rank 0 maps the file, the others
        hold nothing.

        Keys: rank 0 lists the parameters `sd` lacks and broadcasts the list before anything is copied; with `strict`
        every rank raises KeyError (as `load_full_state_dict`), otherwise the missing parameters keep their current
        values on every rank (nothing is overwritten with a placeholder)."""
        from ..utils.fsdp_utils import IO_STATS

        multi = dist.is_available() and dist.is_initialized()
        missing = None
        if sd is not None:
            missing = [info.fqn for unit in self.units for info in unit.infos if info.fqn not in sd]
            missing += [name for name, _ in self._extras() if name not in sd]
        if multi:
            box = [missing]
            dist.broadcast_object_list(box, src=0)
            missing = box[0]
        if missing is None:
            raise ValueError("load_full_state_dict_broadcast: global rank 0 must hold the state dict")
        if strict and missing:
            raise KeyError(f"Missing keys in state dict: {missing[:5]}...")
        skip = set(missing)
        for unit in self.units:
            full = torch.zeros(unit.padded, dtype=torch.float32, device=self.device)
            if sd is not None:
                for info in unit.infos:
                    if info.fqn in skip:
                        continue
                    t = sd[info.fqn]
                    IO_STATS["bytes_read"] += t.numel() * t.element_size()
                    full[info.offset : info.offset + info.numel].copy_(t.reshape(-1).to(self.device, torch.float32))
            self.broadcast_full(full)
            if not any(info.fqn in skip for info in unit.infos):
                unit.master.copy_(unit.local_of_full(full).to(unit.master.device))
            else:  # copy only the parameters the checkpoint holds
                for info in unit.infos:
                    if info.fqn in skip or info.local_hi <= info.local_lo:
                        continue
                    lo = info.offset + info.param_lo
                    unit.master[info.local_lo : info.local_hi].copy_(
                        full[lo : lo + (info.local_hi - info.local_lo)].to(unit.master.device))
            if unit.shard_lp is not unit.master:
                unit.shard_lp.copy_(unit.master.to(unit.shard_lp.device))
            del full
        self.refresh_fp8()
        for name, p in self._extras():
            if name in skip:
                continue
            spec = getattr(p, "_ep_spec", None)
            shape = ((spec[1] * p.shape[0],) + tuple(p.shape[1:])) if spec is not None else tuple(p.shape)
            full = torch.zeros(shape, dtype=torch.float32, device=p.device)
            if sd is not None:
                full.copy_(sd[name].to(p.device, torch.float32))
            if multi:
                dist.broadcast(full, src=0)
            self._load_extra(name, full)
        if missing:
            import logging

            logging.getLogger(__name__).warning(f"FULL_STATE_DICT load: {len(missing)} keys missing from the checkpoint, e.g. {missing[:3]}")
        return missing

    @torch.no_grad()
    def load_sharded_pieces(self, pieces: list[tuple[dict, dict]]):
        """Load from any number of saved shards (resharding): each piece is (tensors, meta) of one saved rank."""
        for unit in self.units:
            for info in unit.infos:
                lo_need, hi_need = info.param_lo, info.param_lo + (info.local_hi - info.local_lo)
                for tensors, meta in pieces:
                    pm = meta["params"].get(info.fqn)
                    if pm is None:
                        continue
                    s_lo, s_hi = pm["param_lo"], pm["param_lo"] + pm["numel"]
                    a, b = max(lo_need, s_lo), min(hi_need, s_hi)
                    if b > a:
                        src = tensors[info.fqn][a - s_lo : b - s_lo]
                        unit.master[info.local_lo + (a - lo_need) : info.local_lo + (b - lo_need)].copy_(src.to(unit.master.device))
            if unit.shard_lp is not unit.master:
                unit.shard_lp.copy_(unit.master.to(unit.shard_lp.device))
        self.refresh_fp8()
        for name, p in self._extras():
            found = [(m.get("extra", {}).get(name), t) for t, m in pieces if name in m.get("extra", {})]
            if not found:
                continue
            if found[0][0]["ep"]:
                # rebuild the full expert stack from every saved rank (any EP degree), then take our slice
                full = torch.cat([t[name] for info, t in sorted(found, key=lambda x: x[0]["rank"])], 0)
            else:
                full = found[0][1][name]
            self._load_extra(name, full)

    @contextmanager
    def summon_full_params(self):
        for u in self.units:
            self._wait_unsharded(u)
        try:
            yield
        finally:
            if self.reshard_after_forward:
                for u in self.units:
                    if not u.is_root:
                        self._free_full(u)


def _grad_update(dst: torch.Tensor, src: torch.Tensor, scale: float, accumulate: bool):
    """fp32 grad shard (=|+=) scale * src in one pass (HIP `grad_shard_update` on GPU)."""
    if dst.is_cuda and src.numel() % 8 == 0 and native_enabled():
        ext().grad_shard_update(dst, src.contiguous(), float(scale), bool(accumulate))
    elif accumulate:
        dst.add_(src.to(dst.dtype), alpha=scale)
    else:
        torch.mul(src.to(dst.dtype), scale, out=dst)


class _GradHolder:
    """Adapter so multi-tensor grad kernels can run over flat grad shards."""

    __slots__ = ("grad",)

    def __init__(self, g):
        self.grad = g


def _flatten_tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _flatten_tensors(o)
    elif isinstance(obj, dict):
        for o in obj.values():
            yield from _flatten_tensors(o)
    elif hasattr(obj, "__dataclass_fields__"):
        for k in obj.__dataclass_fields__:
            yield from _flatten_tensors(getattr(obj, k))
    elif hasattr(obj, "to_tuple"):
        yield from _flatten_tensors(obj.to_tuple())


class FullyShardedModule(nn.Module):
    """Wrapper returned by `Accelerator.prepare` for FSDP models (the analogue of an FSDP2 root module).

    `parameters()` / `named_parameters()` return the fp32 master shard parameters (what an optimizer should
    see); `module` is the original model whose parameters are the gathered compute-dtype views."""

    def __init__(self, module: nn.Module, engine: FSDPEngine):
        super().__init__()
        self.module = module
        self._engine = [engine]  # list: keep out of nn.Module registration

    @property
    def engine(self) -> FSDPEngine:
        return self._engine[0]

    def forward(self, *args, **kwargs):
        eng = self.engine
        eng.pre_root_forward()
        if eng.param_dtype != torch.float32:
            args = tuple(_cast_floats(a, eng.param_dtype) for a in args)
            kwargs = {k: _cast_floats(v, eng.param_dtype) for k, v in kwargs.items()}
        out = self.module(*args, **kwargs)
        return eng.post_root_forward(out)

    def parameters(self, recurse: bool = True):
        return self.engine.shard_parameters()

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):
        for n, p in self.engine.named_shard_parameters():
            yield (prefix + "." + n if prefix else n), p

    def set_requires_gradient_sync(self, flag: bool):
        self.engine.set_requires_gradient_sync(flag)

    @contextmanager
    def no_sync(self):
        old = self.engine.requires_grad_sync
        self.engine.set_requires_gradient_sync(False)
        try:
            yield
        finally:
            self.engine.set_requires_gradient_sync(old)

    def clip_grad_norm_(self, max_norm, norm_type=2.0):
        return self.engine.clip_grad_norm_(max_norm, norm_type)

    def state_dict(self, *args, **kwargs):
        return self.engine.full_state_dict(rank0_only=False)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        return self.engine.load_full_state_dict(state_dict, strict=strict)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)


class _ExpertAmax:
    """Per-expert amax [E] of an fp8 MoE weight stack, written by the fused AdamW (ops/multi_tensor.py); `fresh` while
    the stack holds the values that launch wrote."""

    __slots__ = ("amax", "seg", "fresh")

    def __init__(self, amax: torch.Tensor, seg: int):
        self.amax, self.seg, self.fresh = amax, seg, False


class _WgradSlot:
    """Where a fused Linear's weight gradient goes. `uses` counts forward applications whose backward is pending so a
    weight applied twice reports grad-ready once (recomputation inside backward is not counted)."""

    __slots__ = ("engine", "unit", "info", "uses")

    def __init__(self, engine, unit, info):
        self.engine, self.unit, self.info, self.uses = engine, unit, info, 0


class _FusedWgradLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, slot):
        x2 = x.reshape(-1, x.shape[-1])
        # Keep a token-contiguous copy xᵀ instead of x: dW = dyᵀ·x then runs in the dgrad-class layout (one operand
        # contiguous along the contraction) instead of the both-token-major one. Llama-3-8B layer, four GEMMs
        # (tools/bench_wgrad_layout.py): fp32 output (world size 1) 2.93 vs 3.50 ms, bf16 output (flat grad buffer,
        # world size > 1) 2.86 vs 3.44 ms; the HIP transpose costs ~0.2 ms.
        # Memory: for q/k/v, gate/up and down projections the copy replaces the saved x (their inputs are not saved by
        # the producing RMSNorm / SwiGLU), but o_proj's input is the attention output that flash attention also keeps,
        # so there the copy is extra: T x 4096 bf16 = 64 MiB per layer, 2 GiB for Llama-3-8B at 8k tokens (peak
        # 175 of 288 GiB; kept for the faster layout). ACCELERATE_FSDP_WGRAD_XT=0 disables it. The opt-in hipBLASLt
        # wgrad runner (ACCELERATE_BLASLT_WGRAD=1) takes either layout (ops/fused.py wgrad_into).
        ctx.x_transposed = (_WGRAD_XT and not fused_ops.ASM_WGRAD_ABMN and x2.is_cuda and x2.dtype == torch.bfloat16 and x2.is_contiguous() and native_enabled()
                            and x2.shape[0] % 64 == 0 and x2.shape[1] % 64 == 0)
        ctx.save_for_backward(ext().transpose_bf16(x2) if ctx.x_transposed else x, weight)
        ctx.slot = slot
        ctx.has_bias = bias is not None
        return linear_fwd(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        xs, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = linear_dgrad(dy2, w).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        db = dy2.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        # (A contiguous dyᵀ as the left operand as well — both operands contraction-contiguous — measured no faster
        # end to end: the transpose of dy costs what the GEMM gains.)
        if ctx.x_transposed:
            ctx.slot.engine._fused_wgrad(ctx.slot, dy2, xs.t())  # [T, K] view of the token-contiguous copy
        else:
            ctx.slot.engine._fused_wgrad(ctx.slot, dy2, xs.reshape(-1, xs.shape[-1]))
        return dx, None, db, None


class _FusedWgradLinear(nn.Linear):
    """`nn.Linear` owned by an FSDP unit: same parameters and forward; its weight gradient is fused into the flat
    grad buffer (Megatron's gradient-accumulation fusion)."""

    def forward(self, x):
        slot = getattr(self.weight, "_acc_wgrad_slot", None)
        if slot is None or not torch.is_grad_enabled() or torch.is_autocast_enabled(x.device.type) or x.dtype != self.weight.dtype:
            return nn.functional.linear(x, self.weight, self.bias)
        if torch._C._current_graph_task_id() == -1:
            slot.uses += 1
        return _FusedWgradLinearFn.apply(x, self.weight, self.bias, slot)


class _FusedSlotEmbeddingFn(torch.autograd.Function):
    """Embedding lookup whose weight gradient is scattered straight into the fp32 grad shard (world size 1): rows of
    dy added at their token ids (`index_put_(accumulate=True)`: sorted, deterministic), untouched rows zero."""

    @staticmethod
    def forward(ctx, ids, weight, slot):
        ctx.save_for_backward(ids)
        ctx.slot = slot
        return nn.functional.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        slot = ctx.slot
        dest, acc = slot.engine._fused_slot_dest(slot)
        if not acc:
            dest.zero_()
        dest.index_put_((ids.reshape(-1),), dy.reshape(-1, dy.shape[-1]).to(dest.dtype), accumulate=True)
        slot.engine._fused_slot_done(slot)
        return None, None, None


class _FusedSlotEmbedding(nn.Embedding):
    """`nn.Embedding` owned by an FSDP unit at world size 1: same parameters and forward; the weight gradient goes to
    the engine's slot (`_FusedSlotEmbeddingFn`)."""

    def forward(self, ids):
        slot = getattr(self.weight, "_acc_wgrad_slot", None)
        if slot is None or not torch.is_grad_enabled() or not self.weight.requires_grad:
            return super().forward(ids)
        if torch._C._current_graph_task_id() == -1:
            slot.uses += 1
        return _FusedSlotEmbeddingFn.apply(ids, self.weight, slot)


def _cast_floats(x, dtype):
    if isinstance(x, torch.Tensor) and x.is_floating_point() and x.dtype != dtype:
        return x.to(dtype)
    return x


def fully_shard(
    model: nn.Module,
    plugin: Optional[FullyShardedDataParallelPlugin] = None,
    device: Optional[torch.device] = None,
    process_group=None,
    replicate_group=None,
    init_fn=None,
    seed: int = 0,
    prefetch_depth: int = 1,
    force_sharded: Optional[bool] = None,
    fp8_all_gather: bool = False,
) -> FullyShardedModule:
    """Shard `model` with the native engine and return the wrapper."""
    if plugin is None:
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if plugin.auto_wrap_policy not in (None, "NO_WRAP") and not callable(getattr(plugin, "_wrap_fn", None)):
        plugin.set_auto_wrap_policy(model)
    if plugin.activation_checkpointing:
        apply_activation_checkpointing(model, plugin)
    if force_sharded is None:
        force_sharded = os.environ.get("ACCELERATE_FSDP_FORCE_SHARDED", "0") == "1"
    engine = FSDPEngine(model, plugin, device, process_group, replicate_group, init_fn, seed, prefetch_depth, force_sharded,
                        fp8_all_gather)
    return FullyShardedModule(model, engine)


def apply_activation_checkpointing(model: nn.Module, plugin: FullyShardedDataParallelPlugin):
    """Non-reentrant activation checkpointing of every wrapped block (reference `fsdp_utils.py:588-618`)."""
    from torch.utils.checkpoint import checkpoint

    wrap = plugin._wrap_fn if getattr(plugin, "_wrap_fn", None) else plugin.set_auto_wrap_policy(model)
    if wrap is None:
        return
    for m in model.modules():
        if m is not model and wrap(m) and not getattr(m, "_acc_ckpt", False):
            orig = m.forward

            def make(orig):
                def fwd(*a, **k):
                    if torch.is_grad_enabled():
                        return checkpoint(orig, *a, use_reentrant=False, **k)
                    return orig(*a, **k)

                return fwd

            m.forward = make(orig)
            m._acc_ckpt = True
