"""Native data-parallel gradient reducer (DDP) for MI355X.

Parity: the reference wraps `torch.nn.parallel.DistributedDataParallel` (`/root/reference/src/accelerate/accelerator.py:1850-1869`)
with kwargs from `DistributedDataParallelKwargs` (`utils/dataclasses.py:154-237`) and toggles sync with
`model.no_sync()` (`accelerator.py:1130-1177`). This module replaces the C++ DDP reducer:

* Gradients live in flat per-bucket buffers (parameters' `.grad` are views into them, i.e. always
  `gradient_as_bucket_view`), so accumulation is in place and the bucket is all-reduced with no pack copy.
* Buckets are filled in reverse registration order (≈ the order gradients become ready) up to
  `bucket_cap_mb` — by default 128 MB (16 MB per peer at 8 GPUs) so each RCCL all-reduce is large enough to drive
  all 7 xGMI links, instead of torch's 25 MB.
* Bucket all-reduces are launched from post-accumulate-grad hooks strictly in bucket-index order (a ready bucket
  waits until every lower-index bucket has launched, like torch's `next_bucket_`), on a dedicated high-priority HIP
  stream and a communicator of its own (overlapping the rest of backward). An autograd final callback flushes the
  remaining buckets in the same order — this covers `find_unused_parameters` even when ranks leave DIFFERENT
  parameters unused (MoE experts, data-dependent branches): every rank issues the same collective sequence — and
  orders the compute stream after the comm stream, with no host blocking.
* Communication hooks: `bf16`/`fp16` compression casts the bucket once, all-reduces in 16-bit and casts back;
  averaging (1/W) is folded into that pass (or done with ReduceOp.AVG on RCCL).
* `no_sync()` skips the launches (grads keep accumulating in the buckets); `broadcast_buffers` re-broadcasts
  buffers from rank 0 each forward with ONE coalesced collective.
"""

from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Optional

import weakref

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops._ext import ext, use_native
from ..ops import fused as fused_ops
from ..ops.fused import linear_dgrad, wgrad_into
from ..utils.dataclasses import DDPCommunicationHookType
from ..utils.fault_tolerance import record_collective
from ..utils.tracing import trace_range


class _Bucket:
    def __init__(self, params, dtype, device):
        self.params = params
        self.offsets = []
        n = 0
        for p in params:
            self.offsets.append(n)
            n += p.numel()
        self.numel = n
        self.buffer = torch.zeros(n, dtype=dtype, device=device)
        self.pending = len(params)
        self.launched = False


def _weak_method_hook(obj, name: str):
    """A parameter hook calling `obj.<name>` through a weak reference: hooks live in the tensor's C++ autograd
    metadata, which the cycle collector cannot traverse, so a bound method there would keep the reducer (and its
    bucket buffers) alive after the user drops the model."""
    ref = weakref.ref(obj)

    def hook(p):
        o = ref()
        if o is not None:
            getattr(o, name)(p)

    return hook


class _DDPWgradSlot:
    """Per-weight state of a fused weight-gradient Linear under the reducer: `uses` counts forward applications whose
    backward is pending (a weight applied twice reports grad-ready once)."""

    __slots__ = ("ddp", "param", "uses")

    def __init__(self, ddp, param):
        self.ddp, self.param, self.uses = weakref.ref(ddp), param, 0


class _DDPFusedLinearFn(torch.autograd.Function):
    """y = x Wᵀ (+ b) in the autocast dtype, with dW = dyᵀ x written by the GEMM itself, in fp32, straight into the
    weight's slot of its reducer bucket (accumulated when the slot already holds this step's gradient). Replaces the
    autocast path's bf16 dW, its cast to fp32 and the hook's copy into the bucket (16 B/param of HBM traffic) with
    the GEMM's one fp32 write (4 B/param)."""

    @staticmethod
    def forward(ctx, x, weight, bias, slot, cdtype):
        xc = x.to(cdtype) if cdtype is not None else x
        wc = weight.to(cdtype) if cdtype is not None else weight
        bc = bias.to(cdtype) if (bias is not None and cdtype is not None) else bias
        x2 = xc.reshape(-1, xc.shape[-1])
        # token-contiguous copy xᵀ for the weight-gradient GEMM (as the FSDP engine does, parallel/fsdp.py
        # _FusedWgradLinearFn): hipBLASLt's fp32-output kernels run that layout with a depth-64 tile instead of a
        # depth-32 one (measured on Llama-3-8B under the reducer: 1.21 ms -> ~0.91 ms per call)
        ctx.x_t = (not fused_ops.ASM_WGRAD_ABMN and x2.is_cuda and x2.dtype == torch.bfloat16 and x2.is_contiguous() and x2.shape[0] % 64 == 0
                   and x2.shape[1] % 64 == 0 and use_native(x2))
        ctx.save_for_backward(ext().transpose_bf16(x2) if ctx.x_t else x2, wc)
        ctx.slot, ctx.xdtype, ctx.xshape = slot, x.dtype, x.shape
        ctx.bdtype = bias.dtype if bias is not None else None
        return nn.functional.linear(xc, wc, bc)

    @staticmethod
    def backward(ctx, dy):
        xs, wc = ctx.saved_tensors
        N, K = wc.shape
        dy = dy.to(wc.dtype)
        dy2 = dy.reshape(-1, N)
        dx = linear_dgrad(dy2, wc).view(*dy.shape[:-1], K).to(ctx.xdtype) if ctx.needs_input_grad[0] else None
        ddp = ctx.slot.ddp()
        if ddp is not None:
            ddp._fused_wgrad(ctx.slot, dy2, xs.t() if ctx.x_t else xs)
        db = dy2.float().sum(0).to(ctx.bdtype) if ctx.bdtype is not None else None
        return dx, None, db, None, None


class _DDPFusedLinear(nn.Linear):
    """`nn.Linear` whose weight gradient goes to its DDP bucket slot through `_DDPFusedLinearFn`."""

    def forward(self, x):
        slot = getattr(self, "_acc_ddp_slot", None)
        if slot is None or slot.ddp() is None or not torch.is_grad_enabled() or not self.weight.requires_grad:
            return nn.functional.linear(x, self.weight, self.bias)
        if torch._C._current_graph_task_id() == -1:  # not an activation-checkpoint recompute inside backward
            slot.uses += 1
        dev = x.device.type
        cdtype = torch.get_autocast_dtype(dev) if torch.is_autocast_enabled(dev) else None
        return _DDPFusedLinearFn.apply(x, self.weight, self.bias, slot, cdtype)


class DistributedDataParallel(nn.Module):
    """Drop-in for `torch.nn.parallel.DistributedDataParallel` built on our bucketed RCCL reducer."""

    def __init__(
        self,
        module: nn.Module,
        device_ids=None,
        output_device=None,
        process_group=None,
        bucket_cap_mb: Optional[float] = None,
        broadcast_buffers: bool = True,
        find_unused_parameters: bool = False,
        gradient_as_bucket_view: bool = True,
        static_graph: bool = False,
        comm_hook: DDPCommunicationHookType = DDPCommunicationHookType.NO,
        comm_wrapper: DDPCommunicationHookType = DDPCommunicationHookType.NO,
        bucket_bytes: Optional[int] = None,
        comm_state_option: Optional[dict] = None,
        own_communicator: bool = False,
        **unused,
    ):
        super().__init__()
        self.module = module
        self.comm_state_option = dict(comm_state_option or {})
        self._psgd: dict = {}
        self._join = None
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        fused_ops.set_dgrad_concurrent(True)  # bucket all-reduces beside the backward (the reducer exists only then)
        self.broadcast_buffers = broadcast_buffers
        self.require_backward_grad_sync = True
        # torch DDP semantics: whether a backward all-reduces is decided by the FORWARD that built its graph (under
        # `no_sync()` or not), unless `trigger_sync()` (Accelerator.trigger_sync_in_backward) forces it.
        self._sync_pending = True
        self.find_unused_parameters = find_unused_parameters
        self.device = next((p.device for p in module.parameters()), torch.device("cpu"))
        self.is_cuda = self.device.type == "cuda"
        self.is_gloo = dist.get_backend(process_group) == "gloo"
        self.comm_hook = DDPCommunicationHookType(comm_hook) if comm_hook is not None else DDPCommunicationHookType.NO
        if comm_wrapper not in (None, DDPCommunicationHookType.NO):
            self.comm_hook = DDPCommunicationHookType(comm_wrapper)
        if bucket_bytes is None:
            bucket_bytes = int((bucket_cap_mb if bucket_cap_mb is not None else 128) * (1 << 20))
        self.bucket_bytes = bucket_bytes
        self.comm_stream = torch.cuda.Stream(device=self.device, priority=-1) if self.is_cuda else None
        # bucket all-reduces run on comm_stream through their own communicator (parallel/comm.duplicate_group), so
        # they never share an RCCL communicator with collectives issued from other streams
        self.comm_group = process_group
        if self.is_cuda and not self.is_gloo and (self.world_size > 1 or own_communicator):
            from .comm import duplicate_group

            self.comm_group = duplicate_group(process_group)
        self._next_bucket = 0
        self._cb_queued = False
        self._unset: set = set()  # ids of params whose grad is None at forward (filled by the hook's copy)
        self._sync_params_and_buffers()
        self._build_buckets()
        self._fused_slots = []
        self._fused_ids: set = set()  # ids of the weights whose gradient the fused GEMM writes (kept here, not on them)
        if os.environ.get("ACCELERATE_DDP_FUSED_WGRAD", "1") != "0":
            self._install_fused_wgrad()

    # ------------------------------------------------------------------------------------------ setup
    @torch.no_grad()
    def _sync_params_and_buffers(self):
        """Broadcast parameters and buffers from rank 0 (one coalesced broadcast per dtype)."""
        tensors = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        self._coalesced_broadcast(tensors)

    def _coalesced_broadcast(self, tensors, chunk_bytes: int = 256 << 20, src: int = 0):
        """Broadcast from rank 0 in packed pieces of at most `chunk_bytes` per dtype (a tensor larger than that goes
        alone, in place). Packing keeps the call count low for many small tensors; the cap keeps the transient pack
        buffer small (a whole-model pack of Llama-3-8B fp32 would be a 32 GB spike on every rank)."""
        src = dist.get_global_rank(self.process_group, src) if self.process_group else src
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)

        def flush(batch):
            if not batch:
                return
            if len(batch) == 1 and batch[0].is_contiguous():
                dist.broadcast(batch[0], src=src, group=self.process_group)
                return
            flat = torch.cat([t.reshape(-1) for t in batch])
            dist.broadcast(flat, src=src, group=self.process_group)
            off = 0
            for t in batch:
                n = t.numel()
                t.copy_(flat[off : off + n].view_as(t))
                off += n

        for ts in by_dtype.values():
            batch, nbytes = [], 0
            for t in ts:
                b = t.numel() * t.element_size()
                if batch and nbytes + b > chunk_bytes:
                    flush(batch)
                    batch, nbytes = [], 0
                batch.append(t)
                nbytes += b
            flush(batch)

    def _build_buckets(self):
        seen = set()
        params = []
        for p in self.module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        params = list(reversed(params))  # gradients become ready roughly in reverse registration order
        self.buckets: list[_Bucket] = []
        self._param_bucket = {}
        cur, cur_bytes, cur_dtype = [], 0, None
        for p in params:
            nbytes = p.numel() * p.element_size()
            if cur and (p.dtype != cur_dtype or cur_bytes + nbytes > self.bucket_bytes):
                self.buckets.append(_Bucket(cur, cur_dtype, self.device))
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
            cur_dtype = p.dtype
        if cur:
            self.buckets.append(_Bucket(cur, cur_dtype, self.device))
        owner = weakref.ref(self)
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._param_bucket[p] = bi
                # the newest reducer owns the parameter: hooks of an earlier wrapper of the same model (re-prepared
                # after free_memory, or by a second Accelerator) stay registered but stand down
                p._acc_ddp_owner = owner
                p.register_post_accumulate_grad_hook(_weak_method_hook(self, "_grad_hook"))
        self._assign_grad_views(zero=True)

    def _assign_grad_views(self, zero: bool):
        for b in self.buckets:
            if zero:
                b.buffer.zero_()
            for p, off in zip(b.params, b.offsets):
                p.grad = b.buffer[off : off + p.numel()].view_as(p)

    def _install_fused_wgrad(self):
        """Route the weight gradient of every plain `nn.Linear` (weight in a bucket, used by no other module) through
        `_DDPFusedLinear`: its backward GEMM writes fp32 straight into the bucket slot."""
        refs = {}
        for m in self.module.modules():
            for q in m._parameters.values():
                if q is not None:
                    refs[id(q)] = refs.get(id(q), 0) + 1
        for m in self.module.modules():
            w = getattr(m, "weight", None)
            # a module an earlier reducer already converted is re-bound to this one (its old slot would write into
            # the old reducer's buckets, or nowhere once that reducer is gone)
            if type(m) in (nn.Linear, _DDPFusedLinear) and w is not None and w.requires_grad and refs.get(id(w), 0) == 1 \
                    and w in self._param_bucket and w.dtype == self.buckets[self._param_bucket[w]].buffer.dtype:
                m.__class__ = _DDPFusedLinear
                m._acc_ddp_slot = _DDPWgradSlot(self, w)
                self._fused_ids.add(id(w))
                self._fused_slots.append(m._acc_ddp_slot)

    @torch.no_grad()
    def _fused_wgrad(self, slot: _DDPWgradSlot, dy2: torch.Tensor, x2: torch.Tensor):
        p = slot.param
        b = self.buckets[self._param_bucket[p]]
        view = self._slot(b, p)
        if p.grad is not None and p.grad.data_ptr() != view.data_ptr():  # a gradient the user set: move it in first
            view.copy_(p.grad)
            p.grad = view
        acc = p.grad is not None  # torch semantics: accumulate unless zero_grad set the grad to None
        wgrad_into(view, dy2, x2, acc)
        p.grad = view
        slot.uses -= 1
        if slot.uses <= 0:
            slot.uses = 0
            self._grad_ready(p)

    # ------------------------------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        # After `zero_grad(set_to_none=True)` the grads are None. They stay None: autograd then hands each parameter a
        # fresh gradient, which the grad hook copies into its bucket slot (one 8 B/param copy) and re-points `.grad`
        # at; no bucket-wide zero fill followed by an accumulate-add (4 + 12 B/param). Slots whose parameter gets no
        # gradient this backward are zeroed in `_finalize`, before their bucket is reduced.
        self._unset = {id(p) for b in self.buckets for p in b.params if p.grad is None}
        join = getattr(self, "_join", None)
        if join is not None:
            syncing = int(self.require_backward_grad_sync and torch.is_grad_enabled())
            join["active"], _ = self._join_counter(1, syncing)
            join["steps"] += 1
            if join["active"] < self.world_size and join["throw"]:
                raise RuntimeError("DDP join: another rank ran out of inputs (throw_on_early_termination=True)")
        uneven = join is not None and join["active"] < self.world_size
        if self.broadcast_buffers and self.world_size > 1 and not uneven:
            bufs = [b for b in self.module.buffers()]
            if bufs:
                with torch.no_grad():
                    self._coalesced_broadcast(bufs)
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        self._next_bucket = 0
        if torch.is_grad_enabled():
            self._sync_pending = self.require_backward_grad_sync
        return self.module(*inputs, **kwargs)

    def trigger_sync(self):
        """Make the next backward all-reduce even though its forward ran under `no_sync()`."""
        self._sync_pending = True

    # ------------------------------------------------------------------------------------------ reduce
    def _grad_hook(self, p):
        owner = getattr(p, "_acc_ddp_owner", None)
        if owner is not None and owner() is not self:
            return  # a later reducer wraps this parameter now
        if id(p) in self._fused_ids:
            return  # autograd still runs the hook of a weight whose Function returned no grad; the GEMM counted it
        b = self.buckets[self._param_bucket[p]]
        if p.grad is not None and b.buffer.numel() and p.grad.data_ptr() != self._slot_ptr(b, p):
            with torch.no_grad():  # first gradient since zero_grad (or one set by the user): move it into the bucket
                view = self._slot(b, p)
                view.copy_(p.grad)
                p.grad = view
        self._grad_ready(p)

    def _grad_ready(self, p):
        b = self.buckets[self._param_bucket[p]]
        self._unset.discard(id(p))
        if not self._cb_queued:
            self._cb_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b.pending -= 1
        join = getattr(self, "_join", None)
        deferred = join is not None and join["active"] < self.world_size  # joined ranks shadow in bucket order
        if b.pending == 0 and self._sync_pending and not deferred:
            self._launch_ready()

    def _launch_ready(self):
        """Launch the ready buckets at the front of the index order (never out of order)."""
        while self._next_bucket < len(self.buckets) and self.buckets[self._next_bucket].pending == 0:
            self._launch(self.buckets[self._next_bucket])
            self._next_bucket += 1

    def _slot(self, b, p):
        i = next(j for j, q in enumerate(b.params) if q is p)
        return b.buffer[b.offsets[i] : b.offsets[i] + p.numel()].view_as(p)

    def _slot_ptr(self, b, p):
        return self._slot(b, p).data_ptr()

    @torch.no_grad()
    def _launch(self, b: _Bucket):
        if b.launched:
            return
        b.launched = True
        if self.is_cuda:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream), trace_range("ddp.bucket_all_reduce"):
                self._allreduce(b)
        else:
            self._allreduce(b)

    def _allreduce(self, b):
        self._allreduce_buffer(b.buffer, key=self.buckets.index(b))
        join = getattr(self, "_join", None)
        if join is not None and not join["divide_initial"] and join["active"] < self.world_size:
            b.buffer.mul_(self.world_size / join["active"])  # average over the ranks still training

    def _allreduce_buffer(self, buf, key: int = 0):
        W = self.world_size
        group = self.comm_group
        record_collective("ddp_all_reduce", buf, self.process_group)
        if self.comm_hook in (DDPCommunicationHookType.POWER_SGD, DDPCommunicationHookType.BATCHED_POWER_SGD) and buf.dtype.is_floating_point:
            self._powersgd(buf, key)
            return
        if self.comm_hook in (DDPCommunicationHookType.BF16, DDPCommunicationHookType.FP16) and buf.dtype == torch.float32:
            dt = torch.bfloat16 if self.comm_hook == DDPCommunicationHookType.BF16 else torch.float16
            tmp = buf.to(dt).div_(W)
            dist.all_reduce(tmp, group=group)
            buf.copy_(tmp)
            return
        if self.is_gloo:
            dist.all_reduce(buf, group=group)
            buf.div_(W)
        else:
            # AVG folds the 1/W into RCCL's reduction; with one rank it is the identity, and RCCL's single-rank AVG
            # still runs a scaling pass over the whole bucket (75 ms/step of fp32 Llama-3-8B buckets, measured), so SUM
            dist.all_reduce(buf, op=dist.ReduceOp.AVG if W > 1 else dist.ReduceOp.SUM, group=group)

    @torch.no_grad()
    def _powersgd(self, buf, key: int):
        """PowerSGD (Vogels et al. 2019), as torch's `powerSGD_hook` used by the reference via
        `DDPCommunicationHookType.POWER_SGD` (dataclasses.py:134-151,197-237): the bucket is viewed as an [n, m]
        matrix M (+ error feedback); P = M·Q is all-reduced and orthonormalised, Q = Mᵀ·P all-reduced, and
        P·Qᵀ/W replaces the bucket. Two small all-reduces instead of one bucket-sized one. Vanilla all-reduce for
        the first `start_powerSGD_iter` iterations and for buckets whose compression rate is too low."""
        opt = self.comm_state_option
        r = int(opt.get("matrix_approximation_rank", 1))
        start_iter = int(opt.get("start_powerSGD_iter", 1000))
        min_rate = float(opt.get("min_compression_rate", 2.0))
        W = self.world_size
        st = self._psgd.setdefault(key, {"iter": 0})
        st["iter"] += 1
        n_el = buf.numel()
        m = max(1, int(n_el ** 0.5))
        n = -(-n_el // m)
        compressible = (n * m) / max(1, r * (n + m)) >= min_rate
        group = self.comm_group
        if st["iter"] <= start_iter or not compressible:
            if self.is_gloo:
                dist.all_reduce(buf, group=group)
                buf.div_(W)
            else:
                dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
            return
        M = torch.zeros(n * m, dtype=torch.float32, device=buf.device)
        M[:n_el] = buf.float()
        M = M.view(n, m)
        if opt.get("use_error_feedback", True):
            err = st.get("err")
            if err is None:
                err = st["err"] = torch.zeros_like(M)
            M += err
        Q = st.get("Q")
        if Q is None or not opt.get("warm_start", True):
            g = torch.Generator(device="cpu").manual_seed(int(opt.get("random_seed", 0)) + key)
            Q = torch.randn(m, r, generator=g).to(buf.device)
        P = M @ Q
        dist.all_reduce(P, group=group)
        P, _ = torch.linalg.qr(P)
        Q = M.t() @ P
        dist.all_reduce(Q, group=group)
        Q.div_(W)
        approx = P @ Q.t()
        if opt.get("use_error_feedback", True):
            st["err"] = M - approx  # note: M is this rank's (grad + error), approx is the global average
        st["Q"] = Q
        buf.copy_(approx.view(-1)[:n_el].to(buf.dtype))

    def _finalize(self):
        self._cb_queued = False
        for slot in self._fused_slots:
            slot.uses = 0  # forwards whose outputs never reached this backward
        if self._unset:  # parameters without a gradient this backward: zero slots, grads point at them
            with torch.no_grad():
                for b in self.buckets:
                    for p in b.params:
                        if id(p) in self._unset:
                            view = self._slot(b, p)
                            view.zero_()
                            p.grad = view
            self._unset.clear()
        if self._sync_pending:
            for b in self.buckets[self._next_bucket :]:  # unused params never fired: flush the rest in index order
                self._launch(b)
            self._next_bucket = len(self.buckets)
            if self.is_cuda:
                torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    # ------------------------------------------------------------------------------------------ API
    @contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    def set_comm_hook(self, hook, wrapper=None, state=None):
        self.comm_hook = DDPCommunicationHookType(hook)
        if wrapper not in (None, DDPCommunicationHookType.NO):
            self.comm_hook = DDPCommunicationHookType(wrapper)
        if isinstance(state, dict):
            self.comm_state_option.update(state)

    @contextmanager
    def join(self, divide_by_initial_world_size: bool = True, enable: bool = True, throw_on_early_termination: bool = False):
        """Uneven inputs (torch `Join` semantics, reference accelerator.py:1298-1379).

        Inside the context every forward all-reduces a tiny [active, syncing] counter. A rank whose data ran out
        leaves the loop and, in `__exit__`, *shadows* the other ranks: for each of their iterations it joins the
        counter all-reduce and, if they sync, all-reduces zero-filled buckets in bucket order (active ranks launch
        their buckets in that same order at the end of backward while joined ranks exist). Gradients are divided
        by the initial world size (joined ranks contribute zeros) or, with `divide_by_initial_world_size=False`,
        by the number of ranks still active. `throw_on_early_termination` raises on active ranks instead."""
        if not enable or self.world_size == 1:
            yield
            return
        self._join = {"divide_initial": divide_by_initial_world_size, "throw": throw_on_early_termination,
                      "active": self.world_size, "steps": 0}
        try:
            yield
        finally:
            try:
                self._shadow_until_all_joined()
                self._sync_from_last_joiner()
            finally:
                self._join = None

    @torch.no_grad()
    def _sync_from_last_joiner(self):
        """Ranks that joined early stopped stepping their optimizer: re-broadcast parameters and buffers from the
        rank that trained the longest (torch Join's `is_last_joiner` sync)."""
        t = torch.tensor([self._join["steps"] * self.world_size + (self.world_size - 1 - self.rank)], dtype=torch.int64,
                         device=self.device if not self.is_gloo else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        src = self.world_size - 1 - int(t.item()) % self.world_size
        self._coalesced_broadcast([p.data for p in self.module.parameters()] + list(self.module.buffers()), src=src)

    def _join_counter(self, active: int, syncing: int) -> tuple[int, int]:
        t = torch.tensor([active, syncing], dtype=torch.int64, device=self.device if not self.is_gloo else "cpu")
        dist.all_reduce(t, group=self.process_group)
        a, s = t.tolist()
        return a, s

    @torch.no_grad()
    def _shadow_until_all_joined(self):
        while True:
            active, syncing = self._join_counter(0, 0)
            if active == 0:
                return
            if self._join["throw"]:
                raise RuntimeError("DDP join: this rank ran out of inputs while others are still training")
            if syncing:
                for i, b in enumerate(self.buckets):  # same collectives, same order, same op as the active ranks
                    self._allreduce_buffer(torch.zeros_like(b.buffer), key=i)
                if self.is_cuda:
                    torch.cuda.current_stream(self.device).synchronize()

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)
