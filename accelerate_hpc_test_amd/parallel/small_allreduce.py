"""Small-message all-reduce over HIP IPC (csrc/kernels/small_allreduce.hip): one kernel, no RCCL ring.

The step's latency-bound collectives — the clip-norm scalar (`FSDPEngine.clip_grad_norm_`), the fp8 per-weight amax
vector (`FSDPEngine.refresh_fp8`), `Accelerator.reduce` / `check_trigger` (reference `accelerator.py:2824-2881`,
`utils/operations.py:727-766`) — carry a few bytes to a few KB. A ring all-reduce costs 2(W-1) dependent xGMI hops plus
a kernel and proxy hand-off per step; here every rank maps the other ranks' buffers (one IPC handle exchange per
group, at first use) and one launch does push -> flag -> peer loads -> reduce.

Eligible: HIP tensors of fp32 / bf16 / int32 / int64, <= 1 MiB, SUM or MAX, a group whose ranks all live on this node
(<= 8). Anything else — and every group whose setup failed on any rank — goes to `torch.distributed.all_reduce`
(RCCL). `ACCELERATE_SMALL_ALLREDUCE=0` disables the path; `ACCELERATE_SMALL_ALLREDUCE_TIMEOUT_S` bounds each kernel
wait for a peer (default 300 s; a timed-out call marks the communicator failed and the next use raises).
"""

from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..ops._ext import ext, native_enabled

MAX_BYTES = 1 << 20
_DTYPES = (torch.float32, torch.bfloat16, torch.int32, torch.int64)
_OPS = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1}
_CACHE: dict = {}


def _enabled() -> bool:
    return os.environ.get("ACCELERATE_SMALL_ALLREDUCE", "1") != "0" and native_enabled()


def _timeout_ms() -> float:
    return float(os.environ.get("ACCELERATE_SMALL_ALLREDUCE_TIMEOUT_S", "300")) * 1e3


class SmallAllReduce:
    """IPC one-shot all-reduce communicator for one process group. Construction is collective over `group`."""

    def __init__(self, group=None, max_bytes: int = MAX_BYTES):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.max_bytes = max_bytes
        self.id: Optional[int] = None
        handle = None
        try:
            self.id, handle = ext().sar_create(self.rank, self.world, max_bytes)
        except Exception:  # noqa: BLE001 - any local failure: this rank votes "no"
            self.id = None
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        ok = all(h is not None for h in handles)
        if ok:
            try:
                ext().sar_open(self.id, [bytes(h) for h in handles])
            except Exception:  # noqa: BLE001
                ok = False
        votes = [None] * self.world
        dist.all_gather_object(votes, ok, group=group)
        self.ok = all(votes)
        if self.ok:
            # self-test on the real peers (short timeout): a mapping that opens but does not deliver stores across the
            # fabric is caught here and the group stays on RCCL
            t = torch.full((64,), float(self.rank + 1), device=torch.cuda.current_device())
            ext().sar_allreduce(self.id, t, t, 0, 10_000.0)
            torch.cuda.synchronize()
            good = ext().sar_status(self.id) == 0 and bool((t == self.world * (self.world + 1) / 2).all())
            votes = [None] * self.world
            dist.all_gather_object(votes, good, group=group)
            self.ok = all(votes)
        if not self.ok and self.id is not None:
            ext().sar_destroy(self.id)
            self.id = None

    def eligible(self, t: torch.Tensor, op) -> bool:
        return (self.ok and t.is_cuda and t.dtype in _DTYPES and t.is_contiguous() and op in _OPS
                and t.numel() * t.element_size() <= self.max_bytes)

    def all_reduce_(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if ext().sar_status(self.id) != 0:
            raise RuntimeError("small all-reduce: an earlier call timed out waiting for a peer rank")
        ext().sar_allreduce(self.id, t, t, _OPS[op], _timeout_ms())
        return t

    def close(self):
        if self.id is not None:
            ext().sar_destroy(self.id)
            self.id = None


def _same_node(group) -> bool:
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0)
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if local <= 0 or world <= 0 or local != world:
        return False  # multi-node (or unknown topology): stay on RCCL
    return dist.get_world_size(group) <= 8


def get(group=None) -> Optional[SmallAllReduce]:
    """The group's communicator (built collectively on first use), or None when the path does not apply."""
    if not (_enabled() and dist.is_available() and dist.is_initialized()):
        return None
    if dist.get_world_size(group) == 1 or not torch.cuda.is_available():
        return None
    # gloo groups normally mean CPU ranks; ACCELERATE_SMALL_ALLREDUCE_GLOO=1 opts in for HIP ranks on a gloo group
    # (several processes sharing one GPU: the multi-rank rehearsal of tests/test_gpu_multirank.py)
    if dist.get_backend(group) == "gloo" and os.environ.get("ACCELERATE_SMALL_ALLREDUCE_GLOO", "0") != "1":
        return None
    if not _same_node(group):
        return None
    key = tuple(dist.get_process_group_ranks(group)) if group is not None else ("world",)
    if key not in _CACHE:
        _CACHE[key] = SmallAllReduce(group)
    c = _CACHE[key]
    return c if c.ok else None


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce: the IPC one-shot kernel for small eligible tensors, RCCL otherwise."""
    c = get(group)
    if c is not None and c.eligible(t, op):
        return c.all_reduce_(t, op)
    dist.all_reduce(t, op=op, group=group)
    return t
