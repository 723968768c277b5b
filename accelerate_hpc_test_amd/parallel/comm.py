"""Dimension-aware collectives shared by the TP / CP / SP / EP layers, plus their autograd wrappers.

On MI355X these are single RCCL calls over xGMI (`all_gather_into_tensor`, `reduce_scatter_tensor`,
`all_to_all_single`) on contiguous buffers laid out so the exchanged dimension is outermost (one collective, no
per-chunk launches). The CPU fake cluster of the test-suite (gloo, host tensors) runs the SAME tensor collectives
(torch's gloo has `all_gather_into_tensor` / `reduce_scatter_tensor` / `all_to_all_single` for host tensors), so the
multi-process CPU tests exercise the exact calls, buffers and shard offsets an RCCL job issues. Only HIP tensors on a
gloo group (several ranks sharing one GPU in the one-GPU rehearsal, `tests/test_gpu_multirank.py`) fall back to the
list / all-reduce forms below.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def group_size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def group_rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _is_gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def tensor_forms(group, t: torch.Tensor) -> bool:
    """Whether `t` goes through the packed tensor collectives on `group`: always on RCCL, and on gloo for host tensors;
    HIP tensors on a gloo group take the list forms (gloo's tensor collectives are host-only)."""
    return not (t.is_cuda and _is_gloo(group))


def duplicate_group(group=None):
    """A new process group over exactly the ranks of `group`, i.e. a separate RCCL communicator.

    Each purpose that issues collectives from its own HIP stream (FSDP all-gather, FSDP reduce-scatter, DDP bucket
    all-reduce) gets one. ProcessGroupNCCL (RCCL here) runs every collective of a process group on that group's own
    internal stream (high priority, `_high_priority_options`), fenced by events: the internal stream first waits for the
    issuing stream's earlier work, and the issuing stream then waits for the collective. Collectives of ONE group
    therefore serialise on its single internal stream whichever stream issued them; separate groups are what let the
    all-gather of one unit and the reduce-scatter of another run at the same time (`profiles/r4_fsdp_forced_sharded.md`:
    the nranks=1 stand-ins of both overlap 76 % with compute). `new_group` has to
    be entered by every rank of the world for every group created, so the member lists of all ranks are exchanged
    first and each distinct list is created, in the same order everywhere (HSDP / mesh sub-groups included)."""
    ranks = tuple(dist.get_process_group_ranks(group if group is not None else dist.group.WORLD))
    world = dist.get_world_size()
    opts = _high_priority_options()
    if world == 1:
        return dist.new_group([0], pg_options=opts)
    lists = [None] * world
    dist.all_gather_object(lists, ranks)
    mine = None
    for rl in sorted(set(tuple(r) for r in lists)):
        g = dist.new_group(list(rl), pg_options=opts)
        if rl == ranks:
            mine = g
    return mine


def _high_priority_options():
    """RCCL process-group options with the communicator's internal HIP streams at high priority (the collectives'
    kernels then win dispatch against queued compute kernels), unless ACCELERATE_RCCL_STREAM_PRIORITY=0. None on gloo."""
    import os

    if dist.get_backend() != "nccl" or os.environ.get("ACCELERATE_RCCL_STREAM_PRIORITY", "-1") == "0":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except Exception:  # noqa: BLE001 - a build without the NCCL/RCCL backend
        return None


# ------------------------------------------------------------------------------------------------ raw collectives
def all_reduce_(t: torch.Tensor, group=None, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if group_size(group) > 1:
        dist.all_reduce(t, op=op, group=group)
    return t


def all_gather_dim(t: torch.Tensor, dim: int, group=None) -> torch.Tensor:
    """Concatenate every rank's `t` along `dim` (rank order)."""
    W = group_size(group)
    if W == 1:
        return t
    dim = dim % t.dim()
    src = t.movedim(dim, 0).contiguous()
    out = torch.empty((W * src.shape[0],) + tuple(src.shape[1:]), dtype=t.dtype, device=t.device)
    if not tensor_forms(group, src):
        dist.all_gather(list(out.chunk(W)), src, group=group)
    else:
        dist.all_gather_into_tensor(out, src, group=group)
    return out.movedim(0, dim)


def reduce_scatter_dim(t: torch.Tensor, dim: int, group=None) -> torch.Tensor:
    """Sum over ranks, then keep this rank's `dim`-chunk."""
    W = group_size(group)
    if W == 1:
        return t
    dim = dim % t.dim()
    src = t.movedim(dim, 0).contiguous()
    if src.shape[0] % W:
        raise ValueError(f"reduce_scatter along dim {dim}: size {src.shape[0]} not divisible by {W}")
    if not tensor_forms(group, src):
        tmp = src.clone()
        dist.all_reduce(tmp, group=group)
        out = tmp.chunk(W)[group_rank(group)].contiguous()
    else:
        out = torch.empty((src.shape[0] // W,) + tuple(src.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, src, group=group)
    return out.movedim(0, dim)


def split_dim(t: torch.Tensor, dim: int, group=None) -> torch.Tensor:
    W = group_size(group)
    if W == 1:
        return t
    if t.shape[dim] % W:
        raise ValueError(f"split along dim {dim}: size {t.shape[dim]} not divisible by {W}")
    return t.chunk(W, dim=dim)[group_rank(group)].contiguous()


def all_to_all_dims(t: torch.Tensor, scatter_dim: int, gather_dim: int, group=None) -> torch.Tensor:
    """Split `t` along `scatter_dim` into W chunks, send chunk j to rank j, concatenate what arrives along
    `gather_dim` (the Ulysses sequence<->head re-partition). One `all_to_all_single` on a packed buffer."""
    W = group_size(group)
    if W == 1:
        return t
    scatter_dim %= t.dim()
    gather_dim %= t.dim()
    if t.shape[scatter_dim] % W:
        raise ValueError(f"all_to_all: dim {scatter_dim} of size {t.shape[scatter_dim]} not divisible by {W}")
    # pack: [W, ...chunk...] with the scatter dim split out front
    chunks = t.chunk(W, dim=scatter_dim)
    send = torch.stack([c.contiguous() for c in chunks], 0)
    recv = torch.empty_like(send)
    if not tensor_forms(group, send):
        # HIP tensors on a gloo group: all_to_all through all_gather
        gathered = [torch.empty_like(send) for _ in range(W)]
        dist.all_gather(gathered, send, group=group)
        me = group_rank(group)
        recv = torch.stack([g[me] for g in gathered], 0)
    else:
        dist.all_to_all_single(recv, send, group=group)
    return torch.cat(list(recv.unbind(0)), dim=gather_dim)


def all_to_all_varlen(t: torch.Tensor, send_counts: list, recv_counts: list, group=None) -> torch.Tensor:
    """Row-wise variable all-to-all: rows [sum(send_counts[:j]), +send_counts[j]) go to rank j (MoE dispatch)."""
    W = group_size(group)
    if W == 1:
        return t
    out = torch.empty((sum(recv_counts),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if not tensor_forms(group, t):
        me = group_rank(group)
        # HIP tensors on a gloo group: exchange via all_gather of padded blocks
        mx = max(max(send_counts), 1)
        pad = torch.zeros((W, mx) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        o = 0
        for j, c in enumerate(send_counts):
            pad[j, :c] = t[o : o + c]
            o += c
        gathered = [torch.empty_like(pad) for _ in range(W)]
        maxes = [torch.zeros(1, dtype=torch.long) for _ in range(W)]
        dist.all_gather(maxes, torch.tensor([mx]), group=group)
        if any(int(m) != mx for m in maxes):
            gmx = max(int(m) for m in maxes)
            pad2 = torch.zeros((W, gmx) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            pad2[:, :mx] = pad
            pad = pad2
            gathered = [torch.empty_like(pad) for _ in range(W)]
        dist.all_gather(gathered, pad, group=group)
        o = 0
        for j, c in enumerate(recv_counts):
            out[o : o + c] = gathered[j][me, :c]
            o += c
        return out
    dist.all_to_all_single(out, t.contiguous(), output_split_sizes=list(recv_counts), input_split_sizes=list(send_counts), group=group)
    return out


# ------------------------------------------------------------------------------------------------ autograd wrappers
class _CopyToGroup(torch.autograd.Function):
    """fwd: identity (input replicated on the group); bwd: all-reduce the partial input-grads."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return all_reduce_(g.contiguous().clone(), ctx.group), None


class _ReduceFromGroup(torch.autograd.Function):
    """fwd: all-reduce partial outputs; bwd: identity."""

    @staticmethod
    def forward(ctx, x, group):
        return all_reduce_(x.contiguous().clone(), group)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherDim(torch.autograd.Function):
    """fwd: all-gather along dim; bwd: reduce-scatter (sum) along dim — sequence-parallel entry."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return all_gather_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_dim(g, ctx.dim, ctx.group), None, None


class _GatherDimNoReduce(torch.autograd.Function):
    """fwd: all-gather along dim; bwd: take own chunk (consumer computed the same full grad on every rank)."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return all_gather_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return split_dim(g, ctx.dim, ctx.group), None, None


class _ReduceScatterDim(torch.autograd.Function):
    """fwd: reduce-scatter along dim; bwd: all-gather — sequence-parallel exit."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return reduce_scatter_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return all_gather_dim(g, ctx.dim, ctx.group), None, None


class _SplitDim(torch.autograd.Function):
    """fwd: keep own chunk; bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        return split_dim(x, dim, group)

    @staticmethod
    def backward(ctx, g):
        return all_gather_dim(g, ctx.dim, ctx.group), None, None


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scatter_dim, gather_dim, group):
        ctx.sd, ctx.gd, ctx.group = scatter_dim, gather_dim, group
        return all_to_all_dims(x, scatter_dim, gather_dim, group)

    @staticmethod
    def backward(ctx, g):
        return all_to_all_dims(g, ctx.gd, ctx.sd, ctx.group), None, None, None


class _AllToAllVar(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, send_counts, recv_counts, group):
        ctx.sc, ctx.rc, ctx.group = send_counts, recv_counts, group
        return all_to_all_varlen(x, send_counts, recv_counts, group)

    @staticmethod
    def backward(ctx, g):
        return all_to_all_varlen(g.contiguous(), ctx.rc, ctx.sc, ctx.group), None, None, None


def copy_to_group(x, group):
    return _CopyToGroup.apply(x, group) if group_size(group) > 1 else x


def reduce_from_group(x, group):
    return _ReduceFromGroup.apply(x, group) if group_size(group) > 1 else x


def gather_along(x, dim, group, reduce_grad: bool = True):
    if group_size(group) == 1:
        return x
    return (_GatherDim if reduce_grad else _GatherDimNoReduce).apply(x, dim, group)


def reduce_scatter_along(x, dim, group):
    return _ReduceScatterDim.apply(x, dim, group) if group_size(group) > 1 else x


def split_along(x, dim, group):
    return _SplitDim.apply(x, dim, group) if group_size(group) > 1 else x


def all_to_all(x, scatter_dim, gather_dim, group):
    return _AllToAll.apply(x, scatter_dim, gather_dim, group) if group_size(group) > 1 else x


def all_to_all_var(x, send_counts, recv_counts, group):
    return _AllToAllVar.apply(x, list(send_counts), list(recv_counts), group) if group_size(group) > 1 else x
