"""Context parallelism: ring attention over the `cp` mesh dimension for long sequences.

Parity target: `/root/reference/src/accelerate/accelerator.py:1641-1654,4075-4140` (`maybe_context_parallel`, which
wraps torch's experimental `context_parallel`: buffers sharded along their sequence dim, SDPA swapped for a ring
variant, K/V rotated by all-gather (default) or all-to-all), and `docs/source/concept_guides/context_parallelism.md`.

MI355X design:
  * Load-balanced ("zig-zag") layout: the sequence is cut into 2·cp chunks and rank r keeps chunks r and
    2·cp-1-r, so every rank does the same causal work (2·cp+1 chunk-blocks).
  * Every attention block is an L×L call of the HIP flash-attention kernel returning its log-sum-exp; the blocks of
    one query chunk are merged in fp32 with the LSE rule. All strictly-lower (full) blocks of a query chunk are
    stacked along the batch axis → one kernel launch per chunk, not one per block.
  * "allgather": one RCCL all-gather of K,V per layer (xGMI all-gather, 2·4 MB/rank/layer at S=128k, cp=8), dK,dV
    returned with one reduce-scatter. "alltoall": K,V stream around a P2P ring (`batch_isend_irecv`) overlapped
    with the block computation in forward.
  * Backward is block-wise with the *global* O and LSE (so every block's softmax is already normalised) —
    the standard ring-attention identity; dQ accumulates locally, dK/dV are reduce-scattered to their owners.
  * Models opt in through `attention_impl` on their attention modules (our models); any other model gets
    `torch.nn.functional.scaled_dot_product_attention` patched for the duration of the context, like torch's CP.
"""

from __future__ import annotations

import contextlib
import math
from typing import Optional

import torch
import torch.distributed as dist

from ..ops._ext import ext, use_native
from ..ops.fused import flash_attn_with_lse
from . import comm


# ------------------------------------------------------------------------------------------------ layout helpers
def zigzag_indices(seq_len: int, world: int, rank: int, device=None) -> torch.Tensor:
    """Global positions held by `rank`: chunks r and 2W-1-r of 2W equal chunks."""
    if seq_len % (2 * world):
        raise ValueError(f"context parallel: sequence length {seq_len} must be divisible by 2*cp={2 * world}")
    L = seq_len // (2 * world)
    a = torch.arange(rank * L, (rank + 1) * L, device=device)
    b = torch.arange((2 * world - 1 - rank) * L, (2 * world - rank) * L, device=device)
    return torch.cat([a, b])


def zigzag_shard(t: torch.Tensor, dim: int, world: int, rank: int) -> torch.Tensor:
    idx = zigzag_indices(t.shape[dim], world, rank, device=t.device)
    return t.index_select(dim, idx).contiguous()


def zigzag_unshard(parts: list, dim: int) -> torch.Tensor:
    """Inverse of zigzag_shard given every rank's local tensor (rank order)."""
    W = len(parts)
    chunks = [None] * (2 * W)
    for r, p in enumerate(parts):
        a, b = p.chunk(2, dim=dim)
        chunks[r], chunks[2 * W - 1 - r] = a, b
    return torch.cat(chunks, dim=dim)


# ------------------------------------------------------------------------------------------------ block math
def _block_fwd(q, k, v, causal, scale):
    """q [B,L,Hq,D], k/v [B,L,Hkv,D] -> (o fp32 [B,L,Hq,D], lse fp32 [B,Hq,L])."""
    o, lse = flash_attn_with_lse(q, k, v, causal=causal, scale=scale)
    return o.float(), lse.float()


def _merge(o, lse, o_blk, lse_blk):
    """Combine two partial attentions over disjoint key sets (fp32)."""
    if o is None:
        return o_blk, lse_blk
    new = torch.logaddexp(lse, lse_blk)
    w_old = torch.exp(lse - new).transpose(1, 2).unsqueeze(-1)
    w_new = torch.exp(lse_blk - new).transpose(1, 2).unsqueeze(-1)
    return o * w_old + o_blk * w_new, new


def _block_bwd(do, q, k, v, o, lse, causal, scale):
    """Gradients of one block given the globally-normalised O / LSE. Returns (dq, dk, dv) in q/k/v dtypes."""
    if use_native(q) and q.dtype == torch.bfloat16:
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ext().flash_attn_bwd(do.contiguous(), q, k, v, o.contiguous(), lse.contiguous(), dq, dk, dv, scale, causal)
        return dq, dk, dv
    B, L, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    dof, of = do.float().transpose(1, 2), o.float().transpose(1, 2)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(L, L, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    p = torch.exp(s - lse.float().unsqueeze(-1))
    dvf = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dqf = torch.matmul(ds, kf)
    dkf = torch.matmul(ds.transpose(-1, -2), qf)
    dkf = dkf.view(B, Hkv, rep, L, D).sum(2)
    dvf = dvf.view(B, Hkv, rep, L, D).sum(2)
    return dqf.transpose(1, 2).to(q.dtype), dkf.transpose(1, 2).to(k.dtype), dvf.transpose(1, 2).to(v.dtype)


def _chunk_plan(world: int, rank: int):
    """Global chunk ids of this rank's two query chunks."""
    return [rank, 2 * world - 1 - rank]


def _attend_chunk(qc, c, kv_chunks, scale):
    """Attention of query chunk with global id `c` against visible key chunks (ids < c full, == c causal)."""
    o, lse = _block_fwd(qc, kv_chunks[c][0], kv_chunks[c][1], True, scale)
    if c > 0:
        B = qc.shape[0]
        ks = torch.cat([kv_chunks[j][0] for j in range(c)], 0)
        vs = torch.cat([kv_chunks[j][1] for j in range(c)], 0)
        qs = qc.repeat(c, 1, 1, 1)
        of, lf = _block_fwd(qs, ks, vs, False, scale)
        # merge the c full blocks (stacked on batch) then the diagonal
        lf = lf.view(c, B, *lf.shape[1:])
        of = of.view(c, B, *of.shape[1:])
        lall = torch.logsumexp(lf, dim=0)
        w = torch.exp(lf - lall.unsqueeze(0)).transpose(2, 3).unsqueeze(-1)  # [c,B,L,Hq,1]
        o_full = (of * w).sum(0)
        o, lse = _merge(o, lse, o_full, lall)
    return o, lse


def _gather_kv_chunks(k, v, group):
    """All-gather local K,V ([B,2L,Hkv,D]) and index them by global chunk id."""
    W = comm.group_size(group)
    kv = torch.stack([k, v], 0)  # one collective for both
    g = comm.all_gather_dim(kv.contiguous(), 2, group)  # [2, B, W*2L, Hkv, D] in rank order
    gk, gv = g[0], g[1]
    L = k.shape[1] // 2
    chunks = [None] * (2 * W)
    for j in range(W):
        a = slice(j * 2 * L, j * 2 * L + L)
        b = slice(j * 2 * L + L, (j + 1) * 2 * L)
        chunks[j] = (gk[:, a], gv[:, a])
        chunks[2 * W - 1 - j] = (gk[:, b], gv[:, b])
    return chunks, gk, gv


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, scale, strategy):
        W, r = comm.group_size(group), comm.group_rank(group)
        L = q.shape[1] // 2
        if strategy == "alltoall" and W > 1:
            outs, gk, gv = _ring_forward(q, k, v, group, scale)
        else:
            chunks, gk, gv = _gather_kv_chunks(k, v, group)
            outs = [_attend_chunk(q[:, i * L : (i + 1) * L], c, chunks, scale) for i, c in enumerate(_chunk_plan(W, r))]
        o = torch.cat([x[0] for x in outs], 1).to(q.dtype)
        lse = torch.cat([x[1] for x in outs], 2).contiguous()
        ctx.save_for_backward(q, gk, gv, o, lse)
        ctx.group, ctx.scale, ctx.kshape = group, scale, k.shape
        return o

    @staticmethod
    def backward(ctx, do):
        q, gk, gv, o, lse = ctx.saved_tensors
        group, scale = ctx.group, ctx.scale
        W, r = comm.group_size(group), comm.group_rank(group)
        L = q.shape[1] // 2
        do = do.contiguous()
        # chunk views into the gathered K/V and matching gradient accumulators (fp32)
        dgk = torch.zeros(gk.shape, dtype=torch.float32, device=gk.device)
        dgv = torch.zeros(gv.shape, dtype=torch.float32, device=gv.device)

        def chunk_slice(cid):
            j = cid if cid < W else 2 * W - 1 - cid
            base = j * 2 * L + (0 if cid < W else L)
            return slice(base, base + L)

        dq = torch.empty_like(q)
        for i, c in enumerate(_chunk_plan(W, r)):
            qs = slice(i * L, (i + 1) * L)
            qc, doc, oc = q[:, qs], do[:, qs], o[:, qs]
            lc = lse[:, :, qs].contiguous()
            sl = chunk_slice(c)
            dqc, dkc, dvc = _block_bwd(doc, qc, gk[:, sl], gv[:, sl], oc, lc, True, scale)
            dq_acc = dqc.float()
            dgk[:, sl] += dkc.float()
            dgv[:, sl] += dvc.float()
            if c > 0:
                B = q.shape[0]
                ks = torch.cat([gk[:, chunk_slice(j)] for j in range(c)], 0)
                vs = torch.cat([gv[:, chunk_slice(j)] for j in range(c)], 0)
                dqs, dks, dvs = _block_bwd(doc.repeat(c, 1, 1, 1), qc.repeat(c, 1, 1, 1), ks, vs,
                                           oc.repeat(c, 1, 1, 1), lc.repeat(c, 1, 1), False, scale)
                dq_acc += dqs.float().view(c, B, *dqs.shape[1:]).sum(0)
                for j in range(c):
                    dgk[:, chunk_slice(j)] += dks[j * B : (j + 1) * B].float()
                    dgv[:, chunk_slice(j)] += dvs[j * B : (j + 1) * B].float()
            dq[:, qs] = dq_acc.to(q.dtype)
        dkv = torch.stack([dgk, dgv], 0)
        dkv = comm.reduce_scatter_dim(dkv, 2, group)  # sum contributions of all ranks, keep own [B,2L] rows
        return dq, dkv[0].to(q.dtype), dkv[1].to(q.dtype), None, None, None


def _global_rank(group, r):
    return r if group is None else dist.get_global_rank(group, r)


def _ring_forward(q, k, v, group, scale):
    """Forward with K/V streamed around a P2P ring (overlap the next transfer with the current blocks)."""
    W, r = comm.group_size(group), comm.group_rank(group)
    L = q.shape[1] // 2
    plan = _chunk_plan(W, r)
    acc = [(None, None), (None, None)]
    cur = torch.stack([k, v], 0).contiguous()
    nxt = torch.empty_like(cur)
    # every chunk that passes through is kept in rank order (same layout as the all-gather) for the backward
    gkv = torch.empty((2, k.shape[0], W * 2 * L) + tuple(k.shape[2:]), dtype=k.dtype, device=k.device)
    send_to, recv_from = (r + 1) % W, (r - 1) % W
    for step in range(W):
        reqs = []
        if step < W - 1:
            ops = [dist.P2POp(dist.isend, cur, _global_rank(group, send_to), group),
                   dist.P2POp(dist.irecv, nxt, _global_rank(group, recv_from), group)]
            reqs = dist.batch_isend_irecv(ops)
        owner = (r - step) % W
        gkv[:, :, owner * 2 * L : (owner + 1) * 2 * L] = cur
        owned = {owner: (cur[0][:, :L], cur[1][:, :L]), 2 * W - 1 - owner: (cur[0][:, L:], cur[1][:, L:])}
        for i, c in enumerate(plan):
            qc = q[:, i * L : (i + 1) * L]
            for cid, (kc, vc) in owned.items():
                if cid > c:
                    continue
                ob, lb = _block_fwd(qc, kc, vc, cid == c, scale)
                acc[i] = _merge(acc[i][0], acc[i][1], ob, lb)
        for req in reqs:
            req.wait()
        cur, nxt = nxt, cur
    return acc, gkv[0], gkv[1]


def ring_attention(q, k, v, group, scale: Optional[float] = None, strategy: str = "allgather"):
    """Causal attention of this rank's zig-zag shard against the full (distributed) sequence.
    q [B, S_local, Hq, D], k/v [B, S_local, Hkv, D] → O [B, S_local, Hq, D]."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if q.shape[1] % 2:
        raise ValueError("context parallel: local sequence must hold two equal zig-zag chunks")
    return _RingAttnFn.apply(q, k, v, group, scale, strategy)


class RingAttention:
    """`attention_impl` for our attention modules: fused qkv [B,S,Hq+2Hkv,D] → O [B,S,Hq,D]."""

    def __init__(self, group, strategy: str = "allgather"):
        self.group, self.strategy = group, strategy

    def __call__(self, qkv, n_q, n_kv):
        q = qkv[:, :, :n_q]
        k = qkv[:, :, n_q : n_q + n_kv]
        v = qkv[:, :, n_q + n_kv :]
        return ring_attention(q, k, v, self.group, strategy=self.strategy)


def _make_ring_sdpa(group, strategy, original):
    def sdpa(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False, **kw):
        if attn_mask is not None or not is_causal or dropout_p:
            # torch CP has the same restriction: only causal, mask-free attention is ring-sharded
            raise ValueError("context parallel supports causal attention without attn_mask/dropout only")
        o = ring_attention(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2), group, scale, strategy)
        return o.transpose(1, 2)

    return sdpa


@contextlib.contextmanager
def context_parallel(mesh, models, buffers, buffer_seq_dims, no_restore_buffers=frozenset(), strategy: str = "allgather"):
    """Shard `buffers` (zig-zag) along `buffer_seq_dims` over the cp group and route attention through ring
    attention inside the block. Buffers not in `no_restore_buffers` get their full content back on exit."""
    group = mesh.group("cp")
    W, r = comm.group_size(group), comm.group_rank(group)
    saved = []
    seq_len = None
    for buf, dim in zip(buffers, buffer_seq_dims):
        seq_len = buf.shape[dim] if seq_len is None else seq_len
        local = zigzag_shard(buf, dim, W, r)
        if not any(buf is x for x in no_restore_buffers):
            saved.append((buf, buf.data))
        buf.data = local
    impl = RingAttention(group, strategy)
    patched_modules, patched_models = [], []
    for m in models:
        inner = getattr(m, "module", m)
        for mod in inner.modules():
            if hasattr(mod, "attention_impl"):
                patched_modules.append((mod, mod.attention_impl))
                mod.attention_impl = impl
        if seq_len is not None and hasattr(inner, "config"):
            B = buffers[0].shape[0] if buffers and buffers[0].dim() > 1 else 1
            pos = zigzag_indices(seq_len, W, r, device=buffers[0].device).unsqueeze(0).expand(B, -1).contiguous()
            patched_models.append((inner, getattr(inner, "_cp_position_ids", None), getattr(inner, "_cp_seq_len", None)))
            inner._cp_position_ids = pos
            inner._cp_seq_len = seq_len
    sdpa_orig = torch.nn.functional.scaled_dot_product_attention
    torch.nn.functional.scaled_dot_product_attention = _make_ring_sdpa(group, strategy, sdpa_orig)
    try:
        yield
    finally:
        torch.nn.functional.scaled_dot_product_attention = sdpa_orig
        for mod, old in patched_modules:
            mod.attention_impl = old
        for inner, pos, sl in patched_models:
            inner._cp_position_ids, inner._cp_seq_len = pos, sl
        for buf, full in saved:
            buf.data = full
