"""Context parallelism: ring attention over the `cp` mesh dimension for long sequences.

Parity target: `/root/reference/src/accelerate/accelerator.py:1641-1654,4075-4140` (`maybe_context_parallel`, which
wraps torch's experimental `context_parallel`: buffers sharded along their sequence dim, SDPA swapped for a ring
variant, K/V rotated by all-gather (default) or all-to-all), and `docs/source/concept_guides/context_parallelism.md`.

MI355X design:
  * Load-balanced ("zig-zag") layout: the sequence is cut into 2·cp chunks and rank r keeps chunks r and
    2·cp-1-r, so every rank does the same causal work (2·cp+1 chunk-blocks).
  * "allgather" (default): K,V are all-gathered straight into global sequence order in two halves (`_KVGather`); each
    query chunk then needs exactly ONE HIP flash-attention call against its whole causal K/V prefix — the kernel
    takes Sk > Sq with a bottom-right-aligned causal mask — so there are no per-block calls, no repeated queries and
    no LSE merges. The second half's all-gather is in flight while the rank's first (shorter-prefix) chunk computes.
  * "alltoall": K,V stream around a P2P ring (`batch_isend_irecv`) overlapped with the block computation in
    forward, partial outputs merged in place in fp32 with the LSE rule.
  * Backward re-gathers K,V (no global K/V is kept between forward and backward: saved activations stay O(local)),
    runs one flash backward per query chunk with the *global* O and LSE, sums dK/dV in one fp32 global-order buffer
    and reduce-scatters it to the owners in one collective. `cp_transient_bytes` gives the per-layer transient.
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
    """q [B,Lq,Hq,D], k/v [B,Lk,Hkv,D] (Lk >= Lq; causal mask bottom-right aligned) -> (o, lse fp32 [B,Hq,Lq])."""
    return flash_attn_with_lse(q, k, v, causal=causal, scale=scale)


def _merge(o, lse, o_blk, lse_blk):
    """Combine two partial attentions over disjoint key sets (fp32 o, in place on `o`)."""
    if o is None:
        return o_blk.float(), lse_blk.float()
    new = torch.logaddexp(lse, lse_blk)
    w_old = torch.exp(lse - new).transpose(1, 2).unsqueeze(-1)
    w_new = torch.exp(lse_blk - new).transpose(1, 2).unsqueeze(-1)
    return o.mul_(w_old).add_(o_blk.float() * w_new), new


def _block_bwd(do, q, k, v, o, lse, causal, scale):
    """Gradients of attention of q against the K/V prefix k/v (Lk >= Lq, bottom-right causal) given the globally
    normalised O / LSE. Returns (dq, dk, dv) in q/k/v dtypes; dk/dv cover the whole prefix."""
    if use_native(q) and q.dtype == torch.bfloat16:
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ext().flash_attn_bwd(do.contiguous(), q, k, v, o.contiguous(), lse.contiguous(), dq, dk, dv, scale, causal)
        return dq, dk, dv
    B, Lq, Hq, D = q.shape
    Lk, Hkv = k.shape[1], k.shape[2]
    rep = Hq // Hkv
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    kf, vf = kf.repeat_interleave(rep, 1), vf.repeat_interleave(rep, 1)
    dof, of = do.float().transpose(1, 2), o.float().transpose(1, 2)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool, device=q.device).triu(1 + Lk - Lq), float("-inf"))
    p = torch.exp(s - lse.float().unsqueeze(-1))
    dvf = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dqf = torch.matmul(ds, kf)
    dkf = torch.matmul(ds.transpose(-1, -2), qf)
    dkf = dkf.view(B, Hkv, rep, Lk, D).sum(2)
    dvf = dvf.view(B, Hkv, rep, Lk, D).sum(2)
    return dqf.transpose(1, 2).to(q.dtype), dkf.transpose(1, 2).to(k.dtype), dvf.transpose(1, 2).to(v.dtype)


def _chunk_plan(world: int, rank: int):
    """Global chunk ids of this rank's two query chunks."""
    return [rank, 2 * world - 1 - rank]


# ------------------------------------------------------------------------------------------------ K/V gather
class _KVGather:
    """All-gather of every rank's zig-zag K/V into GLOBAL sequence order, in two halves so compute can start early.

    Rank j holds chunks j and 2W-1-j. Gathering every rank's first chunk gives chunks 0..W-1 already in global order
    (rank order == chunk order); gathering the second chunks gives W..2W-1 in reverse chunk order, flipped by one
    copy of that half. The first half is waited for before the rank's first query chunk (global id r < W, whose causal
    prefix lies entirely in it); the second half is issued asynchronously and is in flight during that computation.
    Result: K and V as [B, 2W*L, Hkv, D] (one buffer, K and V stacked on dim 0)."""

    def __init__(self, k, v, group):
        W = comm.group_size(group)
        B, L2, H, D = k.shape
        self.L, self.W, self.group = L2 // 2, W, group
        kv = torch.stack([k, v], 0)  # [2, B, 2L, H, D]
        L = self.L
        first = kv[:, :, :L].movedim(2, 0).contiguous()  # [L, 2, B, H, D]: the gathered dim outermost
        second = kv[:, :, L:].movedim(2, 0).contiguous()
        self.h1 = torch.empty((W * L,) + tuple(first.shape[1:]), dtype=k.dtype, device=k.device)
        self.h2 = torch.empty_like(self.h1)
        self.async_ok = W > 1 and comm.tensor_forms(group, first)
        if W == 1:
            self.h1.copy_(first)
            self.h2.copy_(second)
            self.w2 = None
        elif self.async_ok:
            dist.all_gather_into_tensor(self.h1, first, group=group)
            self.w2 = dist.all_gather_into_tensor(self.h2, second, group=group, async_op=True)
        else:
            self.h1.copy_(comm.all_gather_dim(first, 0, group))
            self.h2.copy_(comm.all_gather_dim(second, 0, group))
            self.w2 = None
        self.full = None

    def prefix(self, n_chunks):
        """K, V of global chunks [0, n_chunks) as [B, n*L, H, D] views."""
        L, W = self.L, self.W
        if n_chunks <= W and self.full is None:
            kv = self.h1[: n_chunks * L]
        else:
            kv = self._full()[: n_chunks * L]
        kv = kv.movedim(0, 2)  # [2, B, n*L, H, D]
        return kv[0], kv[1]

    def _full(self):
        if self.full is None:
            if self.w2 is not None:
                self.w2.wait()
                self.w2 = None
            L, W = self.L, self.W
            # second half arrived as chunks 2W-1, ..., W (rank order): flip the chunk order
            h2 = self.h2.view(W, L, *self.h2.shape[1:]).flip(0).reshape(self.h2.shape)
            self.full = torch.cat([self.h1, h2], 0)
            self.h1 = self.h2 = None
        return self.full


def _rank_order_rows(t, W, L):
    """[B, 2W*L, ...] in global chunk order -> rank order (rank j: chunks j, 2W-1-j), the reduce-scatter layout."""
    idx = torch.cat([torch.cat([torch.arange(j * L, (j + 1) * L), torch.arange((2 * W - 1 - j) * L, (2 * W - j) * L)])
                     for j in range(W)]).to(t.device)
    return t.index_select(1, idx)


class _RingAttnFn(torch.autograd.Function):
    """Causal attention of this rank's two zig-zag query chunks against the distributed sequence.

    Forward ("allgather"): the K/V all-gather (two halves, second one overlapped with the first chunk's compute), then
    ONE flash call per query chunk against its whole causal K/V prefix (bottom-right-aligned mask; no per-block calls,
    no repeated queries, no LSE merge). ("alltoall"): K/V stream around a P2P ring, one block per arriving chunk,
    merged in place in fp32 with the LSE rule, the next transfer overlapped with the current blocks.
    Backward (both): the K/V are re-gathered (nothing of the global K/V is kept between forward and backward: O(local)
    activation memory per layer), one flash backward per query chunk against its prefix, dK/dV summed in one fp32
    global-order buffer and reduce-scattered to their owners in one collective."""

    @staticmethod
    def forward(ctx, q, k, v, group, scale, strategy):
        W, r = comm.group_size(group), comm.group_rank(group)
        L = q.shape[1] // 2
        if strategy == "alltoall" and W > 1:
            outs = _ring_forward(q, k, v, group, scale)
        else:
            g = _KVGather(k, v, group)
            outs = []
            for i, c in enumerate(_chunk_plan(W, r)):  # chunk r (< W) first: it only needs the first half
                kp, vp = g.prefix(c + 1)
                outs.append(_block_fwd(q[:, i * L : (i + 1) * L], kp, vp, True, scale))
            del g
        o = torch.cat([x[0].to(q.dtype) for x in outs], 1)
        lse = torch.cat([x[1].float() for x in outs], 2).contiguous()
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.group, ctx.scale = group, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, scale = ctx.group, ctx.scale
        W, r = comm.group_size(group), comm.group_rank(group)
        L = q.shape[1] // 2
        do = do.contiguous()
        g = _KVGather(k, v, group)
        B, Hkv, D = k.shape[0], k.shape[2], k.shape[3]
        dkv = None  # fp32 [2, B, 2W*L, Hkv, D] in global order, allocated at the longest prefix
        dq = torch.empty_like(q)
        for i, c in sorted(enumerate(_chunk_plan(W, r)), key=lambda x: -x[1]):  # longest prefix first
            qs = slice(i * L, (i + 1) * L)
            kp, vp = g.prefix(c + 1)
            dqc, dkc, dvc = _block_bwd(do[:, qs], q[:, qs], kp, vp, o[:, qs], lse[:, :, qs].contiguous(), True, scale)
            dq[:, qs] = dqc
            n = (c + 1) * L
            if dkv is None:
                dkv = torch.zeros((2, B, 2 * W * L, Hkv, D), dtype=torch.float32, device=q.device)
            dkv[0, :, :n] += dkc.float()
            dkv[1, :, :n] += dvc.float()
            del kp, vp
        del g
        if W > 1:
            dkv = torch.stack([_rank_order_rows(dkv[0], W, L), _rank_order_rows(dkv[1], W, L)], 0)
            dkv = comm.reduce_scatter_dim(dkv, 2, group)  # sum over ranks, keep own [B, 2L] rows
        else:
            dkv = torch.stack([_rank_order_rows(dkv[0], 1, L), _rank_order_rows(dkv[1], 1, L)], 0)
        return dq, dkv[0].to(k.dtype), dkv[1].to(v.dtype), None, None, None


def _global_rank(group, r):
    return r if group is None else dist.get_global_rank(group, r)


def _ring_forward(q, k, v, group, scale):
    """Forward with K/V streamed around a P2P ring (overlap the next transfer with the current blocks). Each arriving
    rank's chunks are attended as blocks (non-causal below the diagonal, causal on it) and merged in place."""
    W, r = comm.group_size(group), comm.group_rank(group)
    L = q.shape[1] // 2
    plan = _chunk_plan(W, r)
    acc = [(None, None), (None, None)]
    cur = torch.stack([k, v], 0).contiguous()
    nxt = torch.empty_like(cur)
    send_to, recv_from = (r + 1) % W, (r - 1) % W
    for step in range(W):
        reqs = []
        if step < W - 1:
            ops = [dist.P2POp(dist.isend, cur, _global_rank(group, send_to), group),
                   dist.P2POp(dist.irecv, nxt, _global_rank(group, recv_from), group)]
            reqs = dist.batch_isend_irecv(ops)
        owner = (r - step) % W
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
    return acc


def cp_transient_bytes(seq_len: int, cp: int, n_q_heads: int, n_kv_heads: int, head_dim: int = 128, batch: int = 1,
                       dtype_bytes: int = 2) -> dict:
    """Peak per-layer transient HBM of this ring attention on one rank (what `_RingAttnFn` allocates beyond its
    inputs / outputs), for sizing long-context runs: forward = the gathered global K/V (two halves, then the flipped
    concatenation: 2x), backward = the same plus one bf16 prefix dK/dV and the fp32 global-order dK/dV accumulator."""
    kv = 2 * batch * seq_len * n_kv_heads * head_dim * dtype_bytes
    fwd = 2 * kv + batch * n_q_heads * (seq_len // cp) * 4
    bwd = 2 * kv + kv + 2 * kv + batch * n_q_heads * (seq_len // cp) * 4 * 2
    return {"forward": fwd, "backward": bwd, "saved_per_layer": 3 * batch * (seq_len // cp) * n_q_heads * head_dim * dtype_bytes}


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
