"""Ulysses sequence parallelism (DeepSpeed ALST semantics) over the `sp` mesh dimension.

Parity target: `/root/reference/src/accelerate/accelerator.py:2357-2409,2458-2476` (`UlyssesSPAttentionHF` +
`UlyssesSPDataLoaderAdapter` from DeepSpeed ≥ 0.18.2) and `examples/alst_ulysses_sequence_parallelism/sp-alst.py`
(loss re-aggregation weighted by each rank's valid-token count).

Mechanics:
  * every rank holds a contiguous 1/sp slice of the sequence (the data-loader adapter cuts `input_ids`,
    `shift_labels` — labels shifted on the *full* sequence first — and `position_ids`);
  * attention: one RCCL all-to-all turns [B, S/sp, heads, D] into [B, S, heads/sp, D] (q, k and v packed into a
    single exchange, grouped per destination so each rank gets whole q/k/v head groups), the HIP flash-attention
    kernel runs on the full sequence for its head group, and one all-to-all brings the output back. On xGMI the
    all-to-all drives all 7 links at once (fully connected), unlike a ring.
  * GQA with fewer kv heads than sp ranks: kv heads are replicated so each rank gets one.
  * parameters are replicated over sp: the FSDP engine shards over `dp_shard × cp × sp`, so gradients are averaged
    across sp exactly like across data-parallel ranks.
"""

from __future__ import annotations

import contextlib
import math
from typing import Optional

import torch
import torch.distributed as dist

from ..ops.fused import attention_reference, flash_attention_qkv
from . import comm


def _pack_heads(q, k, v, W):
    """[B,S,h,D] x3 → [B,S,W,(hq+2hkv)/W,D] with q|k|v head groups per destination rank."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    if Hkv < W:
        if W % Hkv:
            raise ValueError(f"Ulysses: sp={W} must be a multiple of the kv head count {Hkv}")
        k = k.repeat_interleave(W // Hkv, dim=2)
        v = v.repeat_interleave(W // Hkv, dim=2)
        Hkv = W
    if Hq % W or Hkv % W:
        raise ValueError(f"Ulysses: sp={W} must divide the head counts (q={Hq}, kv={Hkv})")
    parts = [t.reshape(B, S, W, t.shape[2] // W, D) for t in (q, k, v)]
    return torch.cat(parts, dim=3), Hq // W, Hkv // W


def ulysses_attention(q, k, v, group, causal: bool = True, scale: Optional[float] = None):
    """q [B, S/sp, Hq, D], k/v [B, S/sp, Hkv, D] (this rank's contiguous sequence slice) → O [B, S/sp, Hq, D]."""
    W = comm.group_size(group)
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if W == 1:
        return _local_attention(q, k, v, q.shape[2], k.shape[2], causal, scale)
    packed, hq, hkv = _pack_heads(q, k, v, W)  # [B, S_l, W, h_loc, D]
    # scatter the rank dim (2), gather the sequence (1): → [B, S, 1, h_loc, D]
    full = comm.all_to_all(packed.contiguous(), 2, 1, group).squeeze(2)
    o = _local_attention(full[:, :, :hq], full[:, :, hq : hq + hkv], full[:, :, hq + hkv :], hq, hkv, causal, scale, fused=full)
    # back: scatter the sequence, gather heads
    o = comm.all_to_all(o.unsqueeze(2).contiguous(), 1, 2, group)  # [B, S_l, W, hq, D]
    return o.reshape(o.shape[0], o.shape[1], W * hq, o.shape[-1])


def _local_attention(q, k, v, hq, hkv, causal, scale, fused=None):
    if fused is not None and fused.shape[-1] == 128 and fused.dtype == torch.bfloat16 and fused.is_cuda:
        return flash_attention_qkv(fused, hq, hkv, causal=causal, scale=scale)
    return attention_reference(q, k, v, causal=causal, scale=scale)


class UlyssesAttention:
    """`attention_impl` for our attention modules (fused qkv [B, S/sp, Hq+2Hkv, D])."""

    def __init__(self, group):
        self.group = group

    def __call__(self, qkv, n_q, n_kv):
        return ulysses_attention(qkv[:, :, :n_q], qkv[:, :, n_q : n_q + n_kv], qkv[:, :, n_q + n_kv :], self.group)


def install_ulysses(model, group, seq_len: Optional[int] = None):
    """Route every attention of `model` through Ulysses (our models via `attention_impl`). HF models get
    `scaled_dot_product_attention` patched inside `ulysses_sdpa_context`."""
    impl = UlyssesAttention(group)
    n = 0
    for mod in model.modules():
        if hasattr(mod, "attention_impl"):
            mod.attention_impl = impl
            n += 1
    model._ulysses_group = group
    model._seq_parallel_factor = comm.group_size(group)  # RoPE tables must cover the full (unsharded) length
    return n


@contextlib.contextmanager
def ulysses_sdpa_context(group):
    orig = torch.nn.functional.scaled_dot_product_attention

    def sdpa(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, scale=None, enable_gqa=False, **kw):
        if attn_mask is not None or dropout_p:
            raise ValueError("Ulysses SP supports mask-free attention without dropout")
        o = ulysses_attention(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2), group, is_causal, scale)
        return o.transpose(1, 2)

    torch.nn.functional.scaled_dot_product_attention = sdpa
    try:
        yield
    finally:
        torch.nn.functional.scaled_dot_product_attention = orig


class UlyssesSPDataLoaderAdapter:
    """Cuts each batch's sequence dimension into `sp_world_size` contiguous slices and keeps this rank's slice.

    `labels` are turned into `shift_labels` on the full sequence *before* cutting (so the slice boundaries lose no
    target), and `position_ids` are added so RoPE sees global positions."""

    def __init__(self, dl, sp_rank: int, sp_group, sp_world_size: int, device=None, seq_keys=("input_ids", "labels", "attention_mask", "position_ids", "shift_labels")):
        self.dl, self.sp_rank, self.sp_group, self.sp_world_size, self.device = dl, sp_rank, sp_group, sp_world_size, device
        self.seq_keys = seq_keys

    def __len__(self):
        return len(self.dl)

    def __getattr__(self, name):
        if name in ("dl", "sp_rank", "sp_group", "sp_world_size", "device", "seq_keys"):
            raise AttributeError(name)
        return getattr(self.dl, name)

    def _shard(self, batch: dict) -> dict:
        batch = dict(batch)
        ids = batch["input_ids"]
        B, S = ids.shape
        W, r = self.sp_world_size, self.sp_rank
        if S % W:
            raise ValueError(f"Ulysses SP: sequence length {S} not divisible by sp={W}; pad the batch")
        if "shift_labels" not in batch and "labels" in batch:
            lab = batch.pop("labels")
            sl = torch.full_like(lab, -100)
            sl[:, :-1] = lab[:, 1:]
            batch["shift_labels"] = sl
        if "position_ids" not in batch:
            batch["position_ids"] = torch.arange(S, device=ids.device).unsqueeze(0).expand(B, -1)
        batch.pop("attention_mask", None)  # causal, mask-free (packed) sequences only
        L = S // W
        for key in self.seq_keys:
            if key in batch and torch.is_tensor(batch[key]) and batch[key].dim() >= 2 and batch[key].shape[1] == S:
                batch[key] = batch[key][:, r * L : (r + 1) * L].contiguous()
        return batch

    def __iter__(self):
        for batch in self.dl:
            yield self._shard(batch)


def sp_loss_aggregate(loss: torch.Tensor, n_valid: torch.Tensor, group) -> torch.Tensor:
    """Token-weighted mean of per-rank mean losses across sp (differentiable; ALST example semantics)."""
    w = n_valid.to(loss.dtype)
    num = comm.reduce_from_group((loss * w).reshape(1), group)
    den = comm.all_reduce_(w.detach().reshape(1).clone(), group)
    return (num / den).reshape(())
