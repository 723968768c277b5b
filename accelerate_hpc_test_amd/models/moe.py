"""Mixture-of-Experts layer (top-k routing, dropless) with optional expert parallelism over RCCL all-to-all.

Used by `models/mixtral.py` (BASELINE config "Mixtral 8×7B FSDP2 + fp8"). The reference has no native MoE/EP
(it defers to Megatron `expert_model_parallel_size`, `/root/reference/src/accelerate/utils/dataclasses.py:2403-2408`,
and DeepSpeed ZeRO-3 leaf modules `:1514-1532`); SURVEY §2.2 C25 asks for RCCL all-to-all dispatch/combine + grouped
expert GEMMs. Design:

  * experts are stored *stacked* (`w_gate_up [E, 2I, H]`, `w_down [E, H, I]`) so FSDP flat-shards them like any
    parameter and the backward writes all expert weight-gradients into one preallocated buffer;
  * tokens are sorted by expert once (stable argsort), each expert runs two large hipBLASLt GEMMs on its contiguous
    segment (no per-token work, no capacity padding, no dropped tokens) with the fused SwiGLU kernel between them;
  * gradients for the whole expert group come from one custom autograd op (`_GroupedExpertsFn`) — indexing
    `w[e]` under autograd would materialise an [E, …]-sized zero gradient per expert;
  * expert parallelism (`ep_group` of size W): rank r owns experts [r·E/W, (r+1)·E/W). Tokens go to their expert's
    owner with one variable-size all-to-all (xGMI: direct, all 7 links), come back with the inverse all-to-all.
    Expert params are then excluded from FSDP (they are already sharded) and their grads are scaled 1/W (each rank's
    loss is its local mean, exactly like the data-parallel average applied to the dense params).
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..ops._ext import ext, use_native
from ..parallel import comm


def _swiglu_fwd(h):
    if use_native(h) and h.dtype == torch.bfloat16 and (h.shape[-1] // 2) % 8 == 0:
        return ext().swiglu_fwd(h.contiguous())
    g, u = h.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(h.dtype)


def _swiglu_bwd(h, da):
    if use_native(h) and h.dtype == torch.bfloat16 and (h.shape[-1] // 2) % 8 == 0:
        return ext().swiglu_bwd(h.contiguous(), da.contiguous())
    g, u = h.float().chunk(2, dim=-1)
    s = torch.sigmoid(g)
    silu = g * s
    daf = da.float()
    dg = daf * u * (s * (1 + g * (1 - s)))
    du = daf * silu
    return torch.cat([dg, du], -1).to(h.dtype)


_FP8_ROW_PAD = 256  # the 256x256-tile fp8 GEMM (csrc/kernels/fp8.hip v2) needs M, N % 256 and K % 128


def _pad_rows(t, rows):
    if t.shape[0] == rows:
        return t.contiguous()
    out = t.new_zeros(rows, t.shape[1])
    out[: t.shape[0]] = t
    return out


def _fp8_ok(x, recipe, dims):
    from ..ops.fp8 import _gemm_ok

    return recipe is not None and x.is_cuda and use_native(x) and x.dtype == torch.bfloat16 and all(
        _gemm_ok(128, d, 64) for d in dims
    )


class _GroupedExpertsFn(torch.autograd.Function):
    """y_e = down_e(swiglu(gate_up_e(x_e))) for contiguous token segments x_e (sizes `counts`).

    bf16: hipBLASLt GEMMs on the raw segments. fp8 (a recipe is attached): each segment is zero-padded to a multiple
    of 256 rows so all six GEMMs per expert (2 fwd, 2 dgrad, 2 wgrad) run on the 256² MX-fp8 MFMA kernel; zero rows add
    nothing to the wgrad sums and the padded output rows are dropped. Forward operands are e4m3, gradients e5m2
    (HYBRID), per-expert per-tensor scales, and the transposed fp8 copies the backward needs come out of the same
    cast kernel as the forward copies.
    """

    @staticmethod
    def forward(ctx, x, w_gu, w_down, counts, recipe):
        y = torch.empty(x.shape[0], w_down.shape[1], dtype=x.dtype, device=x.device)
        fp8 = _fp8_ok(x, recipe, (w_gu.shape[1], w_gu.shape[2], w_down.shape[2]))
        saved = []
        off = 0
        for e, c in enumerate(counts):
            if c == 0:
                saved.append(None)
                continue
            xe = x[off : off + c]
            if fp8:
                y[off : off + c], st = _fp8_expert_fwd(xe, w_gu[e], w_down[e], recipe, e)
                saved.append(st)
            else:
                h = xe @ w_gu[e].t()
                y[off : off + c] = _swiglu_fwd(h) @ w_down[e].t()
                saved.append(h)
            off += c
        ctx.save_for_backward(x, w_gu, w_down)
        ctx.saved, ctx.counts, ctx.recipe, ctx.fp8 = saved, counts, recipe, fp8
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_gu, w_down = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dw_gu = torch.empty_like(w_gu)  # every expert's slice is written below (zeroed when it got no tokens)
        dw_down = torch.empty_like(w_down)
        off = 0
        for e, c in enumerate(ctx.counts):
            if c == 0:
                dw_gu[e].zero_()
                dw_down[e].zero_()
                continue
            xe, dye = x[off : off + c], dy[off : off + c]
            if ctx.fp8:
                dx[off : off + c] = _fp8_expert_bwd(dye, ctx.saved[e], ctx.recipe, e, dw_gu[e], dw_down[e])
            else:
                h = ctx.saved[e]
                a = _swiglu_fwd(h)
                torch.mm(dye.t(), a, out=dw_down[e]) if dw_down.dtype == dye.dtype else dw_down[e].copy_(dye.t() @ a)
                dh = _swiglu_bwd(h, dye @ w_down[e])
                torch.mm(dh.t(), xe, out=dw_gu[e]) if dw_gu.dtype == dh.dtype else dw_gu[e].copy_(dh.t() @ xe)
                dx[off : off + c] = dh @ w_gu[e]
            off += c
        ctx.saved = None
        return dx, dw_gu, dw_down, None, None


def _fp8_expert_fwd(xe, w_gu, w_down, recipe, e):
    from ..ops.fp8 import E4M3_MAX, cast, gemm

    c = xe.shape[0]
    cp = (c + _FP8_ROW_PAD - 1) // _FP8_ROW_PAD * _FP8_ROW_PAD
    xp = _pad_rows(xe, cp)
    sx = recipe.scale(f"x{e}", xp, E4M3_MAX)
    sgu = recipe.scale(f"wgu{e}", w_gu, E4M3_MAX)
    x8, x8t = cast(xp, sx, False, transpose=True)
    gu8, gu8t = cast(w_gu.contiguous(), sgu, False, transpose=True)
    h = gemm(x8, gu8, sx, sgu, None, torch.bfloat16)  # [cp, 2I]; padded rows stay 0
    a = _swiglu_fwd(h)
    sa = recipe.scale(f"a{e}", a, E4M3_MAX)
    sd = recipe.scale(f"wd{e}", w_down, E4M3_MAX)
    a8, a8t = cast(a, sa, False, transpose=True)
    d8, d8t = cast(w_down.contiguous(), sd, False, transpose=True)
    yp = gemm(a8, d8, sa, sd, None, torch.bfloat16)
    return yp[:c], (h, x8t, gu8t, a8t, d8t, sx, sgu, sa, sd)


def _fp8_expert_bwd(dye, st, recipe, e, dw_gu_e, dw_down_e):
    from ..ops.fp8 import E4M3_MAX, E5M2_MAX, cast, gemm

    h, x8t, gu8t, a8t, d8t, sx, sgu, sa, sd = st
    c, cp = dye.shape[0], h.shape[0]
    e5 = recipe.grad_e5m2()
    gmax = E5M2_MAX if e5 else E4M3_MAX
    dyp = _pad_rows(dye.to(torch.bfloat16), cp)
    sg = recipe.scale(f"gy{e}", dyp, gmax)
    dy8, dy8t = cast(dyp, sg, e5, transpose=True)
    gemm(dy8t, a8t, sg, sa, None, out=dw_down_e)
    da = gemm(dy8, d8t, sg, sd, None, torch.bfloat16)  # [cp, I]
    dh = _swiglu_bwd(h, da)  # [cp, 2I]
    sh = recipe.scale(f"gh{e}", dh, gmax)
    dh8, dh8t = cast(dh, sh, e5, transpose=True)
    gemm(dh8t, x8t, sh, sx, None, out=dw_gu_e)
    return gemm(dh8, gu8t, sh, sgu, None, torch.bfloat16)[:c]


class MoEExperts(nn.Module):
    """Stacked SwiGLU experts. With expert parallelism only the local slice [E_local, ...] is materialised."""

    def __init__(self, num_experts: int, hidden: int, intermediate: int):
        super().__init__()
        self.num_experts = num_experts
        self.w_gate_up = nn.Parameter(torch.empty(num_experts, 2 * intermediate, hidden))
        self.w_down = nn.Parameter(torch.empty(num_experts, hidden, intermediate))
        self.fp8_recipe = None

    def forward(self, x_sorted, counts):
        w_gu, w_down = self.w_gate_up, self.w_down
        if w_gu.dtype != x_sorted.dtype:
            w_gu, w_down = w_gu.to(x_sorted.dtype), w_down.to(x_sorted.dtype)
        return _GroupedExpertsFn.apply(x_sorted, w_gu, w_down, counts, self.fp8_recipe)


class MoELayer(nn.Module):
    def __init__(self, hidden: int, intermediate: int, num_experts: int, top_k: int, norm_topk: bool = True):
        super().__init__()
        self.num_experts, self.top_k, self.norm_topk = num_experts, top_k, norm_topk
        self.gate = nn.Linear(hidden, num_experts, bias=False)
        self.experts = MoEExperts(num_experts, hidden, intermediate)
        self.ep_group = None
        self.last_router_logits = None

    # --------------------------------------------------------------------------------------------- EP setup
    def shard_experts(self, group, device=None) -> bool:
        """Keep experts [r·E/W, (r+1)·E/W) of this rank on `device`. Returns True when the weights still need
        initialisation (they were on the meta device)."""
        W, r = comm.group_size(group), comm.group_rank(group)
        if self.num_experts % W:
            raise ValueError(f"expert parallel: {self.num_experts} experts not divisible by ep={W}")
        El = self.num_experts // W
        was_meta = False
        for name in ("w_gate_up", "w_down"):
            p = getattr(self.experts, name)
            local = p.data[r * El : (r + 1) * El]
            if p.device.type == "meta":
                was_meta = True
                data = torch.empty(local.shape, dtype=p.dtype, device=device if device is not None else "meta")
            else:
                data = local.clone().to(device) if device is not None else local.clone()
            newp = nn.Parameter(data, requires_grad=p.requires_grad)
            newp._ep_spec = (group, W)
            setattr(self.experts, name, newp)
            scale = 1.0 / W
            newp.register_hook(lambda g, s=scale: g * s)
        self.ep_group = group
        return was_meta

    # --------------------------------------------------------------------------------------------- forward
    def forward(self, x):
        shape = x.shape
        t = x.reshape(-1, shape[-1])
        T = t.shape[0]
        logits = self.gate(t)
        self.last_router_logits = logits
        probs = torch.softmax(logits.float(), dim=-1)
        w, idx = torch.topk(probs, self.top_k, dim=-1)
        if self.norm_topk:
            w = w / w.sum(-1, keepdim=True)
        w = w.to(t.dtype)
        flat_e = idx.reshape(-1)
        order = torch.argsort(flat_e, stable=True)
        src_tok = order // self.top_k
        w_sorted = w.reshape(-1)[order]
        x_sorted = t.index_select(0, src_tok)
        if self.ep_group is None or comm.group_size(self.ep_group) == 1:
            counts = torch.bincount(flat_e, minlength=self.num_experts).tolist()
            y_sorted = self.experts(x_sorted, counts)
        else:
            y_sorted = self._ep_experts(x_sorted, flat_e[order])
        out = torch.zeros_like(t).index_add_(0, src_tok, y_sorted * w_sorted.unsqueeze(-1))
        return out.view(shape)

    def _ep_experts(self, x_sorted, e_sorted):
        group = self.ep_group
        W = comm.group_size(group)
        El = self.num_experts // W
        dest = e_sorted // El
        send_counts = torch.bincount(dest, minlength=W)
        recv_counts = torch.empty_like(send_counts)
        if dist.get_backend(group) == "gloo":
            gathered = [torch.empty_like(send_counts) for _ in range(W)]
            dist.all_gather(gathered, send_counts, group=group)
            me = comm.group_rank(group)
            recv_counts = torch.stack([g[me] for g in gathered])
        else:
            dist.all_to_all_single(recv_counts, send_counts, group=group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        x_recv = comm.all_to_all_var(x_sorted, sc, rc, group)
        e_recv = comm.all_to_all_varlen((e_sorted % El).unsqueeze(-1).to(torch.float32), sc, rc, group).squeeze(-1).long()
        order2 = torch.argsort(e_recv, stable=True)
        counts2 = torch.bincount(e_recv, minlength=El).tolist()
        y_local_sorted = self.experts(x_recv.index_select(0, order2), counts2)
        inv = torch.empty_like(order2)
        inv[order2] = torch.arange(order2.numel(), device=order2.device)
        y_recv = y_local_sorted.index_select(0, inv)
        return comm.all_to_all_var(y_recv, rc, sc, group)


def load_balancing_loss(router_logits: list, num_experts: int, top_k: int) -> torch.Tensor:
    """Switch-style auxiliary loss (HF `load_balancing_loss_func`): E · Σ_e f_e · P_e over all layers' tokens."""
    logits = torch.cat([l.float() for l in router_logits], 0)
    probs = torch.softmax(logits, -1)
    _, sel = torch.topk(probs, top_k, -1)
    mask = F.one_hot(sel, num_experts).float()  # [T, k, E]
    tokens_per_expert = mask.mean(0)  # [k, E]
    prob_per_expert = probs.mean(0)  # [E]
    return (tokens_per_expert * prob_per_expert.unsqueeze(0)).sum() * num_experts
