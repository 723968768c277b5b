"""Mixture-of-Experts layer (top-k routing, dropless) with optional expert parallelism over RCCL all-to-all.

Used by `models/mixtral.py` (BASELINE config "Mixtral 8×7B FSDP2 + fp8"). The reference has no native MoE/EP
(it defers to Megatron `expert_model_parallel_size`, `/root/reference/src/accelerate/utils/dataclasses.py:2403-2408`,
and DeepSpeed ZeRO-3 leaf modules `:1514-1532`); SURVEY §2.2 C25 asks for RCCL all-to-all dispatch/combine + grouped
expert GEMMs. Design:

  * experts are stored *stacked* (`w_gate_up [E, 2I, H]`, `w_down [E, H, I]`) so FSDP flat-shards them like any
    parameter and the backward writes all expert weight-gradients into one preallocated buffer;
  * routing is laid out ON THE DEVICE (`expert_layout`: bincount / cumsum / stable argsort, no `.tolist()`): the
    (token, slot) entries are copied into one buffer where expert e owns rows [seg[e], seg[e+1]) (its count rounded
    up to 64 rows, zero pad); no capacity factor, no dropped tokens;
  * each projection and direction is ONE grouped GEMM launch over the device segment table
    (csrc/kernels/grouped_gemm.hip, bf16 or MX-fp8 MFMA): forward gate_up + down, backward 2 dgrad + 2
    weight-gradient GEMMs (K-segmented), with the fused SwiGLU kernels between them — no per-expert launch loop;
  * gradients for the whole expert group come from one custom autograd op (`_GroupedExpertsFn`) — indexing
    `w[e]` under autograd would materialise an [E, …]-sized zero gradient per expert;
  * expert parallelism (`ep_group` of size W): rank r owns experts [r·E/W, (r+1)·E/W). Tokens go to their expert's
    owner with one variable-size all-to-all (xGMI: direct, all 7 links), come back with the inverse all-to-all. The
    only other exchange is one [E] per-expert count all-to-all (its host copy = the split sizes, the single host
    sync per MoE layer); receivers derive each row's local expert from those counts, so no ids travel.
    Expert params are then excluded from FSDP (they are already sharded) and their grads are scaled 1/W (each rank's
    loss is its local mean, exactly like the data-parallel average applied to the dense params).
"""

from __future__ import annotations

import os
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


# every expert's segment of the routed-token buffer starts at a multiple of 128 rows: the asm grouped GEMM's 128-byte
# K-tiles then never straddle two experts in the fp8 weight-gradient product (mode 2 reduces over tokens)
SEG_ALIGN = 128


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def expert_layout(flat_e: torch.Tensor, num_experts: int, align: int = SEG_ALIGN):
    """Device-side routing layout (no host synchronisation): for the (token, slot) entries sorted stably by expert,
    `dest[j]` is entry j's row in a buffer where expert e owns rows [seg[e], seg[e + 1]) — its token count rounded
    up to `align` (the pad rows stay zero). `R`, the buffer's row count, is a host-side bound that does not depend on
    the routing: N + (align - 1) * E, rounded up to 256, plus 256 rows of slack so that a 256-row tile of the last
    expert's segment stays inside the buffer (the asm grouped GEMM reads whole tiles, rows past a segment unused)."""
    N = flat_e.numel()
    counts = torch.bincount(flat_e, minlength=num_experts)
    padded = (counts + align - 1) // align * align
    seg = torch.zeros(num_experts + 1, dtype=torch.int32, device=flat_e.device)
    seg[1:] = torch.cumsum(padded, 0)
    order = torch.argsort(flat_e, stable=True)
    e_sorted = flat_e[order]
    start = torch.cumsum(counts, 0) - counts
    dest = seg[:-1].long()[e_sorted] + (torch.arange(N, device=flat_e.device) - start[e_sorted])
    R = _round_up(N + (align - 1) * num_experts, 256) + 256
    return order, dest, seg, R


_ONES = {}


def _ones(n, device):
    key = (n, str(device))
    if key not in _ONES:
        _ONES[key] = torch.ones(n, dtype=torch.float32, device=device)
    return _ONES[key]


def _native_ok(x, *dims):
    return x.is_cuda and use_native(x) and x.dtype == torch.bfloat16 and all(d % 256 == 0 for d in dims)


def _gg_native_ok(a, b, mode, out) -> bool:
    """Shapes / dtypes the grouped MFMA kernel tiles (256x256 output tiles, 256-byte K steps)."""
    if not (a.is_cuda and use_native(a) and a.dtype in (torch.bfloat16, torch.float8_e4m3fn, torch.float8_e5m2)):
        return False
    if out.dtype not in (torch.bfloat16, torch.float32):
        return False
    es = a.element_size()
    if mode == 1:
        return b.shape[1] % 256 == 0 and (a.shape[1] * es) % 256 == 0
    return a.shape[0] % 256 == 0 and b.shape[0] % 256 == 0 and (a.shape[1] * es) % 16 == 0


# Expert GEMM backend: "blaslt" = one hipBLASLt GEMM per expert on its segment (bf16 through torch, fp8 through our
# runner), which needs the segment table on the host: `expert_layout` callers attach it (`seg._acc_bounds`, ONE device
# -> host copy per MoE layer forward; the backward reuses it). Measured at Mixtral-8x7B shapes (tools/bench_moe_gemm.py,
# profiles/r3_moe_gemm.md) 1.2-1.5x faster than the HIP grouped kernel even with that sync. "grouped" = the HIP grouped
# kernel over the device table (no host sync at all), also used whenever no host table is attached.
_MOE_GEMM = os.environ.get("ACCELERATE_MOE_GEMM", "blaslt")
# fp8 expert GEMMs stay on the HIP grouped kernel by default. The fp8 hipBLASLt runner's dynamic-shape mode (one timed
# search per power-of-two bucket of the changing row counts, no per-step searches) brought the per-expert path from
# 14.3k to 34.4k tok/s on Mixtral-8x7B-8l, still under the grouped kernel's 36.2k: a ~2k-row expert GEMM fills half
# the chip (profiles/r3_moe_gemm.md).
_MOE_FP8_BLASLT = os.environ.get("ACCELERATE_MOE_FP8_BLASLT", "0") == "1"
# fp8 expert GEMMs on the asm-scheduled grouped kernel (csrc/kernels/fp8_gemm_asm.hip modes 1 / 2: 256x256 tiles of
# 16x16x128 MFMAs, persistent over (expert, tile) items from the host segment table) when the table is on the host.
_MOE_ASM = os.environ.get("ACCELERATE_MOE_ASM_GEMM", "1") != "0"
# bf16 expert GEMMs on the same asm grouped kernel (its bf16 mode: two 16x16x32 bf16 MFMAs per 128-byte K-tile), by
# product: "fwd" (mode 1 on the stored stacks), "wgrad" (mode 2), "dgrad" (mode 1 on a transposed copy of the stack);
# the others stay on per-expert hipBLASLt. Chosen per product by measurement (profiles/r6_mixtral.md).
_MOE_ASM_BF16 = {k.strip() for k in os.environ.get("ACCELERATE_MOE_ASM_BF16", "fwd,wgrad,dgrad").split(",") if k.strip()}
_F8 = (torch.float8_e4m3fn, torch.float8_e5m2)


def _asm_grouped_mm(a, b, bounds, mode, out, sa, sb, smul, accumulate, kind=None) -> bool:
    """grouped_mm on the asm kernel (fp8 operands, or bf16 ones for the products in ACCELERATE_MOE_ASM_BF16; host
    `bounds`); False when it does not apply. Mode-2 experts with fewer than 256 bytes of K (the kernel's two-K-tile
    minimum) are finished here: zero, or one small product."""
    if not (_MOE_ASM and a.is_cuda and use_native(a)):
        return False
    f8 = a.dtype in _F8 and b.dtype in _F8
    bf = (a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and sa is None and sb is None
          and kind is not None and kind in _MOE_ASM_BF16)
    if not (f8 or bf):
        return False
    if not ext().grouped_gemm_asm(a, b, out, list(bounds), mode, sa, sb, float(smul), bool(accumulate)):
        return False
    if mode == 2:
        es = a.element_size()
        for e in range(len(bounds) - 1):
            lo, hi = bounds[e], bounds[e + 1]
            if (hi - lo) * es >= 256:
                continue
            o = out[e]
            if hi == lo:
                if not accumulate:
                    o.zero_()
                continue
            res = a[:, lo:hi].float() @ b[:, lo:hi].float().t()
            if sa is not None:
                res = res * (sa.reshape(-1)[0] * sb.reshape(-1)[0])
            res = res * smul
            o.add_(res.to(o.dtype)) if accumulate else o.copy_(res)
    return True


def _per_expert_mm(a, b, bounds, mode, out, sa, sb, smul, accumulate) -> bool:
    """grouped_mm as one library GEMM per expert; False when a problem has no library path (then the HIP kernel runs).
    (Spreading the experts over side HIP streams was tried: the Mixtral training step hung in its first warm-up step.)"""
    E = len(bounds) - 1
    fp8 = a.dtype in (torch.float8_e4m3fn, torch.float8_e5m2)
    if fp8 and (sa is None or sb is None or not _MOE_FP8_BLASLT):
        return False
    for e in range(E):
        if not _expert_mm(a, b, bounds, e, mode, out, sa, sb, smul, accumulate, fp8):
            return False
    if mode == 1 and not accumulate and bounds[E] < out.shape[0]:
        out[bounds[E] :].zero_()  # rows past the last segment are defined (zero), as the grouped kernel leaves them
    return True


def _expert_mm(a, b, bounds, e, mode, out, sa, sb, smul, accumulate, fp8) -> bool:
    """Expert e's GEMM of grouped_mm on the current stream (mode 1: its row segment; mode 2: its column window)."""
    lo, hi = bounds[e], bounds[e + 1]
    if mode == 1:
        if hi <= lo:
            return True
        if fp8:
            return ext().blaslt_fp8_gemm(a[lo:hi], b[e], sa, sb[e : e + 1], smul, out[lo:hi], accumulate, True)
        o = out[lo:hi]
        res = torch.mm(a[lo:hi], b[e].t(), out_dtype=out.dtype) if out.dtype != a.dtype else torch.mm(a[lo:hi], b[e].t())
        if smul != 1.0:
            res = res * smul
        o.add_(res) if accumulate else o.copy_(res)
        return True
    o = out[e]
    if hi <= lo:
        if not accumulate:
            o.zero_()
        return True
    if fp8:
        return ext().blaslt_fp8_gemm(a[:, lo:hi], b[:, lo:hi], sa, sb, smul, o, accumulate, True)
    if o.dtype == a.dtype and smul == 1.0:
        o.addmm_(a[:, lo:hi], b[:, lo:hi].t()) if accumulate else torch.mm(a[:, lo:hi], b[:, lo:hi].t(), out=o)
    elif o.dtype == torch.float32 and smul == 1.0:
        torch.addmm(o, a[:, lo:hi], b[:, lo:hi].t(), out_dtype=torch.float32, out=o) if accumulate else \
            torch.mm(a[:, lo:hi], b[:, lo:hi].t(), out_dtype=torch.float32, out=o)
    else:
        res = (a[:, lo:hi].float() @ b[:, lo:hi].float().t()) * smul
        o.add_(res.to(o.dtype)) if accumulate else o.copy_(res)
    return True


def grouped_mm(a, b, seg, mode, out, sa=None, sb=None, smul=1.0, accumulate=False, kind=None):
    """One grouped GEMM over the expert segment table `seg` (csrc/kernels/grouped_gemm.hip):
    mode 1: out[r] = a[r] . b[e]^T for rows r of segment e (a [R, K], b [E, N, K], out [R, N]; rows past seg[E] -> 0);
    mode 2: out[e] = a[:, seg_e] . b[:, seg_e]^T (a [M, T], b [N, T], out [E, M, N]).
    sa / sb: fp32 amax-style scale tensors ([1] and [E] (mode 1) / [1] (mode 2)), times `smul`. Off the GPU (and for
    shapes the kernel does not tile) the same product runs in PyTorch from a host copy of `seg`. `kind` ("fwd" /
    "dgrad" / "wgrad") names the product for the bf16 backend choice."""
    E = seg.numel() - 1
    bounds = getattr(seg, "_acc_bounds", None)
    if bounds is not None and _asm_grouped_mm(a, b, bounds, mode, out, sa, sb, smul, accumulate, kind):
        return out
    if (bounds is not None and _MOE_GEMM == "blaslt" and a.is_cuda and use_native(a)
            and _per_expert_mm(a, b, bounds, mode, out, sa, sb, smul, accumulate)):
        return out
    if _gg_native_ok(a, b, mode, out):
        sa = sa if sa is not None else _ones(1, a.device)
        sb = sb if sb is not None else _ones(E if mode == 1 else 1, a.device)
        ext().grouped_gemm(a, b, out, seg, mode, sa, sb, float(smul), bool(accumulate))
        return out
    bounds = seg.tolist()
    s_a = 1.0 if sa is None else float(sa.reshape(-1)[0])
    res = torch.zeros(out.shape, dtype=torch.float32, device=out.device)
    if mode == 1:
        for e in range(E):
            lo, hi = bounds[e], bounds[e + 1]
            if hi > lo:
                res[lo:hi] = (a[lo:hi].float() @ b[e].float().t()) * (s_a * smul * (1.0 if sb is None else float(sb[e])))
    else:
        s = s_a * smul * (1.0 if sb is None else float(sb.reshape(-1)[0]))
        for e in range(E):
            lo, hi = bounds[e], bounds[e + 1]
            res[e] = (a[:, lo:hi].float() @ b[:, lo:hi].float().t()) * s
    if accumulate:
        out.add_(res.to(out.dtype))
    else:
        out.copy_(res)
    return out


def _t(x):
    """Transposed contiguous copy of a 2-D bf16 activation (the K-contiguous operand of a weight-gradient GEMM)."""
    if x.is_cuda and use_native(x) and x.dtype == torch.bfloat16 and x.shape[0] % 64 == 0 and x.shape[1] % 64 == 0:
        return ext().transpose_bf16(x)
    return x.t().contiguous()


# bf16 expert dgrad on the per-expert library path straight from the stored stack (NN layout) instead of through a
# transposed copy of both stacks per backward: an expert sees ~1/E of the tokens, so re-laying out its whole weight
# costs more than the layout gains (ACCELERATE_MOE_DGRAD_NN=0: the transposed copy, as the grouped kernel needs).
_MOE_DGRAD_NN = os.environ.get("ACCELERATE_MOE_DGRAD_NN", "1") != "0"


def _dgrad_mm(a, w, seg, out):
    """out[r] = a[r] . w[e] for the rows r of expert e's segment (w [E, N, K] as stored: the dgrad of a mode-1
    product). The per-expert hipBLASLt path (host segment bounds attached) runs it on w itself; otherwise the grouped
    kernel takes the K-contiguous copy `_bt(w)`."""
    bounds = getattr(seg, "_acc_bounds", None)
    if "dgrad" in _MOE_ASM_BF16 and bounds is not None and a.is_cuda and use_native(a) and _MOE_ASM:
        return grouped_mm(a, _bt(w), seg, 1, out, kind="dgrad")
    if (_MOE_DGRAD_NN and bounds is not None and _MOE_GEMM == "blaslt" and a.is_cuda and use_native(a)
            and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and out.dtype == torch.bfloat16
            and a.is_contiguous() and w.is_contiguous() and out.is_contiguous()):
        E = len(bounds) - 1
        for e in range(E):
            lo, hi = bounds[e], bounds[e + 1]
            if hi > lo:
                torch.mm(a[lo:hi], w[e], out=out[lo:hi])
        if bounds[E] < out.shape[0]:
            out[bounds[E] :].zero_()  # rows past the last segment are defined (zero), as in grouped_mm
        return out
    return grouped_mm(a, _bt(w), seg, 1, out)


def _bt(w):
    """[E, N, K] -> [E, K, N] (expert weight stacks; bf16 or fp8)."""
    if w.is_cuda and use_native(w) and (w.element_size() == 1 or (w.shape[1] % 64 == 0 and w.shape[2] % 64 == 0)):
        return ext().batched_transpose(w.contiguous())
    return w.transpose(1, 2).contiguous()


# Token dispatch / combine through the HIP row kernels (csrc/kernels/moe_route.hip) instead of torch index_copy /
# index_select / bf16 index_add (ACCELERATE_MOE_ROUTE_HIP=0 restores those).
_MOE_ROUTE_HIP = os.environ.get("ACCELERATE_MOE_ROUTE_HIP", "1") != "0"


def _route_native_ok(t: torch.Tensor, K: int) -> bool:
    return (_MOE_ROUTE_HIP and t.is_cuda and use_native(t) and t.dtype == torch.bfloat16 and t.dim() == 2
            and t.shape[1] % 8 == 0 and 1 <= K <= 8)


class _RouteDispatch(torch.autograd.Function):
    """x_routed [R, H]: row pos[t*K + k] = token t, pad rows zero (each slot owns a unique row). Backward: the token
    gradient is the sum of its K rows (a gather, no atomics)."""

    @staticmethod
    def forward(ctx, t, pos, R, K):
        out = t.new_zeros(R, t.shape[1])
        ext().moe_scatter_rows(t.contiguous(), pos, None, out, None, None, K)
        ctx.save_for_backward(pos)
        ctx.T, ctx.K = t.shape[0], K
        return out

    @staticmethod
    def backward(ctx, g):
        (pos,) = ctx.saved_tensors
        return ext().moe_gather_rows(g.contiguous(), pos, None, ctx.T, ctx.K), None, None, None


class _RouteCombine(torch.autograd.Function):
    """out[t] = sum_k w[t*K + k] * y[pos[t*K + k]] (fp32 accumulation). Backward: dy rows = w * dout (pad rows zero) and
    dw = <dout[t], y[pos]>, one kernel."""

    @staticmethod
    def forward(ctx, y, pos, w, K):
        y = y.contiguous()
        wf = w.float().contiguous()
        T = pos.numel() // K
        out = ext().moe_gather_rows(y, pos, wf, T, K)
        ctx.save_for_backward(y, pos, wf)
        ctx.K, ctx.w_dtype = K, w.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        y, pos, wf = ctx.saved_tensors
        dy = torch.zeros_like(y)
        dw = torch.empty_like(wf)
        ext().moe_scatter_rows(g.contiguous(), pos, wf, dy, y, dw, ctx.K)
        return dy, None, dw.to(ctx.w_dtype), None


class _GroupedExpertsFn(torch.autograd.Function):
    """y = down_e(swiglu(gate_up_e(x))) for the rows of each expert segment of the routed buffer `x` [R, H].

    Every projection and direction is ONE grouped GEMM over the device segment table (forward: 2, backward: 2 dgrad
    + 2 weight-gradient), so the expert count costs no launches and no host syncs. The weight gradients are the
    K-segmented form (each expert's K range = its token rows) on transposed activations.

    bf16: bf16 MFMA grouped kernel. fp8 (a recipe is attached): operands e4m3 (forward) / e5m2 (gradients, HYBRID),
    one per-tensor scale per activation buffer and one per expert weight (segment amax over the stacked weights), and
    the transposed fp8 copies the backward needs come out of the same cast pass as the forward copies.
    """

    @staticmethod
    def forward(ctx, x, w_gu, w_down, seg, recipe, slots=(None, None)):
        ctx.bounds = getattr(seg, "_acc_bounds", None)
        R, H = x.shape
        E, I2, _ = w_gu.shape
        I = w_down.shape[2]
        fp8 = recipe is not None and _native_ok(x, H, I2, I)
        if fp8:
            y, st = _fp8_fwd(x, w_gu, w_down, seg, recipe)
            ctx.st = st
        else:
            h = grouped_mm(x, w_gu, seg, 1, x.new_empty(R, I2), kind="fwd")
            y = grouped_mm(_swiglu_fwd(h), w_down, seg, 1, x.new_empty(R, H), kind="fwd")
            ctx.st = h
        ctx.save_for_backward(x, w_gu, w_down, seg)
        ctx.recipe, ctx.fp8, ctx.slots = recipe, fp8, slots
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_gu, w_down, seg = ctx.saved_tensors
        if ctx.bounds is not None:
            seg._acc_bounds = ctx.bounds  # the forward's host copy of the segment table: no second sync
        dy = dy.contiguous().to(x.dtype)
        # weight-gradient destinations: the FSDP engine's slot (fp32 grad shard at world size 1, flat bf16 grad buffer
        # otherwise; the grouped GEMM accumulates into it) or a fresh tensor returned to autograd
        dsts = []
        for w, slot in zip((w_gu, w_down), ctx.slots):
            if slot is not None:
                dest, acc = slot.engine._fused_slot_dest(slot)
                dsts.append((dest, acc, slot))
            else:
                dsts.append((w.new_empty(w.shape), False, None))
        (g_gu, acc_gu, _), (g_d, acc_d, _) = dsts
        if ctx.fp8:
            dx = _fp8_bwd(dy, x, w_gu, w_down, seg, ctx.st, ctx.recipe, (g_gu, acc_gu), (g_d, acc_d))
        else:
            h = ctx.st
            R, H = x.shape
            I = w_down.shape[2]
            a = _swiglu_fwd(h)
            da = _dgrad_mm(dy, w_down, seg, x.new_empty(R, I))
            grouped_mm(_t(dy), _t(a), seg, 2, g_d, accumulate=acc_d, kind="wgrad")
            dh = _swiglu_bwd(h, da)
            grouped_mm(_t(dh), _t(x), seg, 2, g_gu, accumulate=acc_gu, kind="wgrad")
            dx = _dgrad_mm(dh, w_gu, seg, x.new_empty(R, H))
        ctx.st = None
        grads = []
        for dest, _, slot in dsts:
            if slot is not None:
                slot.engine._fused_slot_done(slot)
                grads.append(None)
            else:
                grads.append(dest)
        return dx, grads[0], grads[1], None, None, None


def _expert_weight_fp8(w, recipe, key):
    """Per-expert e4m3 copy of a stacked weight [E, N, K] (one scale per expert: segment amax over the flat stack)
    and its [E, K, N] transpose. Returns (w8, w8t, amax [E])."""
    from ..ops.fp8 import E4M3_MAX

    E = w.shape[0]
    flat = w.contiguous().view(-1)
    n = flat.numel() // E
    lo = torch.arange(E, device=w.device, dtype=torch.long) * n
    held = getattr(w, "_acc_fp8_expert_amax", None)  # FSDP world size 1: reduced by the fused AdamW that wrote w
    if held is not None and held.fresh and held.amax.numel() == E:
        amax = held.amax
    else:
        amax = torch.empty(E, dtype=torch.float32, device=w.device)
        ext().fp8_segment_amax(flat, lo, lo + n, amax, n)
    if os.environ.get("ACCELERATE_MOE_FP8_CAST_T", "1") != "0":
        # one pass writes both layouts (per-expert scale): no byte transpose re-reading the e4m3 stack
        w8 = torch.empty(w.shape, dtype=torch.float8_e4m3fn, device=w.device)
        w8t = torch.empty((E, w.shape[2], w.shape[1]), dtype=torch.float8_e4m3fn, device=w.device)
        ext().fp8_cast_batched_into(flat.view(w.shape), amax, E4M3_MAX, w8, w8t)
        return w8, w8t, amax
    w8 = torch.empty(flat.numel(), dtype=torch.float8_e4m3fn, device=w.device)
    ext().fp8_segment_cast(flat, lo, lo + n, amax, E4M3_MAX, w8, n)
    w8 = w8.view(w.shape)
    return w8, _bt(w8), amax


def _swiglu_amax(h, da=None):
    """SwiGLU forward (da None) or backward with the abs-max of its output from the same kernel (the amax a consuming
    fp8 cast needs), or (output, None) off the HIP path."""
    if use_native(h) and h.dtype == torch.bfloat16 and (h.shape[-1] // 2) % 8 == 0:
        am = torch.empty(1, dtype=torch.float32, device=h.device)
        if da is None:
            return ext().swiglu_fwd(h.contiguous(), am), am
        return ext().swiglu_bwd(h.contiguous(), da.contiguous(), am), am
    return (_swiglu_fwd(h) if da is None else _swiglu_bwd(h, da)), None


def _fp8_fwd(x, w_gu, w_down, seg, recipe):
    from ..ops.fp8 import E4M3_MAX, cast, producer_amax

    R, H = x.shape
    sx = recipe.scale("x", x, E4M3_MAX, producer_amax(x))  # tagged by the dispatch when the norm produced it
    x8, x8t = cast(x, sx, False, transpose=True)
    gu8, gu8t, a_gu = _expert_weight_fp8(w_gu, recipe, "wgu")
    d8, d8t, a_d = _expert_weight_fp8(w_down, recipe, "wd")
    q2 = 1.0 / (E4M3_MAX * sx.qmax)
    h = grouped_mm(x8, gu8, seg, 1, x.new_empty(R, w_gu.shape[1]), sx.amax, a_gu, q2)
    a, am_a = _swiglu_amax(h)
    sa = recipe.scale("a", a, E4M3_MAX, am_a)
    a8, a8t = cast(a, sa, False, transpose=True)
    y = grouped_mm(a8, d8, seg, 1, x.new_empty(R, H), sa.amax, a_d, 1.0 / (E4M3_MAX * sa.qmax))
    return y, (h, x8t, a8t, gu8t, d8t, sx, sa, a_gu, a_d)


def _fp8_bwd(dy, x, w_gu, w_down, seg, st, recipe, gu_out, d_out):
    from ..ops.fp8 import E4M3_MAX, E5M2_MAX, cast

    h, x8t, a8t, gu8t, d8t, sx, sa, a_gu, a_d = st
    R, H = x.shape
    E, I2, _ = w_gu.shape
    I = w_down.shape[2]
    e5 = recipe.grad_e5m2()
    gmax = E5M2_MAX if e5 else E4M3_MAX
    sg = recipe.scale("gy", dy, gmax)
    dy8, dy8t = cast(dy, sg, e5, transpose=True)
    da = grouped_mm(dy8, d8t, seg, 1, x.new_empty(R, I), sg.amax, a_d, 1.0 / (sg.qmax * E4M3_MAX))
    grouped_mm(dy8t, a8t, seg, 2, d_out[0], sg.amax, sa.amax, 1.0 / (sg.qmax * sa.qmax), accumulate=d_out[1])
    dh, am_dh = _swiglu_amax(h, da)
    sh = recipe.scale("gh", dh, gmax, am_dh)
    dh8, dh8t = cast(dh, sh, e5, transpose=True)
    grouped_mm(dh8t, x8t, seg, 2, gu_out[0], sh.amax, sx.amax, 1.0 / (sh.qmax * sx.qmax), accumulate=gu_out[1])
    return grouped_mm(dh8, gu8t, seg, 1, x.new_empty(R, H), sh.amax, a_gu, 1.0 / (sh.qmax * E4M3_MAX))


class MoEExperts(nn.Module):
    """Stacked SwiGLU experts. With expert parallelism only the local slice [E_local, ...] is materialised."""

    def __init__(self, num_experts: int, hidden: int, intermediate: int):
        super().__init__()
        self.num_experts = num_experts
        self.w_gate_up = nn.Parameter(torch.empty(num_experts, 2 * intermediate, hidden))
        self.w_down = nn.Parameter(torch.empty(num_experts, hidden, intermediate))
        self.fp8_recipe = None

    def forward(self, x_routed, seg):
        """x_routed: [R, H] routed-token buffer (expert e's rows are [seg[e], seg[e+1]), zero pad rows)."""
        w_gu, w_down = self.w_gate_up, self.w_down
        slots = (None, None)
        if w_gu.dtype != x_routed.dtype:
            w_gu, w_down = w_gu.to(x_routed.dtype), w_down.to(x_routed.dtype)
        elif torch.is_grad_enabled():
            # FSDP fused weight-gradient slots (parallel/fsdp.py): the grouped wgrad GEMMs write into the grad shard
            slots = tuple(getattr(w, "_acc_wgrad_slot", None) for w in (w_gu, w_down))
            if torch._C._current_graph_task_id() == -1:
                for sl in slots:
                    if sl is not None:
                        sl.uses += 1
        return _GroupedExpertsFn.apply(x_routed, w_gu, w_down, seg, self.fp8_recipe, slots)


class MoELayer(nn.Module):
    def __init__(self, hidden: int, intermediate: int, num_experts: int, top_k: int, norm_topk: bool = True):
        super().__init__()
        self.num_experts, self.top_k, self.norm_topk = num_experts, top_k, norm_topk
        self.gate = nn.Linear(hidden, num_experts, bias=False)
        self.experts = MoEExperts(num_experts, hidden, intermediate)
        self.ep_group = None
        self.last_router_logits = None
        # optional per-expert selection bias (DeepSeek-V3-style aux-loss-free balancing): shifts which experts are
        # chosen, not the combine weights; None = plain top-k of the router softmax (Mixtral)
        self.router_bias: Optional[torch.Tensor] = None

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
        if self.router_bias is None:
            w, idx = torch.topk(probs, self.top_k, dim=-1)
        else:
            idx = torch.topk(probs + self.router_bias.to(probs), self.top_k, dim=-1)[1]
            w = probs.gather(-1, idx)
        if self.norm_topk:
            w = w / w.sum(-1, keepdim=True)
        w = w.to(t.dtype)
        flat_e = idx.reshape(-1)
        if self.ep_group is None or comm.group_size(self.ep_group) == 1:
            order, dest, seg, R = expert_layout(flat_e, self.num_experts)
            _attach_bounds(seg)
            if _route_native_ok(t, self.top_k):
                from ..ops.fp8 import producer_amax, tag_amax

                pos = torch.empty_like(dest)
                pos[order] = dest  # routed row of slot t*K + k
                x_routed = _RouteDispatch.apply(t, pos, R, self.top_k)
                am = producer_amax(x)
                if am is not None:  # every token lands in the routed buffer, the pad rows are zero: same abs-max
                    tag_amax(x_routed, am)
                out = _RouteCombine.apply(self.experts(x_routed, seg), pos, w.reshape(-1), self.top_k)
                return out.view(shape)
            src_tok = order // self.top_k
            w_sorted = w.reshape(-1)[order]
            x_routed = t.new_zeros(R, t.shape[1]).index_copy(0, dest, t.index_select(0, src_tok))
            y_sorted = self.experts(x_routed, seg).index_select(0, dest)
        else:
            order = torch.argsort(flat_e, stable=True)
            if _route_native_ok(t, self.top_k):
                # expert-sorted rows, one per slot: the same atomic-free dispatch / combine with R = T * K (no pads)
                pos = torch.empty_like(order)
                pos[order] = torch.arange(order.numel(), device=order.device)
                x_sorted = _RouteDispatch.apply(t, pos, order.numel(), self.top_k)
                y_sorted = self._ep_experts(x_sorted, flat_e[order])
                return _RouteCombine.apply(y_sorted, pos, w.reshape(-1), self.top_k).view(shape)
            src_tok = order // self.top_k
            w_sorted = w.reshape(-1)[order]
            y_sorted = self._ep_experts(t.index_select(0, src_tok), flat_e[order])
        out = torch.zeros_like(t).index_add_(0, src_tok, y_sorted * w_sorted.unsqueeze(-1))
        return out.view(shape)

    def _ep_experts(self, x_sorted, e_sorted):
        """Expert-parallel dispatch / combine. `x_sorted` rows are sorted by global expert id, so the rows bound for
        rank d are contiguous and already grouped by d's local experts. One [E]-sized count all-to-all (how many rows
        of each of MY local experts every source rank sends) is the only exchange besides the payload, and its host
        copy (the split sizes `all_to_all_single` needs) is the only host sync: each receiver rebuilds the local expert
        id of every received row from those counts, so no ids travel with the tokens."""
        group = self.ep_group
        W = comm.group_size(group)
        El = self.num_experts // W
        send_e = torch.bincount(e_sorted, minlength=self.num_experts).to(torch.int64)  # [W * El], rank-major
        recv_e = self._exchange_counts(send_e, W, group)  # recv_e[s * El + j]: rows of my expert j from rank s
        host = torch.cat([send_e.view(W, El).sum(1), recv_e.view(W, El).sum(1), recv_e]).tolist()
        sc, rc, rcv = host[:W], host[W : 2 * W], host[2 * W :]
        x_recv = comm.all_to_all_var(x_sorted, sc, rc, group)
        local_ids = torch.arange(El, device=x_sorted.device).repeat(W)
        e_recv = torch.repeat_interleave(local_ids, recv_e, output_size=sum(rc))
        # local experts: the same device-side layout + grouped GEMMs as the single-rank path
        order2, dest2, seg2, R2 = expert_layout(e_recv, El)
        if seg2.is_cuda and _MOE_GEMM == "blaslt" and use_native(seg2):  # host segment table from the same copy
            bounds = [0]
            for j in range(El):
                c = sum(rcv[s_ * El + j] for s_ in range(W))
                bounds.append(bounds[-1] + _round_up(c, SEG_ALIGN))
            seg2._acc_bounds = bounds
        x_routed = x_recv.new_zeros(R2, x_recv.shape[1]).index_copy(0, dest2, x_recv.index_select(0, order2))
        y_local_sorted = self.experts(x_routed, seg2).index_select(0, dest2)
        inv = torch.empty_like(order2)
        inv[order2] = torch.arange(order2.numel(), device=order2.device)
        y_recv = y_local_sorted.index_select(0, inv)
        return comm.all_to_all_var(y_recv, rc, sc, group)

    @staticmethod
    def _exchange_counts(send_e, W, group):
        """All-to-all of equal El-sized slices of the per-expert count vector (HIP tensors on gloo: via all_gather)."""
        El = send_e.numel() // W
        if not comm.tensor_forms(group, send_e):
            gathered = [torch.empty_like(send_e) for _ in range(W)]
            dist.all_gather(gathered, send_e, group=group)
            me = comm.group_rank(group)
            return torch.cat([g[me * El : (me + 1) * El] for g in gathered])
        recv_e = torch.empty_like(send_e)
        dist.all_to_all_single(recv_e, send_e, group=group)
        return recv_e


def _attach_bounds(seg):
    """Host copy of the segment table for the per-expert library GEMMs (one device -> host copy per MoE layer)."""
    if seg.is_cuda and (_MOE_GEMM == "blaslt" or _MOE_ASM) and use_native(seg):
        seg._acc_bounds = seg.tolist()
    return seg


def load_balancing_loss(router_logits: list, num_experts: int, top_k: int) -> torch.Tensor:
    """Switch-style auxiliary loss (HF `load_balancing_loss_func`): E · Σ_e f_e · P_e over all layers' tokens."""
    logits = torch.cat([l.float() for l in router_logits], 0)
    probs = torch.softmax(logits, -1)
    _, sel = torch.topk(probs, top_k, -1)
    mask = F.one_hot(sel, num_experts).float()  # [T, k, E]
    tokens_per_expert = mask.mean(0)  # [k, E]
    prob_per_expert = probs.mean(0)  # [E]
    return (tokens_per_expert * prob_per_expert.unsqueeze(0)).sum() * num_experts
