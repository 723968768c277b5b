"""fp8 training on MI355X: per-tensor scaling, OCP e4m3/e5m2 casts and MX-MFMA GEMMs (csrc/kernels/fp8.hip).

Parity: the reference delegates fp8 to torchao `Float8Linear` (`/root/reference/src/accelerate/utils/ao.py:32-143`,
`accelerator.py:2042-2068`) or TransformerEngine (`utils/transformer_engine.py`). Here `Fp8Linear` implements both
recipes with our kernels:

* dynamic scaling (torchao-style, `AORecipeKwargs`): scale = fp8_max / amax of the current tensor;
* delayed scaling (TE-style, `TERecipeKwargs`): scale from the max of an amax history ring buffer kept on the device
  (length `amax_history_len`), `margin` applied as 2^-margin; format "HYBRID" = e4m3 forward, e5m2 gradients;
* MXFP8 block scaling (TE `MXFP8BlockScaling`, `TERecipeKwargs(use_mxfp8_block_scaling=True)`): one e8m0 scale per 32
  elements along each GEMM's reduction dimension, applied by the MFMA itself (`v_mfma_scale_f32_32x32x64_f8f6f4`'s
  block-scale operands); every tensor is quantised twice in one pass (row blocks and column blocks), so forward,
  dgrad and wgrad each read K-contiguous operands with their own block scales. Reference:
  `/root/reference/src/accelerate/utils/transformer_engine.py:165-186`, `utils/dataclasses.py:404,433-434`.

Forward  y  = (x8 · w8ᵀ) / (sx·sw)                      — fp8 GEMM, bf16 out
Backward dx = (dy8 · w8ᵀᵀ) / (sg·sw),  dW = (dy8ᵀ · x8ᵀᵀ) / (sg·sx) — the cast kernel writes the transposed copies
so every GEMM reads K-contiguous operands. Everything stays on the device (no host syncs).

The module filter follows the reference: first and last `nn.Linear` are skipped and both dims must be divisible by 16
(`filter_first_and_last_linear_layers`, `filter_linear_layers`).
"""

from __future__ import annotations

import os
from typing import Callable, NamedTuple, Optional

import torch
import torch.nn as nn

from ._ext import ext, use_native

E4M3_MAX = 448.0
E5M2_MAX = 57344.0
# Per-tensor-scaled fp8 GEMM backend. "hip" (default) = the hand-written kernels: the asm-scheduled 256x256 kernel
# (csrc/kernels/fp8_gemm_asm.hip, 0.95-1.04x hipBLASLt on the Llama-3-8B shapes, profiles/r5_gemm_fp8_asm.md) for
# every M, N multiple of 256 and K multiple of 128, the HIP-only variants of csrc/kernels/fp8.hip for a bias epilogue;
# other shapes take hipBLASLt when it accepts them. "blaslt" = hipBLASLt's fp8 kernels through our runner
# (csrc/runtime/blaslt_gemm.cpp) whenever there is no bias.
_FP8_GEMM_BACKEND = os.environ.get("ACCELERATE_FP8_GEMM", "hip")
# The backward GEMMs on the asm kernel's MN-major modes (csrc/kernels/fp8_gemm_asm.hip `fp8_gemm_amn_kernel`,
# ds_read_b64_tr_b8): dx^T = w8^T . dy8^T reads the e4m3 weight as it is, dW = (x8^T . dy8)^T reads x8 and dy8 as they
# are, so every cast writes one layout (no transposed copies of x, dy or the weight). ACCELERATE_FP8_MN=0: the
# transposing casts + K-major GEMMs.
_FP8_MN = os.environ.get("ACCELERATE_FP8_MN", "1") != "0"


def _asm_tileable(m: int, n: int, k: int) -> bool:
    """Shapes the asm-scheduled kernel tiles (fp8_gemm_asm_launch's host check)."""
    return m % 256 == 0 and n % 256 == 0 and k % 128 == 0 and k >= 256 and 256 * k < 2**31


def amax(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """abs-max of a bf16 tensor as fp32 [1] (device)."""
    if use_native(x) and x.dtype == torch.bfloat16:
        return ext().fp8_amax(x.contiguous(), out)
    r = x.detach().abs().max().float().reshape(1)
    if out is not None:
        out.copy_(r)
        return out
    return r


def scale_from_amax(a: torch.Tensor, fp8_max: float, margin: int = 0) -> torch.Tensor:
    return (fp8_max / (2.0**margin)) / a.clamp_min(1e-12)


def tag_amax(t: torch.Tensor, amax: torch.Tensor) -> torch.Tensor:
    """Attach a producer-computed abs-max (fp32 [1], device) to `t`: an fp8 linear consuming `t` as its input (or as
    its output gradient) then skips its own amax pass over it. Valid only while `t` is unmodified (version check)."""
    t._acc_amax = (amax, t._version)
    return t


def producer_amax(t: torch.Tensor) -> Optional[torch.Tensor]:
    a = getattr(t, "_acc_amax", None)
    if a is None or a[1] != t._version:
        return None
    return a[0]


def fp8_tensorwise(m) -> bool:
    """Whether module `m` runs a per-tensor-scaled fp8 GEMM now (the consumer of a producer amax). Producer amax is
    switched off with ACCELERATE_FP8_PRODUCER_AMAX=0 (then every fp8 linear runs its own amax pass)."""
    rec = getattr(m, "fp8_recipe", None)
    return (isinstance(m, Fp8Linear) and rec is not None and not rec.mx and _FP8_ON[0]
            and os.environ.get("ACCELERATE_FP8_PRODUCER_AMAX", "1") != "0")


class Scale(NamedTuple):
    """A per-tensor fp8 scale kept as (amax buffer, qmax = fp8_max / 2^margin): the cast kernel computes
    qmax / amax and the GEMM epilogue amax / qmax on the device, so no scale arithmetic is launched separately."""

    amax: torch.Tensor
    qmax: float

    def scale(self) -> torch.Tensor:
        return self.qmax / self.amax.clamp_min(1e-12)

    def inv(self) -> torch.Tensor:
        return self.amax.clamp_min(1e-12) / self.qmax


def cast(x: torch.Tensor, scale, e5m2: bool = False, transpose: bool = False):
    """sat(x * scale) → fp8 (and its transpose when `transpose`). `scale` is a `Scale` or a plain fp32 [1] tensor."""
    if use_native(x) and x.dtype == torch.bfloat16 and x.dim() == 2:
        if isinstance(scale, Scale):
            outs = ext().fp8_cast(x.contiguous(), scale.amax, scale.qmax, True, e5m2, transpose)
        else:
            outs = ext().fp8_cast(x.contiguous(), scale.float().reshape(1), 1.0, False, e5m2, transpose)
        return (outs[0], outs[1]) if transpose else outs[0]
    s = scale.scale() if isinstance(scale, Scale) else scale
    mx = E5M2_MAX if e5m2 else E4M3_MAX
    dt = torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn
    y = (x.float() * s).clamp(-mx, mx).to(dt)
    if transpose:
        return y, y.t().contiguous()
    return y


def _inv_parts(si):
    if isinstance(si, Scale):
        return si.amax, 1.0 / si.qmax
    return si.float().reshape(1), 1.0


def gemm(a8: torch.Tensor, b8: torch.Tensor, a_scale_inv, b_scale_inv, bias=None, out_dtype=torch.bfloat16,
         out: Optional[torch.Tensor] = None, accumulate: bool = False):
    """C = (a8 · b8ᵀ) · a_scale_inv · b_scale_inv (+ bias); a8 [M,K], b8 [N,K]. Inverse scales are `Scale`s (the
    operand's cast scale) or plain fp32 [1] tensors. With `out`, the result is written (or with `accumulate` added)
    into that contiguous [M, N] tensor — e.g. a weight-gradient slot of the FSDP flat gradient buffer."""
    if out is not None:
        out_dtype = out.dtype
    if a8.is_cuda and use_native(a8):
        e5a = a8.dtype == torch.float8_e5m2
        e5b = b8.dtype == torch.float8_e5m2
        ta, ma = _inv_parts(a_scale_inv)
        tb, mb = _inv_parts(b_scale_inv)
        m, k = a8.shape
        n = b8.shape[0]
        if bias is None and (_FP8_GEMM_BACKEND == "blaslt" or not _asm_tileable(m, n, k)):
            dst = out if out is not None else torch.empty((a8.shape[0], b8.shape[0]), dtype=out_dtype, device=a8.device)
            if ext().blaslt_fp8_gemm(a8, b8, ta, tb, ma * mb, dst, accumulate):
                return dst
        return ext().fp8_gemm(a8, b8, ta, tb, ma * mb, e5a, e5b, bias, out_dtype == torch.float32, out, accumulate)
    ia = a_scale_inv.inv() if isinstance(a_scale_inv, Scale) else a_scale_inv
    ib = b_scale_inv.inv() if isinstance(b_scale_inv, Scale) else b_scale_inv
    res = (a8.float() @ b8.float().t()) * ia * ib
    if bias is not None:
        res = res + bias.float()
    if out is None:
        return res.to(out_dtype)
    if accumulate:
        out.add_(res.to(out.dtype))
    else:
        out.copy_(res)
    return out


def _mn_ok(T: int, N: int, K: int) -> bool:
    """The three products of an fp8 linear (x [T, K], w [N, K]) all tile on the MN-major / K-major asm kernels."""
    return (_FP8_MN and _FP8_GEMM_BACKEND == "hip" and T % 256 == 0 and N % 256 == 0 and K % 256 == 0
            and T >= 256 and _asm_tileable(T, N, K))


def gemm_t(a_t8: torch.Tensor, b8: torch.Tensor, a_scale_inv, b_scale_inv, out: torch.Tensor, b_mn: bool = False,
           accumulate: bool = False):
    """out (=|+=) ((a_t8ᵀ · b8ᵀ)ᵀ) · a_scale_inv · b_scale_inv on the MN-major asm kernel: a_t8 [K, M] (M contiguous),
    b8 [N, K] or (b_mn) [K, N]; out [N, M]. Returns False when the kernel does not take the shape."""
    ta, ma = _inv_parts(a_scale_inv)
    tb, mb = _inv_parts(b_scale_inv)
    return ext().fp8_gemm_asm_amn(a_t8, b8, ta, tb, ma * mb, out, accumulate, b_mn)


def transpose_fp8(w8: torch.Tensor) -> torch.Tensor:
    """K-major copy of a 2-D fp8 tensor (HIP byte transpose on GPU)."""
    if w8.is_cuda and use_native(w8):
        return ext().u8_transpose(w8.contiguous())
    return w8.t().contiguous()


def _gemm_ok(M, N, K):
    return M % 128 == 0 and N % 128 == 0 and K % 64 == 0


# ------------------------------------------------------------------------------------------------------------ MXFP8
MX_BLOCK = 32


def _mx_pos(nblk: int, device=None) -> torch.Tensor:
    """Byte position of each 32-element block in a row of the grouped scale layout (csrc fp8.hip `mx_pos`): the 8 blocks
    of a 256-element group are stored [hf = 0: q = 0..3 | hf = 1: q = 0..3] for block 8g + 2q + hf."""
    b = torch.arange(nblk, device=device)
    return (b & ~7) | ((b & 1) << 2) | ((b >> 1) & 3)


def mx_scales_natural(s: torch.Tensor) -> torch.Tensor:
    """Grouped-layout e8m0 scales [R, K/32] -> scales in block order."""
    return s[:, _mx_pos(s.shape[1], s.device)]


def _mx_quant_rows(x: torch.Tensor, e5m2: bool):
    """Reference MX quantisation of x [R, C] along C (PyTorch; the HIP kernel's oracle and CPU path)."""
    R, C = x.shape
    fmax = E5M2_MAX if e5m2 else E4M3_MAX
    blocks = x.float().reshape(R, C // MX_BLOCK, MX_BLOCK)
    amax = blocks.abs().amax(-1)
    v = amax * (1.0 / fmax)
    bits = v.view(torch.int32)
    e = (bits >> 23) + ((bits & 0x7FFFFF) != 0).to(torch.int32)  # exponent of amax / fp8_max, rounded up
    e = e.clamp(max=253)
    inv = torch.exp2((127 - e).float())
    dt = torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn
    q = (blocks * inv.unsqueeze(-1)).clamp(-fmax, fmax).to(dt).reshape(R, C)
    s = torch.empty(R, C // MX_BLOCK, dtype=torch.uint8, device=x.device)
    s[:, _mx_pos(C // MX_BLOCK, x.device)] = e.to(torch.uint8)
    return q, s


def mx_quant(x: torch.Tensor, e5m2: bool = False, colwise: bool = True):
    """MXFP8-quantise a 2-D bf16 tensor: (q, s) with 32-element blocks along its columns, plus (qt, st) = x^T quantised
    with blocks along x's rows when `colwise` (the wgrad / dgrad operands). s / st are uint8 e8m0 in the grouped layout."""
    if x.is_cuda and use_native(x) and x.dtype == torch.bfloat16:
        return tuple(ext().mx_quant(x.contiguous(), e5m2, colwise))
    q, s = _mx_quant_rows(x, e5m2)
    if not colwise:
        return q, s
    qt, st = _mx_quant_rows(x.t().contiguous(), e5m2)
    return q, s, qt, st


def mx_dequant(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """fp32 value of an MX tensor (q [R, K], grouped scales s [R, K/32])."""
    R, K = q.shape
    sc = torch.exp2(mx_scales_natural(s).float() - 127.0)
    return (q.float().reshape(R, K // MX_BLOCK, MX_BLOCK) * sc.unsqueeze(-1)).reshape(R, K)


def mx_gemm(a8, b8, sa, sb, bias=None, out_dtype=torch.bfloat16, out: Optional[torch.Tensor] = None,
            accumulate: bool = False):
    """C = (a · bᵀ) with MX block scales (+ bias): a8 [M, K], b8 [N, K] fp8 with e8m0 scales [M, K/32] / [N, K/32]. The
    block scales ride in the MFMA (no dequantisation pass). `out` / `accumulate` as in `gemm`."""
    if out is not None:
        out_dtype = out.dtype
    if a8.is_cuda and use_native(a8):
        return ext().mx_gemm(a8, b8, sa, sb, 1.0, bias, out_dtype == torch.float32, out, accumulate)
    res = mx_dequant(a8, sa) @ mx_dequant(b8, sb).t()
    if bias is not None:
        res = res + bias.float()
    if out is None:
        return res.to(out_dtype)
    if accumulate:
        out.add_(res.to(out.dtype))
    else:
        out.copy_(res)
    return out


def _mx_ok(M, N, K):
    """Shapes the MX GEMM tiles (256 x 256 output tiles, K in 256-element scale groups) for all three GEMMs."""
    return M % 256 == 0 and N % 256 == 0 and K % 256 == 0


class _MxLinearFn(torch.autograd.Function):
    """MXFP8 linear: y = x wᵀ, dx = dy w, dW = dyᵀ x, each GEMM on MX operands blocked along its own reduction dim.
    x, w and dy are each quantised once into row-blocked and column-blocked copies (one HIP pass per tensor)."""

    @staticmethod
    def forward(ctx, x, w, bias, recipe, slot=None):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        e5 = recipe.fwd_e5m2()
        xq, xs, xqt, xst = mx_quant(x2, e5, True)
        wq, ws, wqt, wst = mx_quant(w, e5, True)
        y = mx_gemm(xq, wq, xs, ws, bias, torch.bfloat16)
        ctx.save_for_backward(xqt, xst, wqt, wst)
        ctx.recipe, ctx.shape, ctx.has_bias, ctx.slot = recipe, shape, bias is not None, slot
        return y.view(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        xqt, xst, wqt, wst = ctx.saved_tensors
        N = dy.shape[-1]
        dy2 = dy.reshape(-1, N).contiguous().to(torch.bfloat16)
        gq, gs, gqt, gst = mx_quant(dy2, ctx.recipe.grad_e5m2(), True)
        dx = mx_gemm(gq, wqt, gs, wst, None, torch.bfloat16)
        db = dy2.float().sum(0).to(dy.dtype) if ctx.has_bias else None
        slot = ctx.slot
        if slot is not None:
            dest, acc = slot.engine._fused_slot_dest(slot)
            mx_gemm(gqt, xqt, gst, xst, None, out=dest, accumulate=acc)
            slot.engine._fused_slot_done(slot)
            return dx.view(ctx.shape), None, db, None, None
        dw = mx_gemm(gqt, xqt, gst, xst, None, torch.bfloat16)
        return dx.view(ctx.shape), dw, db, None, None


class Fp8Recipe:
    """Runtime scaling state of one Fp8Linear."""

    def __init__(self, delayed: bool = False, history_len: int = 16, margin: int = 0, fmt: str = "HYBRID", algo: str = "max",
                 mx: bool = False):
        self.mx = mx  # MXFP8 block scaling (no per-tensor scale state)
        self.delayed = delayed and not mx
        self.history_len = history_len
        self.margin = margin
        self.fmt = fmt.upper()
        self.algo = algo
        self.hist = {}

    def grad_e5m2(self):
        return self.fmt in ("HYBRID", "E5M2")

    def fwd_e5m2(self):
        return self.fmt == "E5M2"

    def scale(self, key: str, x: torch.Tensor, fp8_max: float, hint: Optional[torch.Tensor] = None) -> Scale:
        """Dynamic: this tensor's amax (`hint`: already computed by the kernel that produced x). Delayed: the history's
        max (or most recent), then the history is rolled."""
        cur = hint if hint is not None else amax(x)
        qmax = fp8_max / (2.0**self.margin)
        if not self.delayed:
            return Scale(cur, qmax)
        h = self.hist.get(key)
        if h is None:
            h = cur.repeat(self.history_len).clone()
            self.hist[key] = h
        past = h.max().reshape(1) if self.algo == "max" else h[-1:].clone()
        self.hist[key] = torch.cat([h[1:], cur])
        return Scale(past, qmax)


class _Fp8LinearFn(torch.autograd.Function):
    """fp8 linear. With an FSDP `slot` (parallel/fsdp.py `_WgradSlot`) the weight-gradient GEMM writes straight into
    the engine's gradient destination (fp32 grad shard at world size 1, the flat bf16 grad buffer otherwise) and
    reports the parameter's gradient as ready — no separate dW tensor, no AccumulateGrad add."""

    @staticmethod
    def forward(ctx, x, w, bias, recipe: Fp8Recipe, slot=None, w_amax=None, w8t_pre=None):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        N = w.shape[0]
        fwd_max = E5M2_MAX if recipe.fwd_e5m2() else E4M3_MAX
        sx = recipe.scale("x", x2, fwd_max, producer_amax(x))
        ctx.mn = x2.is_cuda and use_native(x2) and _mn_ok(x2.shape[0], N, x2.shape[1])
        if ctx.mn:  # one layout of everything: the backward reads x8 and the weight as they are (MN-major kernels)
            x8 = cast(x2, sx, recipe.fwd_e5m2())
            ctx.pre_quantised = w_amax is not None
            if ctx.pre_quantised:
                sw = Scale(w_amax, E4M3_MAX)
                w8 = w
            else:
                sw = recipe.scale("w", w, fwd_max)
                w8 = cast(w, sw, recipe.fwd_e5m2())
            y = gemm(x8, w8, sx, sw, bias, torch.bfloat16)
            ctx.save_for_backward(x8, w8, sx.amax, sw.amax)
            ctx.qmax = (sx.qmax, sw.qmax)
            ctx.recipe, ctx.shape, ctx.has_bias, ctx.slot = recipe, shape, bias is not None, slot
            return y.view(*shape[:-1], N)
        x8, x8t = cast(x2, sx, recipe.fwd_e5m2(), transpose=True)
        ctx.pre_quantised = w_amax is not None
        if ctx.pre_quantised:
            # FSDP fp8 all-gather: `w` already IS the e4m3 weight (gathered, scale 448 / w_amax); its K-major copy
            # for the dgrad GEMM is made in backward from the (re-gathered) weight instead of being kept alive.
            sw = Scale(w_amax, E4M3_MAX)
            w8 = w
            y = gemm(x8, w8, sx, sw, bias, torch.bfloat16)
            # world size 1: the engine keeps the K-major copy (written with the weight each step), nothing to transpose
            ctx.transpose_w = w8t_pre is None
            ctx.save_for_backward(x8t, w if w8t_pre is None else w8t_pre, sx.amax, sw.amax)
        else:
            sw = recipe.scale("w", w, fwd_max)
            w8, w8t = cast(w, sw, recipe.fwd_e5m2(), transpose=True)
            y = gemm(x8, w8, sx, sw, bias, torch.bfloat16)
            ctx.save_for_backward(x8t, w8t, sx.amax, sw.amax)
        ctx.qmax = (sx.qmax, sw.qmax)
        ctx.recipe, ctx.shape, ctx.has_bias, ctx.slot = recipe, shape, bias is not None, slot
        return y.view(*shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        if ctx.mn:
            return _Fp8LinearFn._backward_mn(ctx, dy)
        x8t, w8t, ax, aw = ctx.saved_tensors
        if ctx.pre_quantised and ctx.transpose_w:
            w8t = transpose_fp8(w8t)
        sx, sw = Scale(ax, ctx.qmax[0]), Scale(aw, ctx.qmax[1])
        recipe = ctx.recipe
        N = dy.shape[-1]
        dy2 = dy.reshape(-1, N).contiguous().to(torch.bfloat16)
        gmax = E5M2_MAX if recipe.grad_e5m2() else E4M3_MAX
        sg = recipe.scale("g", dy2, gmax, producer_amax(dy))
        dy8, dy8t = cast(dy2, sg, recipe.grad_e5m2(), transpose=True)
        dx = gemm(dy8, w8t, sg, sw, None, torch.bfloat16)
        db = dy2.float().sum(0).to(dy.dtype) if ctx.has_bias else None
        slot = ctx.slot
        if slot is not None:
            dest, acc = slot.engine._fused_slot_dest(slot)
            gemm(dy8t, x8t, sg, sx, None, out=dest, accumulate=acc)
            slot.engine._fused_slot_done(slot)
            return dx.view(ctx.shape), None, db, None, None, None, None
        dw = gemm(dy8t, x8t, sg, sx, None, torch.bfloat16)
        return dx.view(ctx.shape), dw, db, None, None, None, None


    @staticmethod
    def _backward_mn(ctx, dy):
        """dx = (w8ᵀ · dy8ᵀ)ᵀ and dW = (x8ᵀ · dy8)ᵀ on the MN-major asm kernel: dy is cast once, row-major."""
        x8, w8, ax, aw = ctx.saved_tensors
        sx, sw = Scale(ax, ctx.qmax[0]), Scale(aw, ctx.qmax[1])
        recipe = ctx.recipe
        N, K = w8.shape
        dy2 = dy.reshape(-1, N).contiguous().to(torch.bfloat16)
        gmax = E5M2_MAX if recipe.grad_e5m2() else E4M3_MAX
        sg = recipe.scale("g", dy2, gmax, producer_amax(dy))
        dy8 = cast(dy2, sg, recipe.grad_e5m2())
        dx = torch.empty((dy2.shape[0], K), dtype=torch.bfloat16, device=dy2.device)
        if not gemm_t(w8, dy8, sw, sg, dx):
            raise RuntimeError(f"fp8 MN-major dgrad GEMM declined shape T={dy2.shape[0]} N={N} K={K}")
        db = dy2.float().sum(0).to(dy.dtype) if ctx.has_bias else None
        slot = ctx.slot
        if slot is not None:
            dest, acc = slot.engine._fused_slot_dest(slot)
            if not gemm_t(x8, dy8, sx, sg, dest, b_mn=True, accumulate=acc):
                raise RuntimeError("fp8 MN-major weight-gradient GEMM declined its shape")
            slot.engine._fused_slot_done(slot)
            return dx.view(ctx.shape), None, db, None, None, None, None
        dw = torch.empty((N, K), dtype=torch.bfloat16, device=dy2.device)
        if not gemm_t(x8, dy8, sx, sg, dw, b_mn=True):
            raise RuntimeError("fp8 MN-major weight-gradient GEMM declined its shape")
        return dx.view(ctx.shape), dw, db, None, None, None, None


class _Fp8GatheredFallbackFn(torch.autograd.Function):
    """y = x · dequant(w8)ᵀ (+ b) for an fp8-gathered weight; backward: dx = dy · w, dW = dyᵀ x into the FSDP slot."""

    @staticmethod
    def forward(ctx, x, w8, w_amax, bias, slot):
        w = (w8.float() * (w_amax.clamp_min(1e-12) / E4M3_MAX)).to(x.dtype)
        ctx.save_for_backward(x, w)
        ctx.slot, ctx.has_bias = slot, bias is not None
        return nn.functional.linear(x, w, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        dx = (dy @ w) if ctx.needs_input_grad[0] else None
        dy2 = dy.reshape(-1, N)
        if ctx.slot is not None:
            ctx.slot.engine._fused_wgrad(ctx.slot, dy2.contiguous(), x.reshape(-1, K).contiguous())
        db = dy2.float().sum(0).to(dy.dtype) if ctx.has_bias else None
        return dx, None, None, db, None


_FP8_ON = [True]


class fp8_enabled:  # noqa: N801 - context manager used like a function
    """`with fp8_enabled(False): ...` runs Fp8Linear layers as plain bf16 linears (TE `fp8_autocast(enabled=)`)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled

    def __enter__(self):
        self.prev = _FP8_ON[0]
        _FP8_ON[0] = self.enabled

    def __exit__(self, *exc):
        _FP8_ON[0] = self.prev


class Fp8Linear(nn.Linear):
    """`nn.Linear` whose matmuls run in fp8 (same parameters, so FSDP / state dicts are unaffected)."""

    fp8_recipe: Fp8Recipe = None

    def forward(self, x):
        M = x.numel() // x.shape[-1]
        gathered = getattr(self.weight, "_acc_fp8_ag", None)  # FSDP fp8 all-gather: the weight arrives as e4m3
        if (
            not self.training
            and not getattr(self, "fp8_in_eval", True)
        ) or not _FP8_ON[0] or not _gemm_ok(M, self.out_features, self.in_features) or x.dtype != torch.bfloat16:
            b = None if self.bias is None else self.bias.to(x.dtype)
            if gathered is not None:
                return self._gathered_fallback(x, gathered, b)
            return nn.functional.linear(x, self.weight.to(x.dtype), b)
        b = None if self.bias is None else self.bias.to(torch.bfloat16)
        if self.fp8_recipe.mx:
            if _mx_ok(M, self.out_features, self.in_features) and gathered is None:
                w = self.weight if self.weight.dtype == torch.bfloat16 else self.weight.to(torch.bfloat16)
                return _MxLinearFn.apply(x, w, b, self.fp8_recipe, self._fp8_wgrad_slot(x))
            if gathered is not None:
                return self._gathered_fallback(x, gathered, b)
            return nn.functional.linear(x, self.weight.to(x.dtype), b)  # shapes the MX tiling cannot cover run in bf16
        if gathered is not None:
            unit, info = gathered
            return _Fp8LinearFn.apply(x, self.weight, b, self.fp8_recipe, self._fp8_wgrad_slot(x),
                                      unit.engine.fp8_weight_scale(unit, info), unit.engine.fp8_weight_t(unit, info))
        w = self.weight if self.weight.dtype == torch.bfloat16 else self.weight.to(torch.bfloat16)
        return _Fp8LinearFn.apply(x, w, b, self.fp8_recipe, self._fp8_wgrad_slot(x))

    def _gathered_fallback(self, x, gathered, b):
        """Non-fp8 path (eval, a batch whose M the fp8 GEMM cannot tile, non-bf16 input) for a weight that arrived as
        e4m3 from the FSDP fp8 all-gather: linear on its dequantised value, with the weight gradient computed in the
        input dtype and written to the weight's FSDP slot (the e4m3 parameter itself cannot hold an autograd grad)."""
        unit, info = gathered
        amax = unit.engine.fp8_weight_scale(unit, info)
        slot = self._fp8_wgrad_slot(x)
        if slot is None and torch.is_grad_enabled() and self.weight.requires_grad:
            raise RuntimeError(f"fp8-gathered weight {info.fqn} has no FSDP gradient slot; its gradient would be lost")
        return _Fp8GatheredFallbackFn.apply(x, self.weight, amax, b, slot)

    def _fp8_wgrad_slot(self, x):
        """The FSDP fused-wgrad slot of this weight (parallel/fsdp.py), when the gradient can be written in place."""
        slot = getattr(self.weight, "_acc_wgrad_slot", None)
        ok_dtype = self.weight.dtype == torch.bfloat16 or getattr(self.weight, "_acc_fp8_ag", None) is not None
        if slot is None or not torch.is_grad_enabled() or not ok_dtype:
            return None
        if torch._C._current_graph_task_id() == -1:
            slot.uses += 1
        return slot


def filter_linear_layers(module: nn.Module, fqn: str, layers_to_filter: list[str]) -> bool:
    """Keep linears whose dims are divisible by 16 and whose name is not filtered (reference ao.py:55-82)."""
    if isinstance(module, nn.Linear):
        if module.in_features % 16 != 0 or module.out_features % 16 != 0:
            return False
    if fqn in layers_to_filter:
        return False
    return True


def find_first_last_linear_layers(model: nn.Module):
    first, last = None, None
    for name, m in model.named_modules():
        if isinstance(m, nn.Linear):
            if first is None:
                first = name
            last = name
    return first, last


def filter_first_and_last_linear_layers(module: nn.Module, fqn: str) -> bool:
    return True


def convert_model_to_fp8(model: nn.Module, recipe=None, backend: str = "AO", module_filter_func: Optional[Callable] = None):
    """Swap eligible `nn.Linear` modules for `Fp8Linear` in place."""
    from ..utils.dataclasses import TERecipeKwargs

    delayed = isinstance(recipe, TERecipeKwargs) or backend == "TE"
    kwargs = {}
    if delayed and recipe is not None and getattr(recipe, "use_mxfp8_block_scaling", False):
        _check_mxfp8_recipe(recipe)
        kwargs = dict(mx=True, fmt=recipe.fp8_format)
    elif delayed and recipe is not None:
        kwargs = dict(delayed=True, history_len=max(1, min(int(recipe.amax_history_len), 1024)), margin=int(recipe.margin), fmt=recipe.fp8_format, algo=recipe.amax_compute_algo)
    else:
        kwargs = dict(delayed=False, fmt="HYBRID")
    if module_filter_func is None and recipe is not None:
        module_filter_func = getattr(recipe, "module_filter_func", None)
    first, last = find_first_last_linear_layers(model)
    skip = {first, last}
    n = 0
    for name, m in list(model.named_modules()):
        if type(m) is not nn.Linear:
            continue
        if name in skip:
            continue
        if not filter_linear_layers(m, name, []):
            continue
        if module_filter_func is not None and not module_filter_func(m, name):
            continue
        m.__class__ = Fp8Linear
        m.fp8_recipe = Fp8Recipe(**kwargs)
        if delayed and recipe is not None:
            m.fp8_in_eval = bool(recipe.use_autocast_during_eval)
        n += 1
    # grouped MoE experts (models/moe.py) run their expert GEMMs in fp8 when they carry a recipe
    for name, m in model.named_modules():
        if not isinstance(m, nn.Linear) and hasattr(m, "fp8_recipe") and hasattr(m, "w_gate_up"):
            if module_filter_func is None or module_filter_func(m, name):
                m.fp8_recipe = Fp8Recipe(**kwargs)
                n += 1
    model._acc_fp8_linears = n
    return model


def _check_mxfp8_recipe(recipe):
    """MXFP8 has no amax history: like TE (reference transformer_engine.py:170-174), an explicitly set history length
    or amax algorithm is an error rather than silently ignored. Only fields differing from the defaults count."""
    from ..utils.dataclasses import TERecipeKwargs

    default = TERecipeKwargs()
    for field in ("amax_compute_algo", "amax_history_len"):
        if getattr(recipe, field) != getattr(default, field):
            raise ValueError(f"`{field}` is not supported for MXFP8 block scaling.")


def has_fp8_layers(model: nn.Module) -> bool:
    return any(isinstance(m, Fp8Linear) for m in model.modules())


def fp8_linear_reference_check(a: torch.Tensor, b: torch.Tensor):
    """Quantise a [M,K] and b [N,K] with dynamic per-tensor scaling and multiply in fp8 (test helper)."""
    sa = Scale(amax(a), E4M3_MAX)
    sb = Scale(amax(b), E4M3_MAX)
    return gemm(cast(a, sa), cast(b, sb), sa, sb, None, torch.float32)
