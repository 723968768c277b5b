"""Autograd wrappers for the fused transformer-block kernels (RMSNorm, SwiGLU, RoPE, cross-entropy, flash
attention). GPU tensors run the HIP kernels in `csrc/kernels/*.hip`; CPU tensors run a PyTorch fp32 reference of
the same op (the reference is also the numerics oracle in tests/test_kernels_gpu.py).
"""

from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ._ext import ext, use_native

# dgrad through a transposed weight copy (ACCELERATE_DGRAD_WT=0 turns it off)
_DGRAD_WT = os.environ.get("ACCELERATE_DGRAD_WT", "1") != "0"
# fp32-output weight-gradient GEMMs through the searched hipBLASLt runner (csrc/runtime/blaslt_gemm.cpp)
_BLASLT_WGRAD = os.environ.get("ACCELERATE_BLASLT_WGRAD", "1") != "0"
# dgrad dx = dy . W in its natural NN layout on the searched hipBLASLt runner (opt-in until measured faster than the
# transposed-weight path below, tools/bench_dgrad.py)
_DGRAD_BLASLT = os.environ.get("ACCELERATE_DGRAD_BLASLT", "0") == "1"
# bf16 Linear GEMMs (forward, dgrad, wgrad) on the asm-scheduled 256x256 MFMA kernel (csrc/kernels/fp8_gemm_asm.hip,
# the fp8 kernel's schedule with two v_mfma_f32_16x16x32_bf16 per block) when the shape tiles. Opt-in
# (ACCELERATE_ASM_BF16_GEMM=1): it runs at 0.93-1.04x hipBLASLt's bf16 kernels on the Llama-3-8B shapes (both ~1.45
# PF/s, the bf16 loop is clock-bound like the fp8 one) and its wgrad needs a transposed dy, so the step is 3 % slower
# with it (profiles/r5_gemm_fp8_asm.md, "bf16 on the same kernel").
# The value is "1" / "all" or a comma list of the products to move: fwd, dgrad, wgrad.
_ASM_BF16_ENV = os.environ.get("ACCELERATE_ASM_BF16_GEMM", "0").strip().lower()
_ASM_BF16_KINDS = ({"fwd", "dgrad", "wgrad"} if _ASM_BF16_ENV in ("1", "all")
                   else {k.strip() for k in _ASM_BF16_ENV.split(",") if k.strip() in ("fwd", "dgrad", "wgrad")})
_ASM_BF16 = bool(_ASM_BF16_KINDS)
# fp32 weight gradients with dy transposed first (ACCELERATE_WGRAD_DYT=1): both hipBLASLt operands token-contiguous,
# the TN class the forward GEMMs run in, for the price of one dy transpose per Linear
_WGRAD_DYT = os.environ.get("ACCELERATE_WGRAD_DYT", "0") == "1"
# weight gradients on the asm kernel's MN-major-A mode (ext().bf16_gemm_asm_amn): dy read as it is ([T, N], the output
# row index contiguous) through transposed LDS reads, x from the saved token-contiguous copy; no transposed dy
# (tools/bench_gemm_amn.py, profiles/r6_gemm_amn.md)
_ASM_WGRAD_AMN = os.environ.get("ACCELERATE_ASM_WGRAD_AMN", "1") != "0"
# weight gradients with BOTH operands read as the step has them (dy [T, N] and the layer input x [T, K], token-major):
# the asm kernel's MN-major-A/B mode computes xᵀ·dy and stores its transpose, so the engines keep x itself instead of
# a token-contiguous copy (no transpose in the forward, 2 GiB less for Llama-3-8B at 8k tokens): 387.4 / 387.8 vs
# 390.9 / 391.1 ms per step on one box (profiles/r6_gemm_amn.md). ACCELERATE_ASM_WGRAD_ABMN=0: the x^T copy + MN-A mode.
ASM_WGRAD_ABMN = os.environ.get("ACCELERATE_ASM_WGRAD_ABMN", "1") != "0"
# dgrad dx = dy . W: on the asm kernel's MN-major-A mode with a transposed store (dx^T = W^T . dy^T, W read as stored,
# no transposed weight copy) or as transpose(W) + hipBLASLt TN. Interleaved bench20 pairs (profiles/r6_gemm_amn.md):
# with the GPU to itself the transpose + TN path is 0.6-2.5 ms per step faster; beside a sharded engine's collectives
# and gradient-shard updates the asm path is 2.6 ms faster (the transpose is one more memory-bound kernel competing with
# them). ACCELERATE_ASM_DGRAD_AMN=auto (default): the asm path once an engine whose collectives run concurrently with
# the backward exists (set_dgrad_concurrent: FSDP sharded / HSDP, DDP at W > 1); 1 / 0 force one path.
_ASM_DGRAD_MODE = os.environ.get("ACCELERATE_ASM_DGRAD_AMN", "auto")
_DGRAD_CONCURRENT = False


def set_dgrad_concurrent(on: bool = True) -> None:
    """Tell the dgrad path that collectives (all-gather / reduce-scatter / all-reduce) run beside the backward."""
    global _DGRAD_CONCURRENT
    _DGRAD_CONCURRENT = bool(on)


def asm_dgrad_enabled() -> bool:
    return _ASM_DGRAD_MODE == "1" or (_ASM_DGRAD_MODE == "auto" and _DGRAD_CONCURRENT)


def asm_gemm_bf16(a: torch.Tensor, b: torch.Tensor, bias=None, out=None, accumulate: bool = False, kind: str = "fwd"):
    """out (=|+=) a . bᵀ (+ bias) for bf16 a [M, K], b [N, K] (both contraction-contiguous) on the asm kernel, or None
    when it does not apply (this product kind not switched on, not native, CPU, shape not a multiple of its 256x256x64
    tile)."""
    if not (kind in _ASM_BF16_KINDS and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2
            and b.dim() == 2 and a.is_contiguous() and b.is_contiguous() and use_native(a)):
        return None
    m, k = a.shape
    n = b.shape[0]
    if m % 256 or n % 256 or k % 64 or k < 128:
        return None
    if out is None:
        if accumulate:
            return None
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    if bias is not None and (bias.dtype != torch.bfloat16 or not bias.is_contiguous()):
        return None
    return out if ext().bf16_gemm_asm(a, b, bias, out, accumulate) else None


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias=None) -> torch.Tensor:
    """y = x · Wᵀ (+ b) for a bf16 Linear: the asm kernel when the token count and both widths tile, else torch."""
    if x.dim() >= 2 and x.is_contiguous():
        y = asm_gemm_bf16(x.reshape(-1, x.shape[-1]), w, bias)
        if y is not None:
            return y.view(*x.shape[:-1], w.shape[0])
    return torch.nn.functional.linear(x, w, bias)


# ----------------------------------------------------------------------------------------------------------
# RMSNorm (optionally fused with the residual add)
# ----------------------------------------------------------------------------------------------------------
def rms_norm_reference(x, weight, eps, residual=None):
    if residual is not None:
        x = (x.float() + residual.float()).to(x.dtype)
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype), x


def _amax_buf(like: torch.Tensor, want: bool):
    return torch.empty(1, dtype=torch.float32, device=like.device) if want else None


class _RMSNormFn(torch.autograd.Function):
    """`amax` / `grad_amax`: also produce max|y| (forward) / max|dx| (backward) for a consuming fp8 linear (its input /
    its output gradient), tagged on the tensor (ops/fp8.py `tag_amax`) instead of re-read by a separate amax pass.
    `slot`: the weight's FSDP gradient slot (parallel/fsdp.py `_WgradSlot`): the backward's column sum writes dweight
    into it (fp32 grad shard at world size 1, flat bf16 grad buffer otherwise) and reports it ready, instead of a new
    tensor that a zero fill, an add and an fp32 copy then move into place (four launches per norm per step)."""

    @staticmethod
    def forward(ctx, x, weight, eps, residual, amax=False, grad_amax=False, slot=None):
        e = ext()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = residual.reshape(-1, shape[-1]).contiguous() if residual is not None else None
        am = _amax_buf(x, amax)
        y, rstd, res_out = e.rmsnorm_fwd(x2, r2, weight.contiguous(), eps, am)
        normed_input = res_out if residual is not None else x2
        ctx.save_for_backward(normed_input, weight, rstd)
        ctx.has_res = residual is not None
        ctx.shape = shape
        ctx.grad_amax = grad_amax
        ctx.slot = slot
        if am is None:
            am = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(am)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the amax / unused residual outputs
        if residual is not None:
            return y.view(shape), res_out.view(shape), am
        return y.view(shape), None, am

    @staticmethod
    def backward(ctx, dy, dres, _dam):
        x, w, rstd = ctx.saved_tensors
        e = ext()
        H = ctx.shape[-1]
        if dy is None:  # y unused: only the residual stream carries a gradient
            dy = torch.zeros(ctx.shape, dtype=x.dtype, device=x.device)
        d2 = dres.reshape(-1, H).contiguous() if (dres is not None and ctx.has_res) else None
        am = _amax_buf(x, ctx.grad_amax)
        slot = ctx.slot
        if slot is not None:
            dest, acc = slot.engine._fused_slot_dest(slot)
            dx, _ = e.rmsnorm_bwd(dy.reshape(-1, H).contiguous(), x, w.contiguous(), rstd, d2, am, dest.view(-1), acc)
            slot.engine._fused_slot_done(slot)
            dw = None
        else:
            dx, dw = e.rmsnorm_bwd(dy.reshape(-1, H).contiguous(), x, w.contiguous(), rstd, d2, am)
        dx = dx.view(ctx.shape)
        if am is not None:
            from .fp8 import tag_amax

            tag_amax(dx, am)
        # d(x + residual) flows to both summands.
        return dx, dw, None, (dx if ctx.has_res else None), None, None, None


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6, residual: Optional[torch.Tensor] = None,
             amax: bool = False, grad_amax: bool = False, slot=None):
    """y = RMSNorm(x [+ residual]) * weight. Returns (y, residual_out) where residual_out = x + residual (or x).
    `amax` / `grad_amax`: tag y / the input gradient with their abs-max for a consuming fp8 linear (HIP path only).
    `slot`: the weight's FSDP gradient slot (see `_RMSNormFn`); every other path leaves the gradient to autograd."""
    if use_native(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        if slot is not None and not (torch.is_grad_enabled() and weight.requires_grad and weight.dtype == x.dtype
                                     and weight.is_contiguous()):
            slot = None
        if slot is not None and torch._C._current_graph_task_id() == -1:
            slot.uses += 1  # a forward whose backward is pending (recomputation inside backward is not counted)
        y, r, am = _RMSNormFn.apply(x, weight, eps, residual, amax, grad_amax, slot)
        if amax:
            from .fp8 import tag_amax

            tag_amax(y, am)
        return y, (r if residual is not None else x)
    return rms_norm_reference(x, weight, eps, residual)


# ----------------------------------------------------------------------------------------------------------
# SwiGLU on a fused [..., 2F] gate|up projection
# ----------------------------------------------------------------------------------------------------------
def swiglu_reference(gu):
    g, u = gu.float().chunk(2, dim=-1)
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, amax=False, grad_amax=False):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        ctx.grad_amax = grad_amax
        am = _amax_buf(gu, amax)
        h = ext().swiglu_fwd(gu, am)
        if am is None:
            am = torch.empty(0, device=gu.device)
        ctx.mark_non_differentiable(am)
        ctx.set_materialize_grads(False)
        return h, am

    @staticmethod
    def backward(ctx, dh, _dam):
        (gu,) = ctx.saved_tensors
        if dh is None:
            return None, None, None
        am = _amax_buf(gu, ctx.grad_amax)
        dgu = ext().swiglu_bwd(gu, dh.contiguous(), am)
        if am is not None:
            from .fp8 import tag_amax

            tag_amax(dgu, am)
        return dgu, None, None


def swiglu(gu: torch.Tensor, amax: bool = False, grad_amax: bool = False) -> torch.Tensor:
    """silu(gate) * up on a fused [..., 2F] projection. `amax` / `grad_amax` as in `rms_norm` (for the fp8 down / gate-up
    projections that consume the output / produce the input)."""
    if use_native(gu) and gu.dtype == torch.bfloat16 and (gu.shape[-1] // 2) % 8 == 0:
        h, am = _SwiGLUFn.apply(gu, amax, grad_amax)
        if amax:
            from .fp8 import tag_amax

            tag_amax(h, am)
        return h
    return swiglu_reference(gu)


# ----------------------------------------------------------------------------------------------------------
# Rotary embeddings (rotate-half convention, as Llama) applied to the Q and K heads of a fused QKV tensor
# ----------------------------------------------------------------------------------------------------------
def rope_tables(seq_len: int, head_dim: int, theta: float = 500000.0, device=None, scaling: Optional[dict] = None):
    """fp32 cos/sin tables [S, D/2]. `scaling` supports Llama-3.1 style frequency scaling."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64, device="cpu") / head_dim))
    if scaling is not None and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        low, high = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        low_wl, high_wl = old / low, old / high
        wl = 2 * math.pi / inv
        smooth = (old / wl - low) / (high - low)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(seq_len, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_reference(qkv, cos, sin, n_rot_heads, positions=None):
    """qkv [..., T, Htot, D] (token-major). Rotates heads [0, n_rot_heads)."""
    T = qkv.shape[-3]
    D = qkv.shape[-1]
    if positions is None:
        c, s = cos[:T], sin[:T]
    else:
        c, s = cos[positions.reshape(-1)], sin[positions.reshape(-1)]
        c = c.view(*positions.shape, D // 2)
        s = s.view(*positions.shape, D // 2)
    c = torch.cat([c, c], dim=-1).unsqueeze(-2)
    s = torch.cat([s, s], dim=-1).unsqueeze(-2)
    x = qkv[..., :n_rot_heads, :].float()
    x1, x2 = x[..., : D // 2], x[..., D // 2 :]
    rot = torch.cat([-x2, x1], dim=-1)
    out = x * c + rot * s
    return torch.cat([out.to(qkv.dtype), qkv[..., n_rot_heads:, :]], dim=-2)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, n_rot_heads, positions):
        # out of place: one read + one write of qkv (V heads copied through), not a clone followed by an in-place pass
        B, S, Htot, D = qkv.shape
        pos = positions.reshape(-1).contiguous() if positions is not None else None
        out = ext().rope_out(qkv, cos, sin, pos, n_rot_heads, Htot, D, 1.0)
        ctx.save_for_backward(cos, sin, pos if pos is not None else torch.empty(0))
        ctx.meta = (n_rot_heads, Htot, D, pos is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        cos, sin, pos = ctx.saved_tensors
        n_rot, Htot, D, has_pos = ctx.meta
        return ext().rope_out(g, cos, sin, pos if has_pos else None, n_rot, Htot, D, -1.0), None, None, None, None


def apply_rope(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_rot_heads: int, positions=None):
    """qkv: [B, S, Htot, D]; rotates the first `n_rot_heads` heads (Q heads then K heads)."""
    if use_native(qkv) and qkv.dtype == torch.bfloat16 and qkv.shape[-1] % 8 == 0:
        return _RopeFn.apply(qkv, cos, sin, n_rot_heads, positions)
    return rope_reference(qkv, cos, sin, n_rot_heads, positions)


# ----------------------------------------------------------------------------------------------------------
# Flash attention on a fused QKV tensor
# ----------------------------------------------------------------------------------------------------------
def attention_reference(q, k, v, causal=True, scale=None):
    """q [B,S,Hq,D], k/v [B,S,Hkv,D] → O [B,S,Hq,D] in fp32 math (GQA by head repetition)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    o = torch.nn.functional.scaled_dot_product_attention(qf, kf, vf, is_causal=causal, scale=scale)
    return o.transpose(1, 2).to(q.dtype)


class _FlashAttnQKVFn(torch.autograd.Function):
    """Attention reading Q/K/V in place from a fused [B, S, Hq+2Hkv, D] activation; the gradient is produced as
    one fused dQKV tensor (what the QKV projection's backward consumes)."""

    @staticmethod
    def forward(ctx, qkv, n_q, n_kv, causal, scale):
        q = qkv[:, :, :n_q]
        k = qkv[:, :, n_q : n_q + n_kv]
        v = qkv[:, :, n_q + n_kv :]
        o, lse = ext().flash_attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (n_q, n_kv, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        n_q, n_kv, causal, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        ext().flash_attn_bwd(
            do.contiguous(),
            qkv[:, :, :n_q],
            qkv[:, :, n_q : n_q + n_kv],
            qkv[:, :, n_q + n_kv :],
            o,
            lse,
            dqkv[:, :, :n_q],
            dqkv[:, :, n_q : n_q + n_kv],
            dqkv[:, :, n_q + n_kv :],
            scale,
            causal,
        )
        return dqkv, None, None, None, None


def flash_attention_qkv(qkv: torch.Tensor, n_q: int, n_kv: int, causal: bool = True, scale: Optional[float] = None):
    """qkv [B, S, n_q + 2 n_kv, D] → O [B, S, n_q, D]."""
    D = qkv.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if use_native(qkv):
        if qkv.dtype != torch.bfloat16 or D != 128 or qkv.shape[1] % 128 != 0:
            raise ValueError(
                f"HIP flash attention needs bf16, head_dim 128 and seq_len % 128 == 0 (got {qkv.dtype}, D={D}, S={qkv.shape[1]})"
            )
        return _FlashAttnQKVFn.apply(qkv, n_q, n_kv, causal, scale)
    q = qkv[:, :, :n_q]
    k = qkv[:, :, n_q : n_q + n_kv]
    v = qkv[:, :, n_q + n_kv :]
    return attention_reference(q, k, v, causal=causal, scale=scale)


def flash_attn_with_lse(q, k, v, causal=True, scale=None):
    """Forward-only attention returning (O, LSE[B,Hq,S]) — context parallelism's building block. k / v may be longer
    than q (a K/V prefix): the causal mask is then aligned bottom-right."""
    D = q.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if use_native(q):
        return ext().flash_attn_fwd(q, k, v, scale, causal)
    B, S, Hq, _ = q.shape
    Sk = k.shape[1]
    rep = Hq // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:  # bottom-right aligned when Sk > S (query i sees keys <= i + Sk - S), as the HIP kernel
        mask = torch.ones(S, Sk, dtype=torch.bool, device=q.device).triu(1 + Sk - S)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    o = torch.matmul(torch.softmax(s, dim=-1), vf)
    return o.transpose(1, 2).to(q.dtype), lse


# ----------------------------------------------------------------------------------------------------------
# Cross entropy (mean over non-ignored targets), gradient written in place over the logits
# ----------------------------------------------------------------------------------------------------------
class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, inplace_backward):
        V = logits.shape[-1]
        l2 = logits.reshape(-1, V)
        if not l2.is_contiguous():
            l2 = l2.contiguous()
        lab = labels.reshape(-1).contiguous()
        row_loss, lse = ext().xent_fwd(l2, lab, ignore_index)
        n_valid = (lab != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(l2, lab, lse, n_valid)
        ctx.meta = (ignore_index, inplace_backward, logits.shape)
        return row_loss.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        l2, lab, lse, n_valid = ctx.saved_tensors
        ignore_index, inplace, shape = ctx.meta
        scale = (g.float() / n_valid).reshape(1).contiguous()
        out = l2 if inplace else torch.empty_like(l2)
        ext().xent_bwd(l2, lab, lse, scale, out, ignore_index)
        return out.view(shape), None, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100, inplace_backward: bool = True):
    """Mean token cross-entropy. With `inplace_backward`, the logits buffer is overwritten by its gradient
    during backward (saves one logits-sized allocation: 2 GB for Llama-3 at 8k tokens)."""
    if use_native(logits) and logits.dtype == torch.bfloat16:
        return _CrossEntropyFn.apply(logits, labels, ignore_index, inplace_backward)
    return torch.nn.functional.cross_entropy(
        logits.reshape(-1, logits.shape[-1]).float(), labels.reshape(-1), ignore_index=ignore_index
    )


def linear_dgrad(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx = dy2 · W for a Linear's weight W [N, K] and output gradient dy2 [T, N].

    hipBLASLt's gfx950 kernels for this product in its natural layout (both operands row-major, the NN class) ran at
    1.35 PF/s in the Llama-3-8B step, its forward-class kernels (TN: the second operand contraction-contiguous) at
    1.54 PF/s. So on the native path W is first turned into a contiguous Wᵀ by the HIP transpose (4.6-6.7 TB/s,
    tools/bench_transpose.py; 436 MB of weights per Llama-3-8B layer ≈ 0.15 ms) and dx = linear(dy2, Wᵀ) runs in the
    forward's layout: 1.1-1.5 % faster end to end on one MI355X (gpu_steps.sh bench8b vs bench8b_dgradwt, two
    boxes). The copy is transient (freed as soon as the GEMM is enqueued)."""
    if (asm_dgrad_enabled() and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and dy2.is_contiguous() and use_native(dy2) and w.shape[1] % 256 == 0 and dy2.shape[0] % 256 == 0
            and w.shape[0] % 64 == 0 and w.shape[0] >= 128):
        out = torch.empty((dy2.shape[0], w.shape[1]), dtype=dy2.dtype, device=dy2.device)
        if ext().bf16_gemm_asm_amn(w, dy2, out, False, True):
            return out
    if _DGRAD_BLASLT and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous() \
            and dy2.is_contiguous() and use_native(dy2):
        # the NN product on a searched hipBLASLt algorithm (csrc/runtime/blaslt_gemm.cpp): no transposed weight copy
        out = torch.empty((dy2.shape[0], w.shape[1]), dtype=dy2.dtype, device=dy2.device)
        if ext().blaslt_dgrad_bf16(dy2, w, out):
            return out
    if (_DGRAD_WT and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0 and use_native(dy2)):
        wt = ext().transpose_bf16(w)
        dx = asm_gemm_bf16(dy2, wt, kind="dgrad") if dy2.is_contiguous() else None
        return dx if dx is not None else torch.nn.functional.linear(dy2, wt)
    return dy2 @ w


def wgrad_into(dest: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, accumulate: bool) -> None:
    """dest (+)= dy2ᵀ · x2: a Linear's weight gradient written by the GEMM itself into its engine slot (FSDP flat grad
    buffer / fp32 grad shard, DDP bucket). x2 is [T, K], token-major contiguous or the transposed view of the
    token-contiguous copy xᵀ the engines save. An fp32 `dest` takes the searched hipBLASLt runner when enabled
    (torch's fp32-output GEMM only reaches hipBLASLt's default heuristic), else torch."""
    a, b = dy2.t(), x2
    if b.dtype != a.dtype:
        b = b.to(a.dtype)
    if (dest.is_cuda and dest.is_contiguous() and a.dtype == torch.bfloat16 and dy2.is_contiguous()
            and dest.dtype in (torch.float32, torch.bfloat16) and use_native(dy2)
            and dy2.shape[1] % 256 == 0 and b.shape[1] % 256 == 0 and dy2.shape[0] % 64 == 0 and dy2.shape[0] >= 128):
        if _ASM_WGRAD_AMN and b.t().is_contiguous() and ext().bf16_gemm_asm_amn(dy2, b.t(), dest, accumulate, False):
            return
        if ASM_WGRAD_ABMN and b.is_contiguous() and ext().bf16_gemm_asm_amn(b, dy2, dest, accumulate, True, True):
            return
    # asm kernel: both operands token-contiguous -- x2 is the transposed view of the saved xᵀ, dy2 is transposed here
    if ("wgrad" in _ASM_BF16_KINDS and dest.is_cuda and dest.is_contiguous() and a.dtype == torch.bfloat16
            and b.t().is_contiguous()
            and dy2.is_contiguous() and dy2.shape[0] % 256 == 0 and dy2.shape[1] % 256 == 0 and b.shape[1] % 256 == 0
            and dest.dtype in (torch.float32, torch.bfloat16) and use_native(dy2)):
        if asm_gemm_bf16(ext().transpose_bf16(dy2), b.t(), None, dest, accumulate, kind="wgrad") is not None:
            return
    if dest.dtype == a.dtype:
        dest.addmm_(a, b) if accumulate else torch.mm(a, b, out=dest)
    elif dest.is_cuda and dest.dtype == torch.float32:
        if _BLASLT_WGRAD and a.dtype == torch.bfloat16 and dy2.is_contiguous():
            if (_WGRAD_DYT and b.t().is_contiguous() and dy2.shape[0] % 64 == 0 and dy2.shape[1] % 64 == 0
                    and ext().blaslt_wgrad_f32(ext().transpose_bf16(dy2), b.t(), dest, accumulate, True, True)):
                return
            if b.is_contiguous() and ext().blaslt_wgrad_f32(dy2, b, dest, accumulate, False):
                return
            if b.t().is_contiguous() and ext().blaslt_wgrad_f32(dy2, b.t(), dest, accumulate, True):
                return
        if accumulate:
            torch.addmm(dest, a, b, out_dtype=torch.float32, out=dest)
        else:
            torch.mm(a, b, out_dtype=torch.float32, out=dest)
    else:
        g = (a.float() @ b.float()).to(dest.dtype)
        dest.add_(g) if accumulate else dest.copy_(g)
