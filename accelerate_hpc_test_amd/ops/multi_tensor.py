"""Multi-tensor HIP kernels: fused Adam/AdamW, global L2 gradient norm and device-side clipping.

One kernel launch covers a whole list of tensors: the host packs (pointer, numel) metadata once, uploads it with
one small copy, and the kernel maps each workgroup to a (tensor, 8192-element chunk). The metadata is cached per
tensor-list identity, so steady-state steps cost one launch per parameter group.

`FusedAdamStep` executes `torch.optim.AdamW` / `torch.optim.Adam` semantics on the optimizer's own param groups
and state (`step`, `exp_avg`, `exp_avg_sq` kept in torch's format, so checkpoints are interchangeable).
Parity target: the optimizer step the reference delegates to torch (`/root/reference/src/accelerate/optimizer.py:145-181`).
"""

from __future__ import annotations

import math
import os
from typing import Iterable, Optional

import torch

from ._ext import ext, use_native

_DT = {torch.float32: 0, torch.bfloat16: 1}
# The fused AdamW also reduces max |bf16(p)| of FSDP fp8-gathered weights into their amax slots (their per-step
# re-quantisation then skips its amax pass over the bf16 shards); ACCELERATE_FP8_AMAX_IN_ADAM=0 turns that off.
_AMAX_IN_ADAM = os.environ.get("ACCELERATE_FP8_AMAX_IN_ADAM", "1") != "0"
_META_COLS = 7  # TensorMeta: p, g, m, v, shadow, n, amax


class _MetaCache:
    def __init__(self):
        self._cache = {}

    def get(self, rows: list[tuple[int, ...]], device):
        key = (tuple(rows), str(device))
        hit = self._cache.get(key)
        if hit is not None:
            return hit
        chunk = ext().multi_tensor_chunk()
        rows = [tuple(r) + (0,) * (_META_COLS - len(r)) for r in rows]  # absent trailing fields (amax) are 0
        meta = torch.tensor(rows, dtype=torch.int64) if rows else torch.zeros((0, _META_COLS), dtype=torch.int64)
        nblocks = [(r[5] + chunk - 1) // chunk for r in rows]
        prefix = [0]
        for n in nblocks:
            prefix.append(prefix[-1] + n)
        entry = (
            meta.to(device, non_blocking=False),
            torch.tensor(prefix, dtype=torch.int64).to(device),
            prefix[-1],
        )
        if len(self._cache) > 64:
            self._cache.clear()
        self._cache[key] = entry
        return entry


_CACHE = _MetaCache()


def _merge_contiguous(rows):
    """Merge rows whose p/g/m/v/shadow ranges are adjacent in memory (per-parameter views of one flat FSDP shard
    become a single range → aligned vector access, fewer chunk boundaries). Rows are (p, g, m, v, shadow, n, p / g / m
    element sizes, amax); a row with an amax slot stays on its own (the slot covers exactly that tensor)."""
    if not rows:
        return rows
    out = [list(rows[0])]
    for r in rows[1:]:
        prev = out[-1]
        n = prev[5]
        ok = prev[9] == 0 and r[9] == 0
        for idx, esz in ((0, r[6]), (1, r[7]), (2, r[8]), (3, r[8])):
            if prev[idx] + n * esz != r[idx]:
                ok = False
                break
        if ok and (prev[4] == 0) == (r[4] == 0) and (r[4] == 0 or prev[4] + n * 2 == r[4]) and prev[6:] == list(r[6:]):
            prev[5] += r[5]
        else:
            out.append(list(r))
    return [tuple(x[:6]) + (x[9],) for x in out]


def adam_state_dtype(param: torch.Tensor) -> torch.dtype:
    """dtype of new `exp_avg` / `exp_avg_sq` tensors: the param's (torch's rule) unless ACCELERATE_ADAM_STATE_DTYPE=bf16
    asks for bf16 moments beside fp32 master weights (4 bytes less per parameter and 8 bytes less of optimizer traffic
    per step; the update itself still runs in fp32 registers)."""
    if param.dtype == torch.float32 and os.environ.get("ACCELERATE_ADAM_STATE_DTYPE", "fp32").lower() in ("bf16", "bfloat16"):
        return torch.bfloat16
    return param.dtype


class FusedAdamStep:
    """Runs Adam/AdamW for a torch optimizer with one HIP launch per param group."""

    def __init__(self, optimizer: torch.optim.Optimizer):
        self.optimizer = optimizer
        self.adamw = isinstance(optimizer, torch.optim.AdamW)

    @torch.no_grad()
    def step(self, grad_scale: Optional[torch.Tensor] = None, only: Optional[set] = None, skip: Optional[set] = None):
        """Update every param with a grad, or only those whose id() is in `only` / not in `skip` (the per-unit
        updates of `fsdp_optimizer_overlap`, and the remainder at `optimizer.step()`)."""
        opt = self.optimizer
        e = ext()
        amax_units = {}  # FSDP units whose fp8 amax slots this call fills: id -> (engine, unit, ids of updated params)
        expert_amax = []  # MoE expert-stack amax holders this call fills (one kernel row per expert)
        for group in opt.param_groups:
            lr = group["lr"]
            if isinstance(lr, torch.Tensor):
                lr = float(lr)
            beta1, beta2 = group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            rows = []
            dtypes = None
            step_val = None
            for p in group["params"]:
                if p.grad is None or p.numel() == 0:
                    continue
                if (only is not None and id(p) not in only) or (skip is not None and id(p) in skip):
                    continue
                st = opt.state[p]
                if len(st) == 0:
                    sdt = adam_state_dtype(p)
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, dtype=sdt, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=sdt, memory_format=torch.preserve_format)
                elif st["exp_avg"].dtype != adam_state_dtype(p) and st["exp_avg"].dtype == torch.float32:
                    # bf16 moments requested but the state came back fp32 (torch's load_state_dict casts optimizer state
                    # to the param dtype): narrow it once
                    st["exp_avg"] = st["exp_avg"].to(torch.bfloat16)
                    st["exp_avg_sq"] = st["exp_avg_sq"].to(torch.bfloat16)
                st["step"] += 1
                s = float(st["step"]) if step_val is None else step_val
                step_val = s
                g = p.grad
                m, v = st["exp_avg"], st["exp_avg_sq"]
                for t in (p, g, m, v):
                    if not t.is_contiguous():
                        raise RuntimeError("FusedAdamStep requires contiguous params/grads/state")
                dt = (_DT[p.dtype], _DT[g.dtype], _DT[m.dtype])
                if dtypes is None:
                    dtypes = dt
                elif dtypes != dt:
                    # Mixed dtypes within a group: flush what we have and start a new launch.
                    self._launch(e, rows, dtypes, lr, beta1, beta2, eps, wd, step_val, grad_scale, p.device)
                    rows, dtypes = [], dt
                shadow = getattr(p, "_acc_bf16_shadow", None)
                segs = getattr(p, "_acc_fp8_amax_segs", None) if (_AMAX_IN_ADAM and shadow is not None) else None
                if segs is not None and segs.seg * segs.amax.numel() == p.numel():
                    segs.amax.zero_()  # stream-ordered before the launch that max-reduces into it
                    expert_amax.append(segs)
                    es = (p.element_size(), g.element_size(), m.element_size())
                    for k in range(segs.amax.numel()):
                        o = k * segs.seg
                        rows.append((p.data_ptr() + o * es[0], g.data_ptr() + o * es[1], m.data_ptr() + o * es[2],
                                     v.data_ptr() + o * es[2], shadow.data_ptr() + o * 2, segs.seg, *es,
                                     segs.amax.data_ptr() + 4 * k))
                    continue
                amax_ptr = 0
                amax_ref = getattr(p, "_acc_fp8_amax", None) if (_AMAX_IN_ADAM and shadow is not None) else None
                if amax_ref is not None:
                    eng, unit, slot = amax_ref
                    if id(unit) not in amax_units:
                        unit.f8_amax.zero_()  # stream-ordered before the launch that max-reduces into it
                        amax_units[id(unit)] = (eng, unit, set())
                    amax_units[id(unit)][2].add(id(p))
                    amax_ptr = slot.data_ptr()
                rows.append(
                    (
                        p.data_ptr(),
                        g.data_ptr(),
                        m.data_ptr(),
                        v.data_ptr(),
                        shadow.data_ptr() if shadow is not None else 0,
                        p.numel(),
                        p.element_size(),
                        g.element_size(),
                        m.element_size(),
                        amax_ptr,
                    )
                )
            if rows:
                self._launch(e, rows, dtypes, lr, beta1, beta2, eps, wd, step_val, grad_scale, group["params"][0].device)
        for eng, unit, seen in amax_units.values():
            eng.fp8_amax_from_optimizer(unit, seen)
        for h in expert_amax:
            h.fresh = True

    def _launch(self, e, rows, dtypes, lr, beta1, beta2, eps, wd, step, grad_scale, device):
        if not rows:
            return
        merged = _merge_contiguous(rows)
        meta, prefix, nblocks = _CACHE.get(merged, device)
        bc1 = 1.0 - beta1**step
        bc2_sqrt = math.sqrt(1.0 - beta2**step)
        e.adam_multi_tensor(meta, prefix, nblocks, dtypes[0], dtypes[1], dtypes[2], lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, self.adamw, grad_scale)


def _grad_rows(params, dtype):
    rows = []
    for p in params:
        g = p.grad
        if g is None or g.numel() == 0 or g.dtype != dtype:
            continue
        if not g.is_contiguous():
            raise RuntimeError("multi-tensor grad norm requires contiguous grads")
        rows.append((0, g.data_ptr(), 0, 0, 0, g.numel()))
    return rows


@torch.no_grad()
def grad_sq_norm(params: Iterable[torch.nn.Parameter], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum of squares of all grads (fp32 device scalar [1]); one launch per grad dtype."""
    params = [p for p in params if p.grad is not None]
    if not params:
        return torch.zeros(1)
    dev = params[0].grad.device
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=dev)
    if not use_native(params[0].grad):
        acc = torch.zeros((), dtype=torch.float32, device=dev)
        for p in params:
            acc += p.grad.float().pow(2).sum()
        out.copy_(acc.reshape(1))
        return out
    e = ext()
    first = True
    for dt in (torch.float32, torch.bfloat16):
        rows = _grad_rows(params, dt)
        if not rows:
            continue
        meta, prefix, nb = _CACHE.get(rows, dev)
        e.sqnorm_multi_tensor(meta, prefix, nb, _DT[dt], out, not first)
        first = False
    if first:
        out.zero_()
    return out


@torch.no_grad()
def clip_grads_by_total_sq(params, total_sq: torch.Tensor, max_norm: float):
    """Scale grads by min(1, max_norm / (sqrt(total_sq) + 1e-6)) entirely on device (no host sync)."""
    params = [p for p in params if p.grad is not None]
    if not params:
        return
    if not use_native(params[0].grad):
        coef = (max_norm / (total_sq.sqrt() + 1e-6)).clamp(max=1.0)
        for p in params:
            p.grad.mul_(coef.to(p.grad.device, p.grad.dtype))
        return
    e = ext()
    dev = params[0].grad.device
    for dt in (torch.float32, torch.bfloat16):
        rows = _grad_rows(params, dt)
        if rows:
            meta, prefix, nb = _CACHE.get(rows, dev)
            e.clip_multi_tensor(meta, prefix, nb, _DT[dt], total_sq, max_norm)


@torch.no_grad()
def unscale_and_check(grads: list, inv_scale: torch.Tensor, found_inf: torch.Tensor):
    """In-place `g *= inv_scale` over a list of same-device grads, setting `found_inf` (fp32 [1]) to 1 when any result is
    inf / NaN — one HIP launch per grad dtype (torch's `_amp_foreach_non_finite_check_and_unscale_`)."""
    grads = [g for g in grads if g is not None and g.numel() > 0]
    if not grads:
        return
    if not use_native(grads[0]):
        torch._amp_foreach_non_finite_check_and_unscale_(grads, found_inf, inv_scale)
        return
    e, dev = ext(), grads[0].device
    for dt in (torch.float32, torch.bfloat16):
        rows = [(0, g.data_ptr(), 0, 0, 0, g.numel()) for g in grads if g.dtype == dt]
        if rows:
            meta, prefix, nb = _CACHE.get(rows, dev)
            e.unscale_multi_tensor(meta, prefix, nb, _DT[dt], inv_scale, found_inf)
    other = [g for g in grads if g.dtype not in _DT]
    if other:  # fp16 grads (fp16 master weights): torch's kernel
        torch._amp_foreach_non_finite_check_and_unscale_(other, found_inf, inv_scale)


class CpuFusedAdamStep:
    """Adam/AdamW for CPU-resident fp32 params (FSDP CPU offload): the native OpenMP kernel
    (`csrc/runtime/cpu_adam.cpp`), one call per parameter, also writing the bf16 upload copy when the engine attached
    one (`p._acc_bf16_shadow_host`). Same `state` layout as torch."""

    def __init__(self, optimizer: torch.optim.Optimizer):
        self.optimizer = optimizer
        self.adamw = isinstance(optimizer, torch.optim.AdamW)

    @torch.no_grad()
    def step(self, grad_scale=None, only: Optional[set] = None, skip: Optional[set] = None):
        opt, e = self.optimizer, ext()
        for group in opt.param_groups:
            lr = float(group["lr"])
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None or p.numel() == 0:
                    continue
                if (only is not None and id(p) not in only) or (skip is not None and id(p) in skip):
                    continue
                st = opt.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                s = float(st["step"])
                g = p.grad if grad_scale is None else p.grad / float(grad_scale)
                e.cpu_adam_step(p.data, g, st["exp_avg"], st["exp_avg_sq"], getattr(p, "_acc_bf16_shadow_host", None),
                                lr, beta1, beta2, group["eps"], group["weight_decay"], 1.0 - beta1**s,
                                math.sqrt(1.0 - beta2**s), self.adamw)
