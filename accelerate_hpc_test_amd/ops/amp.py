"""fp16 AMP loss scaling with the unscale / overflow check on our multi-tensor HIP kernel.

`HipGradScaler` is `torch.amp.GradScaler` (same API, state_dict, growth / backoff logic — what the reference's
`Accelerator` builds at `/root/reference/src/accelerate/accelerator.py:561-575`) whose `unscale_` runs
`ops/multi_tensor.py::unscale_and_check`: one launch per grad dtype multiplies every gradient by 1/scale in place and
raises the found-inf flag on any inf / NaN, instead of torch's per-dtype foreach kernel. Sparse and non-contiguous
gradients, and CPU tensors, keep torch's kernel.
"""

from __future__ import annotations

from collections import defaultdict

import torch
from torch.amp.grad_scaler import _MultiDeviceReplicator

from .multi_tensor import unscale_and_check


class HipGradScaler(torch.amp.GradScaler):
    def _unscale_grads_(self, optimizer, inv_scale, found_inf, allow_fp16):
        per_device_inv_scale = _MultiDeviceReplicator(inv_scale)
        per_device_found_inf = _MultiDeviceReplicator(found_inf)
        native = defaultdict(list)  # device -> dense contiguous GPU grads
        fallback = defaultdict(lambda: defaultdict(list))  # device -> dtype -> grads for torch's kernel
        with torch.no_grad():
            for group in optimizer.param_groups:
                for param in group["params"]:
                    g = param.grad
                    if g is None:
                        continue
                    if not allow_fp16 and g.dtype == torch.float16:
                        raise ValueError("Attempting to unscale FP16 gradients.")
                    if g.is_sparse:
                        if g.dtype is torch.float16:
                            param.grad = g = g.coalesce()
                        fallback[g.device][g.dtype].append(g._values())
                    elif g.is_cuda and g.is_contiguous() and g.dtype in (torch.float32, torch.bfloat16):
                        native[g.device].append(g)
                    else:
                        fallback[g.device][g.dtype].append(g)
            for device, grads in native.items():
                unscale_and_check(grads, per_device_inv_scale.get(device), per_device_found_inf.get(device))
            for device, per_dtype in fallback.items():
                for grads in per_dtype.values():
                    torch._amp_foreach_non_finite_check_and_unscale_(
                        grads, per_device_found_inf.get(device), per_device_inv_scale.get(device))
        return per_device_found_inf._per_device_tensors
