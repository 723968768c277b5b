"""Moving individual parameters / buffers of a module between devices (GPU, host, meta) and keeping tied
parameters tied while doing so.

Reference behaviour: `/root/reference/src/accelerate/utils/modeling.py:217-425,609-637,2134-2186`
(`set_module_tensor_to_device`, `retie_parameters`, `has_offloaded_params`, `align_module_device`).
`tests/test_big_modeling.py` pins the semantics.
"""

from __future__ import annotations

import contextlib
from typing import Optional, Union

import torch
import torch.nn as nn

from .device_map import find_tied_parameters  # noqa: F401  (re-exported: the reference keeps both in one module)

_INTEGRAL = ("torch.uint", "torch.int", "torch.bool")


def _is_integral(t: torch.Tensor) -> bool:
    return str(t.dtype).startswith(_INTEGRAL)


def _resolve(module: nn.Module, dotted: str):
    """(owning module, attribute name) of a dotted tensor name."""
    owner_path, _, attr = dotted.rpartition(".")
    owner = module
    for part in owner_path.split(".") if owner_path else ():
        owner = getattr(owner, part)
        if owner is None:
            raise ValueError(f"{module} has no attribute {part}.")
    return owner, attr


def _same_device(a, b) -> bool:
    a, b = torch.device(a), torch.device(b)
    if a.type != b.type:
        return False
    if a.type == "cuda":
        cur = torch.cuda.current_device() if torch.cuda.is_available() else 0
        return (a.index if a.index is not None else cur) == (b.index if b.index is not None else cur)
    return True


def _device_key(device):
    """`device` as given (int GPU ordinals stay ints), the key used in tied-parameter caches."""
    return device


def set_module_tensor_to_device(
    module: nn.Module,
    tensor_name: str,
    device: Union[int, str, torch.device],
    value: Optional[torch.Tensor] = None,
    dtype: Optional[Union[str, torch.dtype]] = None,
    fp16_statistics: Optional[torch.Tensor] = None,
    tied_params_map: Optional[dict] = None,
    non_blocking: bool = False,
    clear_cache: bool = True,
):
    """Put parameter / buffer `tensor_name` (dotted) of `module` on `device`, optionally replacing its data by
    `value` (cast to the old dtype, or to `dtype` for floating values). The Parameter subclass and `requires_grad`
    survive; a `tied_params_map` ({data_ptr: {device: tensor}}) lets tied parameters share one copy per device."""
    owner, attr = _resolve(module, tensor_name)
    is_param = attr in owner._parameters
    if not is_param and attr not in owner._buffers:
        raise ValueError(f"{module} does not have a parameter or a buffer named {attr}.")
    old = getattr(owner, attr)

    if tied_params_map is not None:
        for ptr in ((value.data_ptr(),) if value is not None else ()) + (old.data_ptr(),):
            cached = tied_params_map.get(ptr, {})
            if device in cached:
                owner._parameters[attr] = cached[device]
                return

    to_meta = str(device) == "meta"
    if old.device.type == "meta" and not to_meta and value is None:
        raise ValueError(f"{attr} is on the meta device, we need a `value` to put in on {device}.")
    if isinstance(dtype, str):
        dtype = getattr(torch, dtype.replace("torch.", ""))

    if value is not None:
        if old.shape != value.shape and type(old).__name__ != "Params4bit":
            raise ValueError(
                f'Trying to set a tensor of shape {value.shape} in "{attr}" (which has shape {old.shape}), this looks incorrect.'
            )
        if dtype is None:
            value = value.to(old.dtype, non_blocking=non_blocking)
        elif not _is_integral(value):
            value = value.to(dtype, non_blocking=non_blocking)

    with torch.no_grad():
        if value is None:
            new = old.to(device, non_blocking=non_blocking)
            if dtype is not None and to_meta and not _is_integral(old):
                new = new.to(dtype, non_blocking=non_blocking)
                if is_param:
                    owner._parameters[attr] = type(old)(new, requires_grad=old.requires_grad)
        elif isinstance(value, torch.Tensor):
            new = value.to(device, non_blocking=non_blocking)
        else:
            new = torch.tensor(value, device=device)

        if not is_param:
            owner._buffers[attr] = new
        elif value is not None or not _same_device(device, owner._parameters[attr].device):
            cur = owner._parameters[attr]
            cls = type(cur)
            if cls.__name__ in ("Int8Params", "FP4Params", "Params4bit"):
                owner._parameters[attr] = cls(new, requires_grad=old.requires_grad, **cur.__dict__).to(device)
            else:
                owner._parameters[attr] = cls(new, requires_grad=old.requires_grad)
            new = owner._parameters[attr]

    if tied_params_map is not None:
        for ptr in (old.data_ptr(),) + ((value.data_ptr(),) if value is not None else ()):
            if ptr in tied_params_map and device not in tied_params_map[ptr]:
                tied_params_map[ptr][device] = new
                break


def retie_parameters(model: nn.Module, tied_params: list):
    """Make every name of each tied group point at one Parameter again: the group's first non-meta member."""
    for group in tied_params:
        anchor = None
        for name in group:
            owner, attr = _resolve(model, name)
            p = getattr(owner, attr)
            if p.device.type != "meta":
                anchor = p
                break
        if anchor is None:
            continue
        for name in group:
            owner, attr = _resolve(model, name)
            setattr(owner, attr, anchor)


def recursive_getattr(obj, attr: str):
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def has_offloaded_params(module: nn.Module) -> bool:
    """Whether `module` has an offloading hook attached (its weights live on the host / disk between forwards)."""
    from ..hooks import AlignDevicesHook

    hook = getattr(module, "_hf_hook", None)
    return isinstance(hook, AlignDevicesHook) and bool(hook.offload)


@contextlib.contextmanager
def align_module_device(module: nn.Module, execution_device=None):
    """Within the context, `module`'s own parameters are materialised on `execution_device` (offloaded modules: by
    running their hook's load / release; resident ones: moved there and back)."""
    if has_offloaded_params(module):
        hook = module._hf_hook
        saved = hook.execution_device
        if execution_device is not None:
            hook.execution_device = execution_device
        try:
            hook.pre_forward(module)
            yield
        finally:
            hook.post_forward(module, None)
            hook.execution_device = saved
        return
    if execution_device is None:
        yield
        return
    homes = {n: p.device for n, p in module.named_parameters(recurse=False)}
    try:
        for n in homes:
            set_module_tensor_to_device(module, n, execution_device)
        yield
    finally:
        for n, d in homes.items():
            set_module_tensor_to_device(module, n, d)
