"""Mixed-precision context managers and model-size helpers (big-model planner lives in big_modeling_utils.py).

Parity: `/root/reference/src/accelerate/utils/modeling.py:2049-2131` (`get_mixed_precision_context_manager`,
`get_grad_scaler`) and the size helpers `compute_module_sizes`, `named_module_tensors`, `dtype_byte_size`
(`modeling.py:120-160,698-760`). The size accounting here is a single pass over `named_parameters` /
`named_buffers` that credits every ancestor prefix of a tensor's name; byte sizes come from a table of
torch dtypes (plus the planner's sub-byte custom dtypes) instead of parsing dtype names.
"""

from __future__ import annotations

import contextlib
import re
from collections import defaultdict
from typing import Dict, Iterator, Optional, Tuple, Union

import torch
import torch.nn as nn

from .dataclasses import AutocastKwargs, CustomDtype, DistributedType

# bf16 autocast is valid on every backend this framework runs (RCCL / gloo / single device).
_BF16_AUTOCAST_TYPES = (DistributedType.NO, DistributedType.MULTI_CPU, DistributedType.MULTI_GPU, DistributedType.FSDP)


def get_mixed_precision_context_manager(native_amp: bool = False, autocast_kwargs: Optional[AutocastKwargs] = None):
    """torch.autocast for the accelerator's mixed precision, or a null context when native AMP is off."""
    if not native_amp:
        return contextlib.nullcontext()
    from ..state import AcceleratorState

    state = AcceleratorState()
    extra = {} if autocast_kwargs is None else autocast_kwargs.to_kwargs()
    dev = "cuda" if state.device.type == "cuda" else "cpu"
    mp = state.mixed_precision
    if mp == "fp16":
        return torch.autocast(device_type=dev, dtype=torch.float16, **extra)
    if mp in ("bf16", "fp8") and state.distributed_type in _BF16_AUTOCAST_TYPES:
        return torch.autocast(device_type=dev, dtype=torch.bfloat16, **extra)
    return contextlib.nullcontext()


def get_grad_scaler(distributed_type: DistributedType = None, **kwargs):
    return torch.amp.GradScaler("cuda" if torch.cuda.is_available() else "cpu", **kwargs)


# Bytes per element. Fractions for the packed sub-byte formats the device-map planner sizes.
_SUBBYTE = {torch.bool: 1 / 8, CustomDtype.INT2: 1 / 4, CustomDtype.INT4: 1 / 2, CustomDtype.FP8: 1}


def dtype_byte_size(dtype: Union[torch.dtype, str]):
    """Storage bytes per element of `dtype` (int for whole-byte types, a fraction for packed ones)."""
    if dtype in _SUBBYTE:
        return _SUBBYTE[dtype]
    if isinstance(dtype, torch.dtype):
        return dtype.itemsize
    # String forms such as "float16" / "torch.int8" / "fp8_e4m3": the first run of digits is the bit width.
    bits = re.search(r"\D(\d+)", "_" + str(dtype).replace("torch.", ""))
    if bits is None:
        raise ValueError(f"`dtype` is not a valid dtype: {dtype}.")
    return int(bits.group(1)) // 8


def named_module_tensors(
    module: nn.Module, include_buffers: bool = True, recurse: bool = False, remove_non_persistent: bool = False
) -> Iterator[Tuple[str, torch.Tensor]]:
    """Parameters, then (optionally persistent-only) buffers of `module`."""
    yield from module.named_parameters(recurse=recurse)
    if not include_buffers:
        return
    skip = get_non_persistent_buffers(module, recurse=recurse) if remove_non_persistent else set()
    yield from ((n, b) for n, b in module.named_buffers(recurse=recurse) if n not in skip)


def get_non_persistent_buffers(module: nn.Module, recurse: bool = False, fqns: bool = False):
    """Names of buffers excluded from the state dict; with `fqns`, fully qualified from `module`.

    Returns a new set: the module's own `_non_persistent_buffers_set` is never extended with descendants' names.
    """
    names = set(module._non_persistent_buffers_set)
    if not recurse:
        return names
    for prefix, sub in module.named_modules():
        for b in sub._non_persistent_buffers_set:
            names.add(f"{prefix}.{b}" if (fqns and prefix) else b)
    return names


def _get_proper_dtype(dtype):
    return getattr(torch, dtype.replace("torch.", "")) if isinstance(dtype, str) else dtype


def _prefixes(name: str):
    parts = name.split(".")
    return (".".join(parts[:i]) for i in range(len(parts) + 1))


def compute_module_sizes(model: nn.Module, dtype=None, special_dtypes=None, buffers_only: bool = False) -> Dict[str, int]:
    """Bytes per module name ("" = whole model), optionally as if floating tensors were cast down to `dtype`.

    Integer / bool tensors keep their own width; a cast never widens a tensor (`min` of the two widths);
    `special_dtypes` pins the dtype of named tensors.
    """
    cast_width = None if dtype is None else dtype_byte_size(_get_proper_dtype(dtype))
    pinned = {k: dtype_byte_size(_get_proper_dtype(v)) for k, v in (special_dtypes or {}).items()}
    tensors = model.named_buffers(recurse=True) if buffers_only else named_module_tensors(model, recurse=True)
    sizes: Dict[str, int] = defaultdict(int)
    for name, t in tensors:
        own = dtype_byte_size(t.dtype)
        if name in pinned:
            width = pinned[name]
        elif cast_width is None or not (t.dtype.is_floating_point or t.dtype.is_complex):
            width = own
        else:
            width = min(cast_width, own)
        nbytes = t.numel() * width
        for p in _prefixes(name):
            sizes[p] += nbytes
    return sizes


def compute_module_total_buffer_size(model: nn.Module, dtype=None, special_dtypes=None):
    return compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes, buffers_only=True).get("", 0)


# Unit suffix -> (multiplier, decimal unit that means bits when written lower-case 'b').
_UNITS = (
    ("GIB", 2**30, False),
    ("MIB", 2**20, False),
    ("KIB", 2**10, False),
    ("GB", 10**9, True),
    ("MB", 10**6, True),
    ("KB", 10**3, True),
)


def convert_file_size_to_int(size: Union[int, str]):
    """'10GB' -> bytes: powers of 10 for GB/MB/KB ('Gb' etc. are bits), powers of 2 for GiB/MiB/KiB."""
    err = f"`size` {size} is not in a valid format. Use an integer for bytes, or a string with an unit (like '5.0GB')."
    if isinstance(size, int):
        if size < 0:
            raise ValueError(err)
        return size
    upper = size.upper()
    for suffix, mult, bits_if_lower in _UNITS:
        if upper.endswith(suffix):
            try:
                value = int(float(size[: -len(suffix)]) * mult)
            except ValueError:
                raise ValueError(err) from None
            if bits_if_lower and size.endswith("b"):
                value //= 8
            if value < 0:
                raise ValueError(err)
            return value
    raise ValueError(err)


def id_tensor_storage(tensor: torch.Tensor):
    """Key that is equal for tensors sharing one storage (tied weights)."""
    st = tensor.untyped_storage()
    return tensor.device, st.data_ptr() if tensor.numel() else id(tensor), st.nbytes()
