"""Mixed-precision context managers and model-size helpers (big-model planner lives in big_modeling_utils.py).

Parity: `/root/reference/src/accelerate/utils/modeling.py:2049-2131` (`get_mixed_precision_context_manager`,
`get_grad_scaler`) and the size helpers `compute_module_sizes`, `named_module_tensors`, `dtype_byte_size`.
"""

from __future__ import annotations

import contextlib
import re
from collections import defaultdict
from typing import Optional, Union

import torch
import torch.nn as nn

from .dataclasses import AutocastKwargs, CustomDtype, DistributedType


def get_mixed_precision_context_manager(native_amp: bool = False, autocast_kwargs: Optional[AutocastKwargs] = None):
    state_mp = None
    from ..state import AcceleratorState

    state = AcceleratorState()
    if autocast_kwargs is None:
        autocast_kwargs = {}
    else:
        autocast_kwargs = autocast_kwargs.to_kwargs()
    if native_amp:
        device_type = "cuda" if state.device.type == "cuda" else "cpu"
        if state.mixed_precision == "fp16":
            return torch.autocast(device_type=device_type, dtype=torch.float16, **autocast_kwargs)
        elif state.mixed_precision in ("bf16", "fp8") and state.distributed_type in (
            DistributedType.NO,
            DistributedType.MULTI_CPU,
            DistributedType.MULTI_GPU,
            DistributedType.FSDP,
        ):
            return torch.autocast(device_type=device_type, dtype=torch.bfloat16, **autocast_kwargs)
    _ = state_mp
    return contextlib.nullcontext()


def get_grad_scaler(distributed_type: DistributedType = None, **kwargs):
    device = "cuda" if torch.cuda.is_available() else "cpu"
    return torch.amp.GradScaler(device, **kwargs)


def dtype_byte_size(dtype: Union[torch.dtype, str]):
    if dtype == torch.bool:
        return 1 / 8
    elif dtype == CustomDtype.INT2:
        return 1 / 4
    elif dtype == CustomDtype.INT4:
        return 1 / 2
    elif dtype == CustomDtype.FP8:
        return 1
    elif isinstance(dtype, torch.dtype) and dtype.is_floating_point is False and "int" not in str(dtype):
        pass
    bit_search = re.search(r"[^\d](\d+)_?", str(dtype))
    if bit_search is None:
        raise ValueError(f"`dtype` is not a valid dtype: {dtype}.")
    bit_size = int(bit_search.groups()[0])
    return bit_size // 8


def named_module_tensors(module: nn.Module, include_buffers: bool = True, recurse: bool = False, remove_non_persistent: bool = False):
    yield from module.named_parameters(recurse=recurse)
    if include_buffers:
        non_persistent_buffers = set()
        if remove_non_persistent:
            non_persistent_buffers = get_non_persistent_buffers(module, recurse=recurse)
        for named_buffer in module.named_buffers(recurse=recurse):
            name, _ = named_buffer
            if name not in non_persistent_buffers:
                yield named_buffer


def get_non_persistent_buffers(module: nn.Module, recurse: bool = False, fqns: bool = False):
    non_persistent_buffers_set = module._non_persistent_buffers_set
    if recurse:
        for n, m in module.named_modules():
            if fqns:
                non_persistent_buffers_set |= {n + "." + b if n else b for b in m._non_persistent_buffers_set}
            else:
                non_persistent_buffers_set |= m._non_persistent_buffers_set
    return non_persistent_buffers_set


def compute_module_sizes(model: nn.Module, dtype=None, special_dtypes=None, buffers_only: bool = False):
    """Bytes per module name ("" = whole model), optionally as if cast to `dtype`."""
    if dtype is not None:
        dtype = _get_proper_dtype(dtype)
        dtype_size = dtype_byte_size(dtype)
    if special_dtypes is not None:
        special_dtypes = {key: _get_proper_dtype(dtyp) for key, dtyp in special_dtypes.items()}
        special_dtypes_size = {key: dtype_byte_size(dtyp) for key, dtyp in special_dtypes.items()}
    module_sizes = defaultdict(int)
    module_list = []
    if not buffers_only:
        module_list = named_module_tensors(model, recurse=True)
    else:
        module_list = model.named_buffers(recurse=True)
    for name, tensor in module_list:
        if special_dtypes is not None and name in special_dtypes:
            size = tensor.numel() * special_dtypes_size[name]
        elif dtype is None:
            size = tensor.numel() * dtype_byte_size(tensor.dtype)
        elif str(tensor.dtype).startswith(("torch.uint", "torch.int", "torch.bool")):
            size = tensor.numel() * dtype_byte_size(tensor.dtype)
        else:
            size = tensor.numel() * min(dtype_size, dtype_byte_size(tensor.dtype))
        name_parts = name.split(".")
        for idx in range(len(name_parts) + 1):
            module_sizes[".".join(name_parts[:idx])] += size
    return module_sizes


def compute_module_total_buffer_size(model: nn.Module, dtype=None, special_dtypes=None):
    module_sizes = compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes, buffers_only=True)
    return module_sizes.get("", 0)


def _get_proper_dtype(dtype):
    if isinstance(dtype, str):
        dtype = dtype.replace("torch.", "")
        dtype = getattr(torch, dtype)
    return dtype


def convert_file_size_to_int(size: Union[int, str]):
    """'10GB' → bytes (powers of 10 for GB/MB/KB, powers of 2 for GiB/MiB/KiB)."""
    mem_size = -1
    err_msg = (
        f"`size` {size} is not in a valid format. Use an integer for bytes, or a string with an unit (like '5.0GB')."
    )
    try:
        if isinstance(size, int):
            mem_size = size
        elif size.upper().endswith("GIB"):
            mem_size = int(float(size[:-3]) * (2**30))
        elif size.upper().endswith("MIB"):
            mem_size = int(float(size[:-3]) * (2**20))
        elif size.upper().endswith("KIB"):
            mem_size = int(float(size[:-3]) * (2**10))
        elif size.upper().endswith("GB"):
            int_size = int(float(size[:-2]) * (10**9))
            mem_size = int_size // 8 if size.endswith("b") else int_size
        elif size.upper().endswith("MB"):
            int_size = int(float(size[:-2]) * (10**6))
            mem_size = int_size // 8 if size.endswith("b") else int_size
        elif size.upper().endswith("KB"):
            int_size = int(float(size[:-2]) * (10**3))
            mem_size = int_size // 8 if size.endswith("b") else int_size
    except ValueError:
        raise ValueError(err_msg)
    if mem_size < 0:
        raise ValueError(err_msg)
    return mem_size


def id_tensor_storage(tensor: torch.Tensor):
    return tensor.device, tensor.untyped_storage().data_ptr() if tensor.numel() else id(tensor), tensor.untyped_storage().nbytes()
