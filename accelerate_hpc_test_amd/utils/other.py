"""Misc model utilities: unwrapping, compile helpers, save/load, safetensors cleaning.

Parity: `/root/reference/src/accelerate/utils/other.py:54-516` (`extract_model_from_parallel`, `compile_regions`,
`is_compiled_module`, `save`, `load`, `clean_state_dict_for_safetensors`, `wait_for_everyone`,
`merge_dicts`, `get_pretty_name`, `check_os_kernel`, `recursive_getattr`).
"""

from __future__ import annotations

import collections
import os
import platform
import re
import socket
from copy import deepcopy
from functools import partial
from types import MethodType
from typing import Any, Callable

import torch

from .constants import SAFE_WEIGHTS_NAME, WEIGHTS_NAME


def PartialState():  # noqa: N802 - lazy accessor (avoids the utils <-> state import cycle)
    from ..state import PartialState as _PartialState

    return _PartialState()
from .dataclasses import DistributedType


def is_compiled_module(module: torch.nn.Module) -> bool:
    return hasattr(torch, "_dynamo") and isinstance(module, torch._dynamo.eval_frame.OptimizedModule)


def has_compiled_regions(module: torch.nn.Module) -> bool:
    if not isinstance(module, torch.nn.Module):
        return False
    if module._modules:
        for sub in module.modules():
            if is_compiled_module(sub):
                return True
    return False


def compile_regions(module: torch.nn.Module, **compile_kwargs) -> torch.nn.Module:
    """Regional compilation: compile each block of repeated ModuleLists separately (reference other.py:102-171).
    Available for users who ask for it; the benchmarked path does not use Inductor."""

    def _compile_regions(module, **compile_kwargs):
        if isinstance(module, torch.nn.ModuleList):
            new_module = torch.nn.ModuleList()
            for submodule in module:
                new_module.append(torch.compile(submodule, **compile_kwargs))
            return new_module
        elif module._modules:
            new_module = deepcopy(module) if False else module
            for name, submodule in list(module.named_children()):
                setattr(new_module, name, _compile_regions(submodule, **compile_kwargs))
            return new_module
        return torch.compile(module, **compile_kwargs)

    new_module = _compile_regions(module, **compile_kwargs)
    if "_orig_mod" not in new_module.__dict__:
        new_module.__dict__["_orig_mod"] = module
    return new_module


def compile_regions_deepspeed(module, **compile_kwargs):
    for sub in module.children():
        compile_regions(sub, **compile_kwargs)


def extract_model_from_parallel(model, keep_fp32_wrapper: bool = True, keep_torch_compile: bool = True, recursive: bool = False):
    """Strip our DDP/FSDP wrappers, torch.compile wrappers and (optionally) the mixed-precision forward."""
    from ..parallel.ddp import DistributedDataParallel as NativeDDP
    from ..parallel.fsdp import FullyShardedModule

    options = (NativeDDP, FullyShardedModule, torch.nn.parallel.DistributedDataParallel, torch.nn.DataParallel)
    is_compiled = is_compiled_module(model)
    if is_compiled:
        compiled_model = model
        model = model._orig_mod
    while isinstance(model, options):
        model = model.module
    if recursive:
        def _recursive_unwrap(module):
            if hasattr(module, "module") and isinstance(module, options):
                unwrapped = module.module
            else:
                unwrapped = module
            for name, child in unwrapped.named_children():
                setattr(unwrapped, name, _recursive_unwrap(child))
            return unwrapped

        model = _recursive_unwrap(model)
    if not keep_fp32_wrapper:
        forward = model.forward
        original_forward = model.__dict__.pop("_original_forward", None)
        if original_forward is not None:
            while hasattr(forward, "__wrapped__"):
                forward = forward.__wrapped__
                if forward == original_forward:
                    break
            model.forward = MethodType(forward, model)
    if keep_torch_compile and is_compiled:
        compiled_model._orig_mod = model
        model = compiled_model
    return model


def wait_for_everyone():
    PartialState().wait_for_everyone()


def clean_state_dict_for_safetensors(state_dict: dict):
    """Drop shared-storage duplicates (tied weights) and make tensors contiguous, as safetensors requires."""
    ptrs = collections.defaultdict(list)
    for name, tensor in state_dict.items():
        if not isinstance(tensor, str):
            ptrs[(tensor.device, tensor.untyped_storage().data_ptr() if tensor.numel() else id(tensor))].append(name)
    shared_ptrs = {ptr: names for ptr, names in ptrs.items() if len(names) > 1}
    warn_names = set()
    for names in shared_ptrs.values():
        found_names = [name for name in names if name in state_dict]
        warn_names.update(found_names[1:])
        for name in found_names[1:]:
            del state_dict[name]
    if len(warn_names) > 0:
        from ..logging import get_logger

        get_logger(__name__).warning(
            f"Removed shared tensor {warn_names} while saving. This should be OK, but check by verifying that you don't receive any warning while reloading"
        )
    state_dict = {k: v.contiguous() if isinstance(v, torch.Tensor) else v for k, v in state_dict.items()}
    return state_dict


def save(obj, f, save_on_each_node: bool = False, safe_serialization: bool = False):
    """Save `obj` once per machine (main process) or per node; safetensors when `safe_serialization`."""
    if PartialState().distributed_type == DistributedType.XLA:
        pass
    if safe_serialization:
        from safetensors.torch import save_file

        save_func = partial(save_file, metadata={"format": "pt"})
        if isinstance(obj, collections.OrderedDict):
            obj = dict(obj)
        obj = clean_state_dict_for_safetensors(obj)
    else:
        save_func = torch.save
    if PartialState().is_main_process and not save_on_each_node:
        save_func(obj, f)
    elif PartialState().is_local_main_process and save_on_each_node:
        save_func(obj, f)


class _UnsafeUnpickleWarning:  # sentinel kept for API similarity
    pass


def load(f, map_location=None, **kwargs):
    """`torch.load` defaulting to `weights_only=True` (never executes code from checkpoint files)."""
    kwargs.setdefault("weights_only", True)
    try:
        return torch.load(f, map_location=map_location, **kwargs)
    except Exception:
        if kwargs.get("weights_only", True):
            import numpy as np

            with torch.serialization.safe_globals([np.core.multiarray._reconstruct, np.ndarray, np.dtype, type(np.dtype("uint32"))]):
                return torch.load(f, map_location=map_location, **kwargs)
        raise


def get_pretty_name(obj) -> str:
    """Readable name of a class, function or instance (its class's qualified name), for log and error messages."""
    for cand in (obj, type(obj)):
        name = getattr(cand, "__qualname__", None) or getattr(cand, "__name__", None)
        if name:
            return name
    return str(obj)


def merge_dicts(source: dict, destination: dict) -> dict:
    """Deep-merge `source` into `destination` in place (nested dicts merged key by key, other values replaced) and
    return `destination`."""
    stack = [(source, destination)]
    while stack:
        src, dst = stack.pop()
        for key, value in src.items():
            if isinstance(value, dict):
                stack.append((value, dst.setdefault(key, {})))
            else:
                dst[key] = value
    return destination


def is_port_in_use(port: int = None) -> bool:
    if port is None:
        port = 29500
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        return s.connect_ex(("localhost", port)) == 0


def get_free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_BYTE_UNITS = ("bytes", "KB", "MB", "GB", "TB", "PB")


def convert_bytes(size) -> str:
    """`size` bytes in the largest binary unit that keeps the value under 1024 (two decimals)."""
    value, unit = size, 0
    while value >= 1024.0 and unit < len(_BYTE_UNITS) - 1:
        value /= 1024.0
        unit += 1
    return f"{round(value, 2)} {_BYTE_UNITS[unit]}"


_MIN_LINUX_KERNEL = (5, 5, 0)


def check_os_kernel():
    """Multi-process jobs are known to hang on Linux kernels older than 5.5: log a warning on such a host."""
    info = platform.uname()
    if info.system != "Linux":
        return
    found = re.search(r"(\d+)\.(\d+)\.(\d+)", info.release)
    if found is None:
        return
    release = tuple(int(x) for x in found.groups())
    if release < _MIN_LINUX_KERNEL:
        from ..logging import get_logger

        have, need = ".".join(map(str, release)), ".".join(map(str, _MIN_LINUX_KERNEL))
        get_logger(__name__).warning(
            f"Linux kernel {have} is older than {need}: multi-process runs can hang on it; upgrade the host kernel.")


def recursive_getattr(obj, attr: str):
    def _getattr(obj, attr):
        return getattr(obj, attr)

    import functools

    return functools.reduce(_getattr, [obj] + attr.split("."))


def get_module_children_bottom_up(model: torch.nn.Module, return_fqns: bool = False):
    top = model if not return_fqns else ("", model)
    stack = [top]
    ordered = []
    while stack:
        current = stack.pop()
        ordered.append(current)
        mod = current if not return_fqns else current[1]
        for name, child in mod.named_children():
            if return_fqns:
                stack.append((f"{current[0]}.{name}" if current[0] else name, child))
            else:
                stack.append(child)
    return ordered[::-1]
