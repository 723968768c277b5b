"""Memory helpers: cache clearing, release and OOM-retry batch-size search.

Parity: `/root/reference/src/accelerate/utils/memory.py:39-180`. On ROCm the HIP caching allocator is reached
through `torch.cuda.*`; HIP's OOM message ("HIP out of memory") is matched explicitly.
"""

from __future__ import annotations

import functools
import gc
import inspect
import warnings

import torch


def clear_device_cache(garbage_collection: bool = False):
    if garbage_collection:
        gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def release_memory(*objects):
    """Drop references to `objects` (returns a list of Nones to rebind) and empty the device cache."""
    if not isinstance(objects, list):
        objects = list(objects)
    for i in range(len(objects)):
        if hasattr(objects[i], "_hf_hook"):
            from ..hooks import remove_hook_from_module

            remove_hook_from_module(objects[i], recurse=True)
        objects[i] = None
    clear_device_cache(garbage_collection=True)
    return objects


def should_reduce_batch_size(exception: Exception) -> bool:
    _statements = [
        " out of memory.",  # CUDA / HIP OOM ("HIP out of memory.")
        "cuDNN error: CUDNN_STATUS_NOT_SUPPORTED.",
        "DefaultCPUAllocator: can't allocate memory",
        "FATAL ERROR :: MODULE:PT_DEVMEM Allocation failed",
        "hipErrorOutOfMemory",
    ]
    if isinstance(exception, RuntimeError) and len(exception.args) == 1:
        return any(err in exception.args[0] for err in _statements)
    return False


def find_executable_batch_size(function=None, starting_batch_size: int = 128, reduce_batch_size_fn=None):
    """Decorator: call `function(batch_size, ...)`, retrying with 90 % of the batch size after each OOM."""
    if function is None:
        return functools.partial(
            find_executable_batch_size, starting_batch_size=starting_batch_size, reduce_batch_size_fn=reduce_batch_size_fn
        )
    batch_size = starting_batch_size
    if reduce_batch_size_fn is None:

        def reduce_batch_size_fn():
            nonlocal batch_size
            batch_size = int(batch_size * 0.9)
            return batch_size

    def decorator(*args, **kwargs):
        nonlocal batch_size
        clear_device_cache(garbage_collection=True)
        params = list(inspect.signature(function).parameters.keys())
        if len(params) < (len(args) + 1):
            arg_str = ", ".join([f"{arg}={value}" for arg, value in zip(params[1:], args[1:])])
            raise TypeError(
                f"Batch size was passed into `{function.__name__}` as the first argument when called."
                f"Remove this as the decorator already does so: `{function.__name__}({arg_str})`"
            )
        while True:
            if batch_size == 0:
                raise RuntimeError("No executable batch size found, reached zero.")
            try:
                return function(batch_size, *args, **kwargs)
            except Exception as e:
                if should_reduce_batch_size(e):
                    clear_device_cache(garbage_collection=True)
                    batch_size = reduce_batch_size_fn()
                else:
                    raise

    return decorator


def get_xpu_available_memory(device_index: int):  # pragma: no cover - API parity
    raise NotImplementedError("XPU is not supported on MI355X builds.")
