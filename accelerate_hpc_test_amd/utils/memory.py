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


class _BatchSizeSearch:
    """Calls `fn(batch_size, *args, **kwargs)`, shrinking the batch size after every out-of-memory failure
    (`reduce` gives the next size; default: 90 % of the current one) until a call succeeds."""

    def __init__(self, fn, start: int, reduce=None):
        self.fn = fn
        self.batch_size = start
        self.reduce = reduce if reduce is not None else (lambda: int(self.batch_size * 0.9))
        functools.update_wrapper(self, fn)

    def _check_call(self, args):
        names = list(inspect.signature(self.fn).parameters)
        if len(names) < len(args) + 1:  # the caller passed the batch size itself
            shown = ", ".join(f"{n}={v}" for n, v in zip(names[1:], args[1:]))
            raise TypeError(
                f"Batch size was passed into `{self.fn.__name__}` as the first argument when called."
                f"Remove this as the decorator already does so: `{self.fn.__name__}({shown})`"
            )

    def __call__(self, *args, **kwargs):
        clear_device_cache(garbage_collection=True)
        self._check_call(args)
        while self.batch_size != 0:
            try:
                return self.fn(self.batch_size, *args, **kwargs)
            except Exception as exc:  # noqa: BLE001 - only OOMs are retried, the rest re-raised
                if not should_reduce_batch_size(exc):
                    raise
                clear_device_cache(garbage_collection=True)
                self.batch_size = self.reduce()
        raise RuntimeError("No executable batch size found, reached zero.")


def find_executable_batch_size(function=None, starting_batch_size: int = 128, reduce_batch_size_fn=None):
    """Decorator: run `function(batch_size, ...)` and retry with a smaller batch size after each out-of-memory error
    (HIP: "HIP out of memory." / hipErrorOutOfMemory), starting from `starting_batch_size`."""
    if function is None:
        return functools.partial(find_executable_batch_size, starting_batch_size=starting_batch_size,
                                 reduce_batch_size_fn=reduce_batch_size_fn)
    return _BatchSizeSearch(function, starting_batch_size, reduce_batch_size_fn)


def get_xpu_available_memory(device_index: int):  # pragma: no cover - API parity
    raise NotImplementedError("XPU is not supported on MI355X builds.")
