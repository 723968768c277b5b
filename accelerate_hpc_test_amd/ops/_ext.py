"""Loader for the in-tree HIP extension `accelerate_hpc_test_amd._C`.

Policy (MI355X-first, no silent fallbacks): ops called on GPU tensors REQUIRE the extension and raise if it
is missing (`use_native(t)` → True → `ext()` raises). The PyTorch reference implementations are used only for
CPU tensors (the CPU plumbing tests) or when `ACCELERATE_NATIVE_KERNELS=0` is set explicitly for debugging.
"""

from __future__ import annotations

import importlib
import os

import torch

_EXT = None
_ERR = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return _EXT
    # ACCELERATE_DEBUG_KERNELS=1: the debug build with device-side bounds checks (`_C_debug`); failed
    # checks are read with `ext().debug_status()` (id << 32 | kernel source line)
    name = "_C_debug" if os.environ.get("ACCELERATE_DEBUG_KERNELS", "0") == "1" else "_C"
    try:
        _EXT = importlib.import_module(f"accelerate_hpc_test_amd.{name}")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e
    return _EXT


def available() -> bool:
    return _load() is not None


def ext():
    mod = _load()
    if mod is None:
        raise RuntimeError(
            "accelerate_hpc_test_amd native extension (_C / _C_debug) is not built or failed to load: "
            f"{_ERR!r}. Build it with `PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace`."
        )
    return mod


def native_enabled() -> bool:
    return os.environ.get("ACCELERATE_NATIVE_KERNELS", "1") != "0"


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on a GPU and native kernels are enabled (then the extension is mandatory)."""
    return t.is_cuda and native_enabled()
