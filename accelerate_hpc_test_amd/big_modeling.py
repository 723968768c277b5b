"""Big-model inference: meta-device init, device-map dispatch, CPU / disk offload.

Parity: `/root/reference/src/accelerate/big_modeling.py:60-790`.
"""

from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.nn as nn


@contextlib.contextmanager
def init_empty_weights(include_buffers: Optional[bool] = None):
    """Create parameters (and optionally buffers) on the meta device: instant construction of huge models."""
    if include_buffers is None:
        import os

        include_buffers = os.environ.get("ACCELERATE_INIT_INCLUDE_BUFFERS", "false").lower() in ("1", "true", "yes")
    with init_on_device(torch.device("meta"), include_buffers=include_buffers) as f:
        yield f


@contextlib.contextmanager
def init_on_device(device: torch.device, include_buffers: Optional[bool] = None):
    """Create every new parameter (and buffer when `include_buffers`) directly on `device`."""
    if include_buffers is None:
        include_buffers = False
    if include_buffers:
        with device:
            yield
        return
    old_register_parameter = nn.Module.register_parameter

    def register_empty_parameter(module, name, param):
        old_register_parameter(module, name, param)
        if param is not None:
            param_cls = type(module._parameters[name])
            kwargs = module._parameters[name].__dict__
            kwargs["requires_grad"] = param.requires_grad
            module._parameters[name] = param_cls(module._parameters[name].to(device), **kwargs)

    try:
        nn.Module.register_parameter = register_empty_parameter
        yield
    finally:
        nn.Module.register_parameter = old_register_parameter


def cpu_offload(*args, **kwargs):
    from ._big_modeling_impl import cpu_offload as f

    return f(*args, **kwargs)


def cpu_offload_with_hook(*args, **kwargs):
    from ._big_modeling_impl import cpu_offload_with_hook as f

    return f(*args, **kwargs)


def disk_offload(*args, **kwargs):
    from ._big_modeling_impl import disk_offload as f

    return f(*args, **kwargs)


def dispatch_model(*args, **kwargs):
    from ._big_modeling_impl import dispatch_model as f

    return f(*args, **kwargs)


def load_checkpoint_and_dispatch(*args, **kwargs):
    from ._big_modeling_impl import load_checkpoint_and_dispatch as f

    return f(*args, **kwargs)
