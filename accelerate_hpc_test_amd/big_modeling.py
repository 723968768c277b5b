"""Big-model inference: build models without memory (meta device), place their blocks over GPUs / host / disk
according to a device map, and run them with weights streamed in.

API parity with `/root/reference/src/accelerate/big_modeling.py:60-790` (`init_empty_weights`, `init_on_device`,
`cpu_offload`, `cpu_offload_with_hook`, `disk_offload`, `dispatch_model`, `load_checkpoint_and_dispatch`,
`attach_layerwise_casting_hooks`). The pieces underneath are this package's own:

* `utils/device_map.py` plans the placement (pinned to upstream results by `tests/test_device_map_parity.py`);
* `utils/checkpoint_io.py` streams checkpoints tensor by tensor, GPU-bound tensors through the native H2D engine;
* `hooks.py` runs each block with its weights on the execution device, offloaded blocks fed by one
  `OffloadScheduler` per dispatched model and GPU that prefetches the next block's weights on its own HIP stream.

A "naive pipeline" (blocks on different MI355X GPUs) hands activations between GPUs with device-to-device copies
over xGMI (the hooks' `send_to_device`).
"""

from __future__ import annotations

import contextlib
import functools
import logging
import os
import re
from typing import Optional, Union

import torch
import torch.nn as nn

from .hooks import (
    AlignDevicesHook,
    CpuOffload,
    LayerwiseCastingHook,
    UserCpuOffloadHook,
    add_hook_to_module,
    attach_align_device_hook,
    attach_align_device_hook_on_blocks,
)
from .utils.checkpoint_io import load_checkpoint_in_model
from .utils.device_map import check_device_map, find_tied_parameters, get_balanced_memory, infer_auto_device_map
from .utils.offload import OffloadedWeightsLoader, extract_submodules_state_dict, offload_state_dict
from .utils.placement import recursive_getattr, retie_parameters

logger = logging.getLogger(__name__)

_HOST = ("cpu", "disk")


# ------------------------------------------------------------------------------------------------ construction
@contextlib.contextmanager
def init_empty_weights(include_buffers: Optional[bool] = None):
    """Build modules with parameters (and, with `include_buffers`, buffers) on the meta device: no memory, instant
    construction of 70B-class models before a device map is applied."""
    if include_buffers is None:
        include_buffers = os.environ.get("ACCELERATE_INIT_INCLUDE_BUFFERS", "false").lower() in ("1", "true", "yes")
    with init_on_device(torch.device("meta"), include_buffers=include_buffers) as f:
        yield f


@contextlib.contextmanager
def init_on_device(device: torch.device, include_buffers: Optional[bool] = None):
    """Create every new parameter (and buffer when `include_buffers`) directly on `device`."""
    if include_buffers:
        with device:
            yield
        return
    original = nn.Module.register_parameter

    def register_on_device(module, name, param):
        original(module, name, param)
        if param is not None:
            p = module._parameters[name]
            extra = dict(p.__dict__)
            extra["requires_grad"] = param.requires_grad
            module._parameters[name] = type(p)(p.to(device), **extra)

    nn.Module.register_parameter = register_on_device
    try:
        yield
    finally:
        nn.Module.register_parameter = original


# ------------------------------------------------------------------------------------------------ offload helpers
def _first_param_device(model):
    return next(iter(model.parameters())).device


def cpu_offload(model: nn.Module, execution_device=None, offload_buffers: bool = False, state_dict=None,
                preload_module_classes=None):
    """Keep every weight on the host; each module's weights are uploaded to `execution_device` for its own forward
    (prefetched one module ahead on MI355X)."""
    execution_device = execution_device if execution_device is not None else _first_param_device(model)
    if state_dict is None:
        state_dict = {n: t.to("cpu") for n, t in model.state_dict().items()}
    add_hook_to_module(model, AlignDevicesHook(io_same_device=True), append=True)
    attach_align_device_hook(model, execution_device=execution_device, offload=True, offload_buffers=offload_buffers,
                             weights_map=state_dict, preload_module_classes=preload_module_classes, schedulers={})
    return model


def cpu_offload_with_hook(model: nn.Module, execution_device=None, prev_module_hook: Optional[UserCpuOffloadHook] = None):
    """Move the whole model to the device for its forward and keep it there until `hook.offload()` (pipelines of
    several models run one after another)."""
    hook = CpuOffload(execution_device=execution_device, prev_module_hook=prev_module_hook)
    add_hook_to_module(model, hook, append=True)
    return model, UserCpuOffloadHook(model, hook)


def disk_offload(model: nn.Module, offload_dir, execution_device=None, offload_buffers: bool = False,
                 preload_module_classes=None):
    """Write every weight to `offload_dir` (unless an index is already there) and read it back per forward."""
    if not (os.path.isdir(offload_dir) and os.path.isfile(os.path.join(offload_dir, "index.json"))):
        offload_state_dict(offload_dir, model.state_dict())
    execution_device = execution_device if execution_device is not None else _first_param_device(model)
    add_hook_to_module(model, AlignDevicesHook(io_same_device=True), append=True)
    attach_align_device_hook(model, execution_device=execution_device, offload=True, offload_buffers=offload_buffers,
                             weights_map=OffloadedWeightsLoader(save_folder=offload_dir),
                             preload_module_classes=preload_module_classes, schedulers={}, cache_host=False)
    return model


# ------------------------------------------------------------------------------------------------ dispatch
def _guard_moves(model: nn.Module):
    """`model.to()` / `.cuda()` on a dispatched model: warn, and refuse when weights are offloaded (meta)."""

    def guard(fn):
        @functools.wraps(fn)
        def wrapped(*args, **kwargs):
            moving = fn.__name__ != "to" or torch._C._nn._parse_to(*args, **kwargs)[0] is not None
            if moving:
                logger.warning("You shouldn't move a model that is dispatched using accelerate hooks.")
            if any(p.device.type == "meta" for p in model.parameters()):
                raise RuntimeError("You can't move a model that has some modules offloaded to cpu or disk.")
            return fn(*args, **kwargs)

        return wrapped

    model.to = guard(model.to)
    model.cuda = guard(model.cuda)


def dispatch_model(
    model: nn.Module,
    device_map: dict,
    main_device: Optional[Union[str, torch.device]] = None,
    state_dict: Optional[dict] = None,
    offload_dir: Optional[Union[str, os.PathLike]] = None,
    offload_index: Optional[dict] = None,
    offload_buffers: bool = False,
    skip_keys: Optional[Union[str, list]] = None,
    preload_module_classes: Optional[list] = None,
    force_hooks: bool = False,
):
    """Place the blocks of `model` per `device_map` and hook them so a forward runs across them: GPU blocks run
    where they sit, host / disk blocks are streamed to `main_device` (default: the first GPU of the map)."""
    check_device_map(model, device_map)
    targets = set(device_map.values())
    if len(targets) == 1 and not force_hooks:
        only = next(iter(targets))
        if only == "disk":
            raise ValueError("You are trying to offload the whole model to the disk. Please use the `disk_offload` function instead.")
        model.to(only)
        model.hf_device_map = dict(device_map)
        return model

    if main_device is None:  # the first GPU in map order; the host when the map names no GPU
        main_device = next((d for d in device_map.values() if d not in _HOST), "cpu")
    host_blocks = [n for n, d in device_map.items() if d == "cpu"]
    disk_blocks = [n for n, d in device_map.items() if d == "disk"]
    if main_device != "cpu" and state_dict is None and host_blocks:
        state_dict = extract_submodules_state_dict(model.state_dict(), host_blocks)
    if disk_blocks and offload_dir is None and offload_index is None:
        raise ValueError(
            "We need an `offload_dir` to dispatch this model according to this `device_map`, the following submodules "
            f"need to be offloaded: {', '.join(disk_blocks)}."
        )
    if disk_blocks and offload_index is None and not (os.path.isdir(offload_dir) and os.path.isfile(os.path.join(offload_dir, "index.json"))):
        offload_state_dict(offload_dir, extract_submodules_state_dict(model.state_dict(), disk_blocks))

    streamed_from = ("disk",) if main_device in ("cpu", "mps") else _HOST
    execution_device = {n: (main_device if d in _HOST else d) for n, d in device_map.items()}
    execution_device[""] = main_device
    offload = {n: d in streamed_from for n, d in device_map.items()}
    folder = offload_dir if disk_blocks else None
    weights_map = None
    if state_dict is not None or folder is not None or offload_index is not None:
        weights_map = OffloadedWeightsLoader(state_dict=state_dict, save_folder=folder, index=offload_index,
                                             device=main_device if offload_index is not None else None)

    tied = find_tied_parameters(model)
    tied_params_map = {recursive_getattr(model, name).data_ptr(): {} for group in tied for name in group}
    attach_align_device_hook_on_blocks(
        model, execution_device=execution_device, offload=offload, offload_buffers=offload_buffers,
        weights_map=weights_map, skip_keys=skip_keys, preload_module_classes=preload_module_classes,
        tied_params_map=tied_params_map, schedulers={},
        cache_host={n: d == "cpu" for n, d in device_map.items()},  # keep pinned copies of host blocks, not disk ones
    )
    spilled = sorted(d for d in targets if d in _HOST)
    if spilled:
        logger.warning(f"Some parameters are on the meta device because they were offloaded to the {' and '.join(spilled)}.")
    retie_parameters(model, tied)
    _guard_moves(model)
    model.hf_device_map = dict(device_map)
    return model


def load_checkpoint_and_dispatch(
    model: nn.Module,
    checkpoint,
    device_map=None,
    max_memory=None,
    no_split_module_classes=None,
    offload_folder=None,
    offload_buffers: bool = False,
    dtype=None,
    offload_state_dict=None,
    skip_keys=None,
    preload_module_classes=None,
    force_hooks: bool = False,
    strict: bool = False,
    full_state_dict: bool = True,
    broadcast_from_rank0: bool = False,
):
    """Load a checkpoint into a (meta-initialised) model and dispatch it. `device_map` may be a dict or one of
    "auto" / "balanced" / "balanced_low_0" (budgets from `get_balanced_memory`) / "sequential"."""
    if isinstance(device_map, str) and device_map not in ("auto", "balanced", "balanced_low_0", "sequential"):
        raise ValueError("If passing a string for `device_map`, please choose 'auto', 'balanced', 'balanced_low_0' or 'sequential'.")
    if isinstance(device_map, str):
        if device_map != "sequential":
            max_memory = get_balanced_memory(model, max_memory=max_memory, no_split_module_classes=no_split_module_classes,
                                             dtype=dtype, low_zero=device_map == "balanced_low_0")
        device_map = infer_auto_device_map(model, max_memory=max_memory, no_split_module_classes=no_split_module_classes,
                                           dtype=dtype, offload_buffers=offload_buffers)
    if offload_state_dict is None and device_map is not None and "disk" in device_map.values():
        offload_state_dict = True
    load_checkpoint_in_model(model, checkpoint, device_map=device_map, offload_folder=offload_folder, dtype=dtype,
                             offload_state_dict=bool(offload_state_dict), offload_buffers=offload_buffers, strict=strict,
                             full_state_dict=full_state_dict, broadcast_from_rank0=broadcast_from_rank0)
    if device_map is None:
        return model
    return dispatch_model(model, device_map=device_map, offload_dir=offload_folder, offload_buffers=offload_buffers,
                          skip_keys=skip_keys, preload_module_classes=preload_module_classes, force_hooks=force_hooks)


# ------------------------------------------------------------------------------------------------ layerwise casting
# The layers whose weights are stored low-precision: the reference's SUPPORTED_PYTORCH_LAYERS_FOR_UPCASTING
# (/root/reference/src/accelerate/utils/constants.py:99-107) -- convolutions and Linear only.
_CASTABLE = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose1d, nn.ConvTranspose2d, nn.ConvTranspose3d, nn.Linear)


def attach_layerwise_casting_hooks(module: nn.Module, storage_dtype: torch.dtype, compute_dtype: torch.dtype,
                                   skip_modules_pattern=None, skip_modules_classes=None, non_blocking: bool = False):
    """Store the weights of supported layers (`Conv*`, `ConvTranspose*`, `Linear`) in `storage_dtype` (e.g. fp8 e4m3:
    half the HBM of bf16) and upcast them to `compute_dtype` around each forward (hooks.py `LayerwiseCastingHook`).
    Modules whose qualified name matches a regex of `skip_modules_pattern`, or that are instances of
    `skip_modules_classes`, are left alone together with their subtree; by default nothing is skipped (reference
    big_modeling.py:724-750). A single string pattern is one regex (the reference iterates a bare string character by
    character)."""
    if isinstance(skip_modules_pattern, str):
        skip_modules_pattern = (skip_modules_pattern,)
    patterns = tuple(skip_modules_pattern or ())
    classes = tuple(skip_modules_classes or ())
    stack = [("", module)]
    while stack:
        name, m = stack.pop()
        if (classes and isinstance(m, classes)) or any(re.search(p, name) for p in patterns):
            continue
        if isinstance(m, _CASTABLE):
            add_hook_to_module(m, LayerwiseCastingHook(storage_dtype, compute_dtype, non_blocking), append=True)
            continue
        stack.extend(reversed([(f"{name}.{n}" if name else n, c) for n, c in m.named_children()]))
