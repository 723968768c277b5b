"""Forward hooks used by big-model inference (device alignment, CPU/disk offload, layerwise casting).

Parity: `/root/reference/src/accelerate/hooks.py:43-783` — `ModelHook`, `SequentialHook`, `add_hook_to_module`,
`remove_hook_from_module`, `AlignDevicesHook`, `attach_execution_device_hook`, `attach_align_device_hook`,
`attach_align_device_hook_on_blocks`, `CpuOffload`, `UserCpuOffloadHook`, `LayerwiseCastingHook`.

MI355X-native addition — **asynchronous offload prefetch** (`OffloadPrefetcher`). The reference uploads every
offloaded module's weights synchronously right before it runs (it notes "need to implement prefetching",
`benchmarks/big_model_inference/README.md:42-44`). Here the offloaded hooks sharing an execution device record their
execution order on the first forward; afterwards, while module i computes, module i+1's weights are copied from
pinned host memory to HBM on a dedicated high-priority copy stream (one HIP event per module), so PCIe transfers
overlap compute. Disabled with `ACCELERATE_OFFLOAD_PREFETCH=0`.
"""

from __future__ import annotations

import functools
import os
from collections.abc import Mapping
from typing import Optional, Union

import torch
import torch.nn as nn

from .utils.memory import clear_device_cache
from .utils.modeling import named_module_tensors
from .utils.offload import PrefixedDataset
from .utils.operations import find_device, send_to_device


class ModelHook:
    """Base hook: `init_hook` at attach time, `pre_forward`/`post_forward` around the module's forward,
    `detach_hook` at removal. `no_grad` runs the wrapped forward without autograd."""

    no_grad = False

    def init_hook(self, module):
        return module

    def pre_forward(self, module, *args, **kwargs):
        return args, kwargs

    def post_forward(self, module, output):
        return output

    def detach_hook(self, module):
        return module


class SequentialHook(ModelHook):
    def __init__(self, *hooks):
        self.hooks = hooks

    def init_hook(self, module):
        for hook in self.hooks:
            module = hook.init_hook(module)
        return module

    def pre_forward(self, module, *args, **kwargs):
        for hook in self.hooks:
            args, kwargs = hook.pre_forward(module, *args, **kwargs)
        return args, kwargs

    def post_forward(self, module, output):
        for hook in self.hooks:
            output = hook.post_forward(module, output)
        return output

    def detach_hook(self, module):
        for hook in self.hooks:
            module = hook.detach_hook(module)
        return module


def add_hook_to_module(module: nn.Module, hook: ModelHook, append: bool = False):
    """Wrap `module.forward` with `hook` (stored as `module._hf_hook`; `append` chains after an existing hook)."""
    if append and (getattr(module, "_hf_hook", None) is not None):
        old_hook = module._hf_hook
        remove_hook_from_module(module)
        hook = SequentialHook(old_hook, hook)
    if hasattr(module, "_hf_hook") and hasattr(module, "_old_forward"):
        old_forward = module._old_forward
    else:
        old_forward = module.forward
        module._old_forward = old_forward
    module = hook.init_hook(module)
    module._hf_hook = hook

    def new_forward(module, *args, **kwargs):
        args, kwargs = module._hf_hook.pre_forward(module, *args, **kwargs)
        if module._hf_hook.no_grad:
            with torch.no_grad():
                output = module._old_forward(*args, **kwargs)
        else:
            output = module._old_forward(*args, **kwargs)
        return module._hf_hook.post_forward(module, output)

    if "GraphModuleImpl" in str(type(module)):
        module.__class__.forward = functools.update_wrapper(functools.partial(new_forward, module), old_forward)
    else:
        module.forward = functools.update_wrapper(functools.partial(new_forward, module), old_forward)
    return module


def remove_hook_from_module(module: nn.Module, recurse: bool = False):
    if hasattr(module, "_hf_hook"):
        module._hf_hook.detach_hook(module)
        delattr(module, "_hf_hook")
    if hasattr(module, "_old_forward"):
        if "GraphModuleImpl" in str(type(module)):
            module.__class__.forward = module._old_forward
        else:
            module.forward = module._old_forward
        delattr(module, "_old_forward")
    for attr in ("_accelerate_added_attributes",):
        for a in getattr(module, attr, []):
            if hasattr(module, a):
                delattr(module, a)
        if hasattr(module, attr):
            delattr(module, attr)
    if recurse:
        for child in module.children():
            remove_hook_from_module(child, recurse)
    return module


def _set_tensor(module: nn.Module, name: str, value: torch.Tensor):
    """Install `value` as parameter/buffer `name` (dotted path allowed) without copying."""
    if "." in name:
        sub, name = name.rsplit(".", 1)
        module = module.get_submodule(sub)
    if name in module._parameters:
        old = module._parameters[name]
        if value.device.type == "meta" or not isinstance(value, nn.Parameter):
            value = nn.Parameter(value, requires_grad=old.requires_grad if old is not None else False)
        module._parameters[name] = value
    else:
        module._buffers[name] = value


class OffloadPrefetcher:
    """Per-device scheduler of offloaded-weight uploads (see module docstring)."""

    _instances: dict = {}

    def __init__(self, device: torch.device):
        self.device = device
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self.order: list = []
        self.recording = True
        self.staged: dict[int, tuple[dict, torch.cuda.Event]] = {}

    @classmethod
    def get(cls, device) -> Optional["OffloadPrefetcher"]:
        device = torch.device(device)
        if device.type != "cuda" or os.environ.get("ACCELERATE_OFFLOAD_PREFETCH", "1") == "0":
            return None
        key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
        if key not in cls._instances:
            cls._instances[key] = OffloadPrefetcher(torch.device("cuda", key[1]))
        return cls._instances[key]

    def note_execution(self, hook):
        if self.recording:
            if hook in self.order:
                self.recording = False  # one full pass recorded
            else:
                self.order.append(hook)

    def take(self, hook):
        item = self.staged.pop(id(hook), None)
        if item is None:
            return None
        tensors, event = item
        torch.cuda.current_stream(self.device).wait_event(event)
        cur = torch.cuda.current_stream(self.device)
        for t in tensors.values():
            t.record_stream(cur)
        return tensors

    def prefetch_after(self, hook):
        if self.recording or hook not in self.order:
            return
        i = self.order.index(hook)
        nxt = self.order[(i + 1) % len(self.order)]
        if id(nxt) in self.staged:
            return
        tensors = {}
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            for name, host in nxt.host_tensors().items():
                tensors[name] = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.staged[id(nxt)] = (tensors, ev)


class AlignDevicesHook(ModelHook):
    """Put a module's weights (from `weights_map` when offloaded) and inputs on `execution_device` for its forward;
    optionally move outputs back to the input device (`io_same_device`) and re-offload weights after the forward."""

    def __init__(
        self,
        execution_device: Optional[Union[int, str, torch.device]] = None,
        offload: bool = False,
        io_same_device: bool = False,
        weights_map: Optional[Mapping] = None,
        offload_buffers: bool = False,
        place_submodules: bool = False,
        skip_keys: Optional[Union[str, list[str]]] = None,
        tied_params_map: Optional[dict[int, dict[torch.device, torch.Tensor]]] = None,
    ):
        self.execution_device = execution_device
        self.offload = offload
        self.io_same_device = io_same_device
        self.weights_map = weights_map
        self.offload_buffers = offload_buffers
        self.place_submodules = place_submodules
        self.skip_keys = skip_keys
        self.input_device = None
        self.param_original_devices = {}
        self.buffer_original_devices = {}
        self.tied_params_names = set()
        self.tied_params_map = tied_params_map
        self._pinned = None
        self._names = None

    def __repr__(self):
        return (
            f"AlignDevicesHook(execution_device={self.execution_device}, offload={self.offload}, "
            f"io_same_device={self.io_same_device}, offload_buffers={self.offload_buffers}, "
            f"place_submodules={self.place_submodules}, skip_keys={repr(self.skip_keys)})"
        )

    def init_hook(self, module):
        if self.execution_device == "meta" or self.execution_device == torch.device("meta"):
            self.tied_params_map = None
        if not self.offload and self.execution_device is not None:
            for name, _ in named_module_tensors(module, recurse=self.place_submodules):
                set_module_tensor_to_device(module, name, self.execution_device, tied_params_map=self.tied_params_map)
        elif self.offload:
            self.original_devices = {
                name: param.device for name, param in named_module_tensors(module, recurse=self.place_submodules)
            }
            if self.weights_map is None:
                self.weights_map = {
                    name: param.to("cpu")
                    for name, param in named_module_tensors(module, include_buffers=self.offload_buffers, recurse=self.place_submodules)
                }
            for name, _ in named_module_tensors(module, include_buffers=self.offload_buffers, recurse=self.place_submodules, remove_non_persistent=True):
                if (
                    self.tied_params_map is not None
                    and recursive_getattr(module, name).data_ptr() in self.tied_params_map
                ):
                    self.tied_params_names.add(name)
                set_module_tensor_to_device(module, name, "meta")
            if not self.offload_buffers and self.execution_device is not None:
                for name, _ in module.named_buffers(recurse=self.place_submodules):
                    set_module_tensor_to_device(module, name, self.execution_device, tied_params_map=self.tied_params_map)
            elif self.offload_buffers and self.execution_device is not None:
                for name in get_non_persistent_buffers(module, recurse=self.place_submodules):
                    set_module_tensor_to_device(module, name, self.execution_device, tied_params_map=self.tied_params_map)
        return module

    # --- async prefetch support ------------------------------------------------------------------------
    def _offload_names(self, module=None):
        if self._names is None and module is not None:
            self._names = [
                name
                for name, _ in named_module_tensors(module, include_buffers=self.offload_buffers, recurse=self.place_submodules, remove_non_persistent=True)
            ]
        return self._names or []

    def host_tensors(self) -> dict:
        """Pinned host copies of this module's offloaded weights (built once)."""
        if self._pinned is None:
            pinned = {}
            for name in self._names or []:
                if name in self.tied_params_names:
                    continue
                v = self.weights_map[name]
                if v.device.type == "cpu":
                    try:
                        v = v.contiguous().pin_memory()
                    except RuntimeError:
                        pass
                pinned[name] = v
            self._pinned = pinned
        return self._pinned

    def pre_forward(self, module, *args, **kwargs):
        if self.io_same_device:
            self.input_device = find_device([args, kwargs])
        if self.offload:
            self.tied_pointers_to_remove = set()
            names = self._offload_names(module)
            pf = OffloadPrefetcher.get(self.execution_device) if self.execution_device is not None else None
            staged = None
            if pf is not None:
                pf.note_execution(self)
                staged = pf.take(self)
            for name in names:
                if staged is not None and name in staged:
                    _set_tensor(module, name, staged[name])
                    continue
                value = self.weights_map[name]
                if name in self.tied_params_names and value.data_ptr() not in self.tied_params_map:
                    self.tied_params_map[value.data_ptr()] = {}
                if (
                    value is not None
                    and self.tied_params_map is not None
                    and value.data_ptr() in self.tied_params_map
                    and self.execution_device not in self.tied_params_map[value.data_ptr()]
                ):
                    self.tied_pointers_to_remove.add((value.data_ptr(), self.execution_device))
                set_module_tensor_to_device(module, name, self.execution_device, value=value, tied_params_map=self.tied_params_map)
            if pf is not None:
                pf.prefetch_after(self)
        return send_to_device(args, self.execution_device), send_to_device(kwargs, self.execution_device, skip_keys=self.skip_keys)

    def post_forward(self, module, output):
        if self.offload:
            for name in self._offload_names(module):
                set_module_tensor_to_device(module, name, "meta")
            for value_pointer, device in getattr(self, "tied_pointers_to_remove", set()):
                if isinstance(device, int):
                    device = f"cuda:{device}"
                if value_pointer in self.tied_params_map and device in self.tied_params_map[value_pointer]:
                    del self.tied_params_map[value_pointer][device]
            self.tied_pointers_to_remove = set()
        if self.io_same_device and self.input_device is not None:
            output = send_to_device(output, self.input_device, skip_keys=self.skip_keys)
        return output

    def detach_hook(self, module):
        if self.offload:
            for name, device in self.original_devices.items():
                if device != torch.device("meta"):
                    set_module_tensor_to_device(module, name, device, value=self.weights_map.get(name, None))
        return module


def attach_execution_device_hook(module, execution_device, skip_keys=None, preload_module_classes=None, tied_params_map=None):
    if not hasattr(module, "_hf_hook") and len(module.state_dict()) > 0:
        add_hook_to_module(module, AlignDevicesHook(execution_device, skip_keys=skip_keys, tied_params_map=tied_params_map))
    if preload_module_classes is not None and module.__class__.__name__ in preload_module_classes:
        return
    for child in module.children():
        attach_execution_device_hook(child, execution_device, skip_keys=skip_keys, tied_params_map=tied_params_map)


def attach_align_device_hook(
    module,
    execution_device=None,
    offload=False,
    weights_map=None,
    offload_buffers=False,
    module_name="",
    skip_keys=None,
    preload_module_classes=None,
    tied_params_map=None,
):
    directs = named_module_tensors(module)
    full_offload = offload and preload_module_classes is not None and module.__class__.__name__ in preload_module_classes
    if len(list(directs)) > 0 or full_offload:
        if weights_map is not None:
            prefix = f"{module_name}." if len(module_name) > 0 else ""
            prefixed_weights_map = PrefixedDataset(weights_map, prefix)
        else:
            prefixed_weights_map = None
        hook = AlignDevicesHook(
            execution_device=execution_device,
            offload=offload,
            weights_map=prefixed_weights_map,
            offload_buffers=offload_buffers,
            place_submodules=full_offload,
            skip_keys=skip_keys,
            tied_params_map=tied_params_map,
        )
        add_hook_to_module(module, hook, append=True)
    if full_offload:
        return
    for child_name, child in module.named_children():
        child_name = f"{module_name}.{child_name}" if len(module_name) > 0 else child_name
        attach_align_device_hook(
            child,
            execution_device=execution_device,
            offload=offload,
            weights_map=weights_map,
            offload_buffers=offload_buffers,
            module_name=child_name,
            preload_module_classes=preload_module_classes,
            skip_keys=skip_keys,
            tied_params_map=tied_params_map,
        )


def remove_hook_from_submodules(module):
    remove_hook_from_module(module)
    for child in module.children():
        remove_hook_from_submodules(child)


def attach_align_device_hook_on_blocks(
    module,
    execution_device=None,
    offload=False,
    weights_map=None,
    offload_buffers=False,
    module_name="",
    skip_keys=None,
    preload_module_classes=None,
    tied_params_map=None,
):
    if not isinstance(execution_device, Mapping) and not isinstance(offload, dict):
        if not offload:
            hook = AlignDevicesHook(execution_device=execution_device, io_same_device=True, skip_keys=skip_keys, place_submodules=True, tied_params_map=tied_params_map)
            add_hook_to_module(module, hook)
        else:
            attach_align_device_hook(
                module,
                execution_device=execution_device,
                offload=True,
                weights_map=weights_map,
                offload_buffers=offload_buffers,
                module_name=module_name,
                skip_keys=skip_keys,
                tied_params_map=tied_params_map,
            )
        return
    if not isinstance(execution_device, Mapping):
        execution_device = {key: execution_device for key in offload.keys()}
    if not isinstance(offload, Mapping):
        offload = {key: offload for key in execution_device.keys()}
    if module_name in execution_device and module_name in offload and not offload[module_name]:
        hook = AlignDevicesHook(
            execution_device=execution_device[module_name],
            offload_buffers=offload_buffers,
            io_same_device=(module_name == ""),
            place_submodules=True,
            skip_keys=skip_keys,
            tied_params_map=tied_params_map,
        )
        add_hook_to_module(module, hook)
        attach_execution_device_hook(module, execution_device[module_name], skip_keys=skip_keys, tied_params_map=tied_params_map)
    elif module_name in execution_device and module_name in offload:
        attach_align_device_hook(
            module,
            execution_device=execution_device[module_name],
            offload=True,
            weights_map=weights_map,
            offload_buffers=offload_buffers,
            module_name=module_name,
            skip_keys=skip_keys,
            preload_module_classes=preload_module_classes,
            tied_params_map=tied_params_map,
        )
        if not hasattr(module, "_hf_hook"):
            hook = AlignDevicesHook(
                execution_device=execution_device[module_name],
                io_same_device=(module_name == ""),
                skip_keys=skip_keys,
                tied_params_map=tied_params_map,
            )
            add_hook_to_module(module, hook)
        attach_execution_device_hook(
            module,
            execution_device[module_name],
            preload_module_classes=preload_module_classes,
            skip_keys=skip_keys,
            tied_params_map=tied_params_map,
        )
    elif module_name == "":
        hook = AlignDevicesHook(execution_device=execution_device.get(""), io_same_device=True, skip_keys=skip_keys, tied_params_map=tied_params_map)
        add_hook_to_module(module, hook)
    for child_name, child in module.named_children():
        child_name = f"{module_name}.{child_name}" if len(module_name) > 0 else child_name
        attach_align_device_hook_on_blocks(
            child,
            execution_device=execution_device,
            offload=offload,
            weights_map=weights_map,
            offload_buffers=offload_buffers,
            module_name=child_name,
            preload_module_classes=preload_module_classes,
            skip_keys=skip_keys,
            tied_params_map=tied_params_map,
        )


class CpuOffload(ModelHook):
    """Keep the whole module on CPU, move it to `execution_device` for each forward (and offload the previous
    module in a chain: `cpu_offload_with_hook`)."""

    def __init__(self, execution_device=None, prev_module_hook: Optional["UserCpuOffloadHook"] = None):
        self.prev_module_hook = prev_module_hook
        self.execution_device = execution_device if execution_device is not None else _default_device()

    def init_hook(self, module):
        return module.to("cpu")

    def pre_forward(self, module, *args, **kwargs):
        if self.prev_module_hook is not None:
            self.prev_module_hook.offload()
            clear_device_cache()
        module.to(self.execution_device)
        return send_to_device(args, self.execution_device), send_to_device(kwargs, self.execution_device)


class UserCpuOffloadHook:
    def __init__(self, model, hook):
        self.model = model
        self.hook = hook

    def offload(self):
        self.hook.init_hook(self.model)

    def remove(self):
        remove_hook_from_module(self.model)


class LayerwiseCastingHook(ModelHook):
    """Store weights in `storage_dtype` (e.g. fp8), cast to `compute_dtype` around each forward."""

    _is_stateful = False

    def __init__(self, storage_dtype: torch.dtype, compute_dtype: torch.dtype, non_blocking: bool):
        self.storage_dtype = storage_dtype
        self.compute_dtype = compute_dtype
        self.non_blocking = non_blocking

    def init_hook(self, module):
        module.to(dtype=self.storage_dtype, non_blocking=self.non_blocking)
        return module

    def pre_forward(self, module, *args, **kwargs):
        module.to(dtype=self.compute_dtype, non_blocking=self.non_blocking)
        return args, kwargs

    def post_forward(self, module, output):
        module.to(dtype=self.storage_dtype, non_blocking=self.non_blocking)
        return output


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def recursive_getattr(obj, attr):
    import functools as _f

    return _f.reduce(getattr, [obj] + attr.split("."))


def get_non_persistent_buffers(module, recurse=False):
    from .utils.modeling import get_non_persistent_buffers as _g

    return _g(module, recurse=recurse)


def set_module_tensor_to_device(*args, **kwargs):
    from ._big_modeling_impl import set_module_tensor_to_device as _s

    return _s(*args, **kwargs)
