"""Forward hooks for big-model inference: run a module's forward with its weights (and inputs) on an execution
device while the weights live elsewhere (another GPU, host RAM, disk).

API parity with `/root/reference/src/accelerate/hooks.py:43-783` (`ModelHook`, `SequentialHook`, `add_hook_to_module`,
`remove_hook_from_module`, `AlignDevicesHook`, the three `attach_*` helpers, `CpuOffload`, `UserCpuOffloadHook`,
`LayerwiseCastingHook`); `tests/test_big_modeling.py` pins the behaviour.

MI355X design: offloaded weights are streamed by an **`OffloadScheduler`**, one per dispatched model and execution
GPU, that owns the upload stream, the pinned host copies of host-offloaded weights, and the execution order of the
offloaded blocks (recorded on the first forward). While block i computes, block i+1's weights are already being
copied host -> HBM on the scheduler's high-priority stream (one HIP event per block), so PCIe transfers overlap
compute instead of sitting in front of every block (the reference uploads synchronously and notes prefetching as
missing, `benchmarks/big_model_inference/README.md:42-44`). `ACCELERATE_OFFLOAD_PREFETCH=0` turns prefetch off.
"""

from __future__ import annotations

import functools
import os
from collections.abc import Mapping
from typing import Optional, Union

import torch
import torch.nn as nn

from .utils.memory import clear_device_cache
from .utils.modeling import get_non_persistent_buffers, named_module_tensors
from .utils.offload import PrefixedDataset
from .utils.operations import find_device, send_to_device
from .utils.placement import recursive_getattr, set_module_tensor_to_device


# --------------------------------------------------------------------------------------------------- hook plumbing
class ModelHook:
    """Callbacks around a module's forward: `init_hook` when attached, `pre_forward` / `post_forward` around each
    call, `detach_hook` when removed. With `no_grad`, the wrapped forward runs without autograd."""

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
    """Several hooks applied in order (`post_forward` in the same order)."""

    def __init__(self, *hooks):
        self.hooks = hooks

    def init_hook(self, module):
        for h in self.hooks:
            module = h.init_hook(module)
        return module

    def pre_forward(self, module, *args, **kwargs):
        for h in self.hooks:
            args, kwargs = h.pre_forward(module, *args, **kwargs)
        return args, kwargs

    def post_forward(self, module, output):
        for h in self.hooks:
            output = h.post_forward(module, output)
        return output

    def detach_hook(self, module):
        for h in self.hooks:
            module = h.detach_hook(module)
        return module


class _HookedForward:
    """The forward installed on a hooked module: hook.pre_forward -> original forward -> hook.post_forward."""

    def __init__(self, module: nn.Module):
        self.module = module

    def __call__(self, *args, **kwargs):
        m = self.module
        hook = m._hf_hook
        args, kwargs = hook.pre_forward(m, *args, **kwargs)
        if hook.no_grad:
            with torch.no_grad():
                out = m._old_forward(*args, **kwargs)
        else:
            out = m._old_forward(*args, **kwargs)
        return hook.post_forward(m, out)


def _is_graph_module(module) -> bool:
    return "GraphModuleImpl" in str(type(module))


def add_hook_to_module(module: nn.Module, hook: ModelHook, append: bool = False):
    """Attach `hook` (stored as `module._hf_hook`, the original forward as `module._old_forward`). An existing hook
    is replaced, or with `append` chained before the new one."""
    if append and getattr(module, "_hf_hook", None) is not None:
        previous = module._hf_hook
        remove_hook_from_module(module)
        hook = SequentialHook(previous, hook)
    base = module._old_forward if (hasattr(module, "_hf_hook") and hasattr(module, "_old_forward")) else module.forward
    module._old_forward = base
    module = hook.init_hook(module)
    module._hf_hook = hook
    fwd = functools.update_wrapper(_HookedForward(module), base)
    if _is_graph_module(module):
        module.__class__.forward = fwd
    else:
        module.forward = fwd
    return module


def remove_hook_from_module(module: nn.Module, recurse: bool = False):
    """Detach the hook (its `detach_hook` runs) and restore the original forward; `recurse` does all submodules."""
    hook = getattr(module, "_hf_hook", None)
    if hook is not None:
        hook.detach_hook(module)
        del module._hf_hook
    if hasattr(module, "_old_forward"):
        if _is_graph_module(module):
            module.__class__.forward = module._old_forward
        else:
            module.forward = module._old_forward
        del module._old_forward
    for name in getattr(module, "_accelerate_added_attributes", []):
        if hasattr(module, name):
            delattr(module, name)
    if hasattr(module, "_accelerate_added_attributes"):
        del module._accelerate_added_attributes
    if recurse:
        for child in module.children():
            remove_hook_from_module(child, recurse=True)
    return module


def remove_hook_from_submodules(module: nn.Module):
    for m in module.modules():
        remove_hook_from_module(m)


def _install(module: nn.Module, name: str, value: torch.Tensor):
    """Make `value` parameter / buffer `name` (dotted) of `module` without a copy."""
    owner_path, _, attr = name.rpartition(".")
    owner = module.get_submodule(owner_path) if owner_path else module
    if attr in owner._parameters:
        old = owner._parameters[attr]
        if not isinstance(value, nn.Parameter):
            value = nn.Parameter(value, requires_grad=old.requires_grad if old is not None else False)
        owner._parameters[attr] = value
    else:
        owner._buffers[attr] = value


# --------------------------------------------------------------------------------------------------- offload stream
class OffloadScheduler:
    """Streams offloaded block weights to one execution GPU ahead of use (see module docstring)."""

    def __init__(self, device):
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.enabled = device.type == "cuda" and os.environ.get("ACCELERATE_OFFLOAD_PREFETCH", "1") != "0"
        self.stream = torch.cuda.Stream(device=device, priority=-1) if self.enabled else None
        self.order: list = []
        self.recording = True
        self.staged: dict = {}
        self.pinned: dict = {}  # (hook id, name) -> pinned host tensor (host-offloaded weights only)

    def host_copy(self, hook: "AlignDevicesHook", name: str, value: torch.Tensor) -> torch.Tensor:
        """A pinned host copy of a weight held in RAM (cached); disk-backed weights are pinned per use."""
        if value.device.type != "cpu":
            return value
        key = (id(hook), name)
        if hook.cache_host and key in self.pinned:
            return self.pinned[key]
        try:
            pinned = value.contiguous().pin_memory()
        except RuntimeError:
            return value
        if hook.cache_host:
            self.pinned[key] = pinned
        return pinned

    def ran(self, hook):
        """Record the block execution order over the first full pass."""
        if not self.recording:
            return
        if hook in self.order:
            self.recording = False
        else:
            self.order.append(hook)

    def take(self, hook) -> Optional[dict]:
        """Tensors prefetched for `hook`, ordered after their upload on the current stream."""
        item = self.staged.pop(id(hook), None)
        if item is None:
            return None
        tensors, event = item
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(event)
        for t in tensors.values():
            t.record_stream(cur)
        return tensors

    def prefetch_next(self, hook):
        if not self.enabled or self.recording or hook not in self.order:
            return
        nxt = self.order[(self.order.index(hook) + 1) % len(self.order)]
        if id(nxt) in self.staged:
            return
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        staged = {}
        with torch.cuda.stream(self.stream):
            for name in nxt.streamed_names():
                if name in nxt.tied_params_names:
                    continue  # tied weights go through the shared tied-parameter cache
                staged[name] = self.host_copy(nxt, name, nxt.weights_map[name]).to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.staged[id(nxt)] = (staged, ev)


def _scheduler_for(device, schedulers: Optional[dict]) -> Optional[OffloadScheduler]:
    if device is None or schedulers is None:
        return None
    dev = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
    if dev.type != "cuda":
        return None
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in schedulers:
        schedulers[key] = OffloadScheduler(torch.device("cuda", key))
    return schedulers[key]


# --------------------------------------------------------------------------------------------------- device hooks
class AlignDevicesHook(ModelHook):
    """Run the module on `execution_device`: inputs are moved there; with `offload`, the module's tensors stay on the
    meta device between calls and are materialised from `weights_map` for each forward (through the model's
    `OffloadScheduler` when it has one); `io_same_device` moves outputs back to where the inputs came from."""

    def __init__(
        self,
        execution_device: Optional[Union[int, str, torch.device]] = None,
        offload: bool = False,
        io_same_device: bool = False,
        weights_map: Optional[Mapping] = None,
        offload_buffers: bool = False,
        place_submodules: bool = False,
        skip_keys: Optional[Union[str, list]] = None,
        tied_params_map: Optional[dict] = None,
        scheduler: Optional[OffloadScheduler] = None,
        cache_host: bool = True,
    ):
        self.execution_device = execution_device
        self.offload = offload
        self.io_same_device = io_same_device
        self.weights_map = weights_map
        self.offload_buffers = offload_buffers
        self.place_submodules = place_submodules
        self.skip_keys = skip_keys
        self.tied_params_map = tied_params_map
        self.scheduler = scheduler
        self.cache_host = cache_host
        self.input_device = None
        self.param_original_devices = {}
        self.buffer_original_devices = {}
        self.tied_params_names = set()
        self.tied_pointers_to_remove = set()
        self._streamed = None

    def __repr__(self):
        return (
            f"AlignDevicesHook(execution_device={self.execution_device}, offload={self.offload}, "
            f"io_same_device={self.io_same_device}, offload_buffers={self.offload_buffers}, "
            f"place_submodules={self.place_submodules}, skip_keys={repr(self.skip_keys)})"
        )

    def _tensors(self, module, include_buffers=True, persistent_only=False):
        return named_module_tensors(module, include_buffers=include_buffers, recurse=self.place_submodules,
                                    remove_non_persistent=persistent_only)

    def streamed_names(self, module=None) -> list:
        """Names of the tensors materialised per forward (offloaded params, persistent buffers if offloaded)."""
        if self._streamed is None and module is not None:
            self._streamed = [n for n, _ in self._tensors(module, include_buffers=self.offload_buffers, persistent_only=True)]
        return self._streamed or []

    def init_hook(self, module):
        if str(self.execution_device) == "meta":
            self.tied_params_map = None
        dev = self.execution_device
        if not self.offload:
            if dev is not None:
                for name, _ in self._tensors(module):
                    set_module_tensor_to_device(module, name, dev, tied_params_map=self.tied_params_map)
            return module
        self.original_devices = {name: t.device for name, t in self._tensors(module)}
        if self.weights_map is None:
            self.weights_map = {name: t.to("cpu") for name, t in self._tensors(module, include_buffers=self.offload_buffers)}
        for name in self.streamed_names(module):
            if self.tied_params_map is not None and recursive_getattr(module, name).data_ptr() in self.tied_params_map:
                self.tied_params_names.add(name)
            set_module_tensor_to_device(module, name, "meta")
        if dev is not None:
            # buffers that are not streamed live on the execution device for good
            kept = (n for n, _ in module.named_buffers(recurse=self.place_submodules)) if not self.offload_buffers else \
                get_non_persistent_buffers(module, recurse=self.place_submodules)
            for name in kept:
                set_module_tensor_to_device(module, name, dev, tied_params_map=self.tied_params_map)
        return module

    def pre_forward(self, module, *args, **kwargs):
        if self.io_same_device:
            self.input_device = find_device([args, kwargs])
        if self.offload:
            self._materialise(module)
        return send_to_device(args, self.execution_device), send_to_device(kwargs, self.execution_device, skip_keys=self.skip_keys)

    def _materialise(self, module):
        self.tied_pointers_to_remove = set()
        sched = self.scheduler
        staged = None
        if sched is not None and sched.enabled:
            sched.ran(self)
            staged = sched.take(self)
        tied = self.tied_params_map
        for name in self.streamed_names(module):
            if staged is not None and name in staged:
                _install(module, name, staged[name])
                continue
            value = self.weights_map[name]
            if name in self.tied_params_names and value.data_ptr() not in tied:
                tied[value.data_ptr()] = {}
            if tied is not None and value.data_ptr() in tied and self.execution_device not in tied[value.data_ptr()]:
                self.tied_pointers_to_remove.add((value.data_ptr(), self.execution_device))
            if sched is not None and sched.enabled and name not in self.tied_params_names:
                value = sched.host_copy(self, name, value)
            set_module_tensor_to_device(module, name, self.execution_device, value=value, tied_params_map=tied)
        if sched is not None and sched.enabled:
            sched.prefetch_next(self)

    def post_forward(self, module, output):
        if self.offload:
            for name in self.streamed_names(module):
                set_module_tensor_to_device(module, name, "meta")
            for ptr, device in self.tied_pointers_to_remove:
                self.tied_params_map.get(ptr, {}).pop(device, None)
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


# --------------------------------------------------------------------------------------------------- attach helpers
def attach_execution_device_hook(module, execution_device, skip_keys=None, preload_module_classes=None, tied_params_map=None):
    """Give every module of the subtree that holds tensors and has no hook an execution-device hook (no offload).
    When the subtree's root is a `preload_module_classes` module, its own hook covers its children (the class test
    applies to the root only, as upstream)."""
    stack = [(module, True)]
    while stack:
        m, is_root = stack.pop()
        if not hasattr(m, "_hf_hook") and len(m.state_dict()) > 0:
            add_hook_to_module(m, AlignDevicesHook(execution_device, skip_keys=skip_keys, tied_params_map=tied_params_map))
        if is_root and preload_module_classes is not None and m.__class__.__name__ in preload_module_classes:
            continue
        stack.extend((c, False) for c in reversed(list(m.children())))


def attach_align_device_hook(module, execution_device=None, offload=False, weights_map=None, offload_buffers=False,
                             module_name="", skip_keys=None, preload_module_classes=None, tied_params_map=None,
                             schedulers=None, cache_host=True):
    """Hook every module of the subtree that directly owns tensors. A `preload_module_classes` module under offload is
    streamed as a whole (one hook, its submodules' tensors included) and not descended into."""
    stack = [(module, module_name)]
    while stack:
        m, name = stack.pop()
        whole = offload and preload_module_classes is not None and m.__class__.__name__ in preload_module_classes
        if whole or next(iter(named_module_tensors(m)), None) is not None:
            view = PrefixedDataset(weights_map, f"{name}." if name else "") if weights_map is not None else None
            add_hook_to_module(
                m,
                AlignDevicesHook(execution_device=execution_device, offload=offload, weights_map=view,
                                 offload_buffers=offload_buffers, place_submodules=whole, skip_keys=skip_keys,
                                 tied_params_map=tied_params_map,
                                 scheduler=_scheduler_for(execution_device, schedulers) if offload else None,
                                 cache_host=cache_host),
                append=True,
            )
        if whole:
            continue
        stack.extend(reversed([(c, f"{name}.{n}" if name else n) for n, c in m.named_children()]))


def attach_align_device_hook_on_blocks(module, execution_device=None, offload=False, weights_map=None,
                                       offload_buffers=False, module_name="", skip_keys=None,
                                       preload_module_classes=None, tied_params_map=None, schedulers=None,
                                       cache_host=None):
    """Hooks for a device map: `execution_device` / `offload` map block names to their execution device and whether
    their weights are offloaded. A resident block gets one hook that places the whole block; an offloaded block is
    streamed per submodule; the root also moves outputs back to the caller's device."""
    if not isinstance(execution_device, Mapping) and not isinstance(offload, dict):
        if offload:
            attach_align_device_hook(module, execution_device=execution_device, offload=True, weights_map=weights_map,
                                     offload_buffers=offload_buffers, module_name=module_name, skip_keys=skip_keys,
                                     tied_params_map=tied_params_map, schedulers=schedulers)
        else:
            add_hook_to_module(module, AlignDevicesHook(execution_device=execution_device, io_same_device=True,
                                                        skip_keys=skip_keys, place_submodules=True,
                                                        tied_params_map=tied_params_map))
        return
    if not isinstance(execution_device, Mapping):
        execution_device = {k: execution_device for k in offload}
    if not isinstance(offload, Mapping):
        offload = {k: offload for k in execution_device}
    cache_host = cache_host or {}

    stack = [(module, module_name)]
    while stack:
        m, name = stack.pop()
        is_root = name == ""
        if name in execution_device and name in offload:
            dev = execution_device[name]
            if not offload[name]:
                add_hook_to_module(m, AlignDevicesHook(execution_device=dev, offload_buffers=offload_buffers,
                                                       io_same_device=is_root, place_submodules=True,
                                                       skip_keys=skip_keys, tied_params_map=tied_params_map))
                attach_execution_device_hook(m, dev, skip_keys=skip_keys, tied_params_map=tied_params_map)
            else:
                attach_align_device_hook(m, execution_device=dev, offload=True, weights_map=weights_map,
                                         offload_buffers=offload_buffers, module_name=name, skip_keys=skip_keys,
                                         preload_module_classes=preload_module_classes, tied_params_map=tied_params_map,
                                         schedulers=schedulers, cache_host=cache_host.get(name, True))
                if not hasattr(m, "_hf_hook"):
                    add_hook_to_module(m, AlignDevicesHook(execution_device=dev, io_same_device=is_root,
                                                           skip_keys=skip_keys, tied_params_map=tied_params_map))
                attach_execution_device_hook(m, dev, preload_module_classes=preload_module_classes,
                                             skip_keys=skip_keys, tied_params_map=tied_params_map)
        elif is_root:
            add_hook_to_module(m, AlignDevicesHook(execution_device=execution_device.get(""), io_same_device=True,
                                                   skip_keys=skip_keys, tied_params_map=tied_params_map))
        stack.extend(reversed([(c, f"{name}.{n}" if name else n) for n, c in m.named_children()]))


# --------------------------------------------------------------------------------------------------- other hooks
class CpuOffload(ModelHook):
    """Whole-model offload between calls: the model lives on the host and moves to `execution_device` for its
    forward; a chained `prev_module_hook` sends the previous model of a pipeline back first."""

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
    """Handle returned by `cpu_offload_with_hook`: `offload()` sends the model back to the host, `remove()` detaches."""

    def __init__(self, model, hook):
        self.model = model
        self.hook = hook

    def offload(self):
        self.hook.init_hook(self.model)

    def remove(self):
        remove_hook_from_module(self.model)


# storage -> compute upcasts that are exact, so that the storage tensor can be kept and the compute copy dropped after
# the forward with the same result as the reference's `.to(storage)` round trip
_EXACT_UPCASTS = {
    (torch.float8_e4m3fn, torch.bfloat16), (torch.float8_e4m3fn, torch.float16), (torch.float8_e4m3fn, torch.float32),
    (torch.float8_e5m2, torch.bfloat16), (torch.float8_e5m2, torch.float16), (torch.float8_e5m2, torch.float32),
    (torch.float16, torch.float32), (torch.bfloat16, torch.float32),
}


class LayerwiseCastingHook(ModelHook):
    """Weights stored in `storage_dtype` (e.g. fp8) and used in `compute_dtype` for the duration of each forward
    (reference hooks.py:757-783: `module.to(compute)` before and `module.to(storage)` after every forward).

    When the upcast is exact (fp8 -> bf16 / fp16 / fp32, fp16 / bf16 -> fp32) the storage tensors stay resident: the
    pre-forward hook upcasts all of the module's floating-point tensors into compute-dtype scratch tensors in one HIP
    launch (`ext().upcast_multi`, csrc/kernels/cast.hip) and points the parameters at them; the post-forward hook points
    them back at the untouched storage tensors and the scratch is freed. One read of the stored weights per forward and
    no downcast pass; values and dtypes seen by the caller are the reference's. Other dtype pairs (a lossy "upcast")
    take the reference's `.to()` round trip."""

    _is_stateful = False

    def __init__(self, storage_dtype: torch.dtype, compute_dtype: torch.dtype, non_blocking: bool):
        self.storage_dtype = storage_dtype
        self.compute_dtype = compute_dtype
        self.non_blocking = non_blocking
        self._keep = (storage_dtype, compute_dtype) in _EXACT_UPCASTS
        self._stored = None

    def init_hook(self, module):
        module.to(dtype=self.storage_dtype, non_blocking=self.non_blocking)
        return module

    def _tensors(self, module):
        """(tensor, data) of the module's own parameters and buffers held in the storage dtype."""
        out = []
        for holder in (module._parameters, module._buffers):
            for t in holder.values():
                if t is not None and t.dtype == self.storage_dtype:
                    out.append(t)
        return out

    def pre_forward(self, module, *args, **kwargs):
        items = self._tensors(module) if self._keep and next(module.children(), None) is None else None
        if not items:
            module.to(dtype=self.compute_dtype, non_blocking=self.non_blocking)
            return args, kwargs
        srcs = [t.data for t in items]
        dsts = [torch.empty(s.shape, dtype=self.compute_dtype, device=s.device) for s in srcs]
        done = False
        if srcs[0].is_cuda and all(s.is_contiguous() for s in srcs):
            from .ops._ext import ext, use_native

            if use_native(srcs[0]):
                done = ext().upcast_multi(srcs, dsts)
        if not done:
            for s, d in zip(srcs, dsts):
                d.copy_(s, non_blocking=self.non_blocking)
        for t, d in zip(items, dsts):
            t.data = d
        self._stored = list(zip(items, srcs))
        return args, kwargs

    def post_forward(self, module, output):
        if self._stored is None:
            module.to(dtype=self.storage_dtype, non_blocking=self.non_blocking)
            return output
        for t, s in self._stored:
            t.data = s
        self._stored = None
        return output


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
