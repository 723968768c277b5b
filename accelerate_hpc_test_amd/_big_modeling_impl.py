"""Big-model inference implementation: device-map planner, checkpoint loading, dispatch / offload.

Parity: `/root/reference/src/accelerate/big_modeling.py:174-790` and `utils/modeling.py:217-1785`:
`set_module_tensor_to_device`, `find_tied_parameters`/`retie_parameters`, `get_max_memory`, `get_balanced_memory`,
`get_max_layer_size`, `infer_auto_device_map` (greedy fill GPU0..N-1 → cpu → disk, reserving the largest
no-split layer on the main devices, splitting modules that may be split, keeping tied parameters together),
`check_device_map`, `load_state_dict`, `load_checkpoint_in_model`, `dispatch_model`, `cpu_offload(_with_hook)`,
`disk_offload`, `load_checkpoint_and_dispatch`, `attach_layerwise_casting_hooks`.

MI355X-specific:
* GPU memory budgets come from `torch.cuda.mem_get_info` on each MI355X (288 GB HBM3E); with 8 devices a 70B bf16
  model (≈140 GB) is spread over a few GPUs instead of needing offload at all.
* Checkpoint tensors bound for a GPU are uploaded through the native `H2DEngine` (csrc/runtime/h2d_engine.cpp):
  pageable (mmap'd safetensors) data is copied by worker threads into a pinned staging ring and DMA'd
  asynchronously, instead of a synchronous pageable `.to(device)` per tensor.
* Offloaded modules get asynchronous next-module prefetch (hooks.OffloadPrefetcher).
"""

from __future__ import annotations

import contextlib
import gc
import json
import logging
import os
import re
import tempfile
from collections import OrderedDict, defaultdict
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
from .logging import get_logger
from .utils.constants import SAFE_WEIGHTS_INDEX_NAME, SAFE_WEIGHTS_NAME, WEIGHTS_INDEX_NAME, WEIGHTS_NAME
from .utils.memory import clear_device_cache
from .utils.modeling import compute_module_sizes, convert_file_size_to_int, dtype_byte_size, named_module_tensors
from .utils.offload import (
    OffloadedWeightsLoader,
    extract_submodules_state_dict,
    load_offloaded_weight,
    offload_state_dict,
    offload_weight,
    save_offload_index,
)

logger = logging.getLogger(__name__)  # plain logger: usable without an Accelerator / PartialState


# ---------------------------------------------------------------------------------------------------- tensors
def _device(d):
    if isinstance(d, int):
        return torch.device("cuda", d)
    return torch.device(d)


def set_module_tensor_to_device(
    module: nn.Module,
    tensor_name: str,
    device: Union[int, str, torch.device],
    value: Optional[torch.Tensor] = None,
    dtype: Optional[Union[str, torch.dtype]] = None,
    fp16_statistics: Optional[torch.HalfTensor] = None,
    tied_params_map: Optional[dict] = None,
    non_blocking: bool = False,
    clear_cache: bool = True,
):
    """Move (or set from `value`) parameter/buffer `tensor_name` of `module` to `device`, keeping the Parameter
    class and `requires_grad`. Reference `utils/modeling.py:217-425`."""
    if "." in tensor_name:
        splits = tensor_name.split(".")
        for split in splits[:-1]:
            new_module = getattr(module, split)
            if new_module is None:
                raise ValueError(f"{module} has no attribute {split}.")
            module = new_module
        tensor_name = splits[-1]
    if tensor_name not in module._parameters and tensor_name not in module._buffers:
        raise ValueError(f"{module} does not have a parameter or a buffer named {tensor_name}.")
    is_buffer = tensor_name in module._buffers
    old_value = getattr(module, tensor_name)
    if (
        value is not None
        and tied_params_map is not None
        and value.data_ptr() in tied_params_map
        and device in tied_params_map[value.data_ptr()]
    ):
        module._parameters[tensor_name] = tied_params_map[value.data_ptr()][device]
        return
    elif (
        tied_params_map is not None
        and old_value.data_ptr() in tied_params_map
        and device in tied_params_map[old_value.data_ptr()]
    ):
        module._parameters[tensor_name] = tied_params_map[old_value.data_ptr()][device]
        return
    if old_value.device == torch.device("meta") and device not in ["meta", torch.device("meta")] and value is None:
        raise ValueError(f"{tensor_name} is on the meta device, we need a `value` to put in on {device}.")
    param = module._parameters[tensor_name] if tensor_name in module._parameters else None
    param_cls = type(param)
    if value is not None:
        if old_value.shape != value.shape and param_cls.__name__ != "Params4bit":
            raise ValueError(
                f'Trying to set a tensor of shape {value.shape} in "{tensor_name}" (which has shape {old_value.shape}), this looks incorrect.'
            )
        if dtype is None:
            value = value.to(old_value.dtype, non_blocking=non_blocking)
        elif not str(value.dtype).startswith(("torch.uint", "torch.int", "torch.bool")):
            value = value.to(dtype, non_blocking=non_blocking)
    device_quantization = None
    with torch.no_grad():
        if value is None:
            new_value = old_value.to(device, non_blocking=non_blocking)
            if dtype is not None and device in ["meta", torch.device("meta")]:
                if not str(old_value.dtype).startswith(("torch.uint", "torch.int", "torch.bool")):
                    new_value = new_value.to(dtype, non_blocking=non_blocking)
                if not is_buffer:
                    module._parameters[tensor_name] = param_cls(new_value, requires_grad=old_value.requires_grad)
        elif isinstance(value, torch.Tensor):
            new_value = value.to(device, non_blocking=non_blocking)
        else:
            new_value = torch.tensor(value, device=device)
        if device_quantization is not None:
            device = device_quantization
        if is_buffer:
            module._buffers[tensor_name] = new_value
        elif value is not None or not _same_device(torch.device(device), module._parameters[tensor_name].device):
            param_cls = type(module._parameters[tensor_name])
            kwargs = module._parameters[tensor_name].__dict__
            if param_cls.__name__ in ["Int8Params", "FP4Params", "Params4bit"]:
                new_value = param_cls(new_value, requires_grad=old_value.requires_grad, **kwargs).to(device)
            else:
                new_value = param_cls(new_value, requires_grad=old_value.requires_grad)
            module._parameters[tensor_name] = new_value
    if device != "cpu" and clear_cache and False:
        clear_device_cache()
    if (
        tied_params_map is not None
        and old_value.data_ptr() in tied_params_map
        and device not in tied_params_map[old_value.data_ptr()]
    ):
        tied_params_map[old_value.data_ptr()][device] = new_value
    elif (
        value is not None
        and tied_params_map is not None
        and value.data_ptr() in tied_params_map
        and device not in tied_params_map[value.data_ptr()]
    ):
        tied_params_map[value.data_ptr()][device] = new_value


def _same_device(a: torch.device, b: torch.device) -> bool:
    if a.type != b.type:
        return False
    if a.type == "cuda":
        ai = a.index if a.index is not None else torch.cuda.current_device()
        bi = b.index if b.index is not None else torch.cuda.current_device()
        return ai == bi
    return True


def find_tied_parameters(model: nn.Module, **kwargs) -> list[list[str]]:
    """Groups of parameter names sharing the same Parameter object (e.g. tied embeddings / lm head)."""
    all_named = {name: p for name, p in model.named_parameters(remove_duplicate=False)}
    by_id = defaultdict(list)
    for name, p in all_named.items():
        by_id[id(p)].append(name)
    return sorted([sorted(v) for v in by_id.values() if len(v) > 1])


def retie_parameters(model, tied_params):
    for tied_group in tied_params:
        param_to_tie = None
        for param_name in tied_group:
            module = model
            splits = param_name.split(".")
            for split in splits[:-1]:
                module = getattr(module, split)
            param = getattr(module, splits[-1])
            if param_to_tie is None and param.device != torch.device("meta"):
                param_to_tie = param
                break
        if param_to_tie is not None:
            for param_name in tied_group:
                module = model
                splits = param_name.split(".")
                for split in splits[:-1]:
                    module = getattr(module, split)
                setattr(module, splits[-1], param_to_tie)


def recursive_getattr(obj, attr: str):
    import functools

    return functools.reduce(getattr, [obj] + attr.split("."))


# ---------------------------------------------------------------------------------------------------- planner
def get_max_memory(max_memory: Optional[dict] = None) -> dict:
    """Available memory per device: GPU i → free HBM (mem_get_info), "cpu" → available RAM."""
    import psutil

    if max_memory is None:
        max_memory = {}
        if torch.cuda.is_available():
            for i in range(torch.cuda.device_count()):
                try:
                    _ = torch.tensor([0], device=i)
                    max_memory[i] = torch.cuda.mem_get_info(i)[0]
                except Exception:
                    continue
        max_memory["cpu"] = psutil.virtual_memory().available
        return max_memory
    for key in max_memory:
        if isinstance(max_memory[key], str):
            max_memory[key] = convert_file_size_to_int(max_memory[key])
    gpu_devices = [k for k in max_memory.keys() if isinstance(k, int)]
    gpu_devices.sort()
    if torch.cuda.is_available():
        num_devices = torch.cuda.device_count()
        for device in gpu_devices:
            if device >= num_devices or device < 0:
                logger.warning(f"Device {device} is not available, available devices are {list(range(num_devices))}")
    all_devices = gpu_devices + [k for k in ["mps", "cpu", "disk"] if k in max_memory.keys()]
    for k in max_memory.keys():
        if k not in all_devices:
            raise ValueError(f"Device {k} is not recognized, available devices are integers(for GPU/XPU), 'mps', 'cpu' and 'disk'")
    return {k: max_memory[k] for k in all_devices}


def clean_device_map(device_map: dict, module_name: str = ""):
    """Collapse sub-entries that all share one device into their parent entry."""
    prefix = "" if module_name == "" else f"{module_name}."
    values = [v for k, v in device_map.items() if k.startswith(prefix)]
    if len(set(values)) == 1 and len(values) > 1:
        for k in [k for k in device_map if k.startswith(prefix)]:
            del device_map[k]
        device_map[module_name] = values[0]
    children_modules = [k for k in device_map.keys() if k.startswith(prefix) and len(k) > len(module_name)]
    idx = len(module_name.split(".")) + 1 if len(module_name) > 0 else 1
    children_modules = set(".".join(k.split(".")[:idx]) for k in children_modules)
    for child in children_modules:
        clean_device_map(device_map, module_name=child)
    return device_map


def get_max_layer_size(modules: list, module_sizes: dict, no_split_module_classes: list[str]):
    """Largest "layer" (a leaf or a no-split module) among `modules` → (size, names)."""
    max_size = 0
    layer_names = []
    modules_to_treat = modules.copy()
    while len(modules_to_treat) > 0:
        module_name, module = modules_to_treat.pop(0)
        modules_children = list(module.named_children()) if isinstance(module, nn.Module) else []
        if len(modules_children) == 0 or module.__class__.__name__ in no_split_module_classes:
            size = module_sizes[module_name]
            if size > max_size:
                max_size = size
                layer_names = [module_name]
            elif size == max_size:
                layer_names.append(module_name)
        else:
            modules_to_treat = [(f"{module_name}.{n}", v) for n, v in modules_children] + modules_to_treat
    return max_size, layer_names


def calculate_maximum_sizes(model: nn.Module):
    sizes = compute_module_sizes(model)
    no_split_modules = getattr(model, "_no_split_modules", None)
    if no_split_modules is None:
        no_split_modules = []
    modules_to_treat = list(model.named_parameters(recurse=False)) + list(model.named_children()) + list(model.named_buffers(recurse=False))
    largest_layer = get_max_layer_size(modules_to_treat, sizes, no_split_modules)
    total_size = sizes[""]
    return total_size, largest_layer


def get_balanced_memory(
    model: nn.Module,
    max_memory: Optional[dict] = None,
    no_split_module_classes: Optional[list[str]] = None,
    dtype=None,
    special_dtypes=None,
    low_zero: bool = False,
):
    """Per-GPU budgets that spread the model evenly (reference utils/modeling.py:918-1049)."""
    user_not_set_max_memory = max_memory is None
    max_memory = get_max_memory(max_memory)
    gpu_keys = [k for k in max_memory if isinstance(k, int) and max_memory[k] > 0]
    num_devices = len(gpu_keys)
    if num_devices == 0:
        return max_memory
    if num_devices == 1:
        low_zero = False
        if user_not_set_max_memory:
            for k in max_memory.keys():
                if isinstance(k, int):
                    max_memory[k] = int(max_memory[k] * 0.9)  # keep headroom for activations
    module_sizes = compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes)
    per_gpu = module_sizes[""] // (num_devices - 1 if low_zero else num_devices)
    if no_split_module_classes is None:
        no_split_module_classes = []
    elif not isinstance(no_split_module_classes, (list, tuple)):
        no_split_module_classes = [no_split_module_classes]
    if len(no_split_module_classes) > 0:
        no_split_children = {}
        for name, size in module_sizes.items():
            if name == "":
                continue
            submodule = model
            for submodule_name in name.split("."):
                submodule = getattr(submodule, submodule_name)
            class_name = submodule.__class__.__name__
            if class_name in no_split_module_classes and class_name not in no_split_children:
                no_split_children[class_name] = size
            if set(no_split_children.keys()) == set(no_split_module_classes):
                break
        buffer = max(no_split_children.values()) if len(no_split_children) > 0 else 0
    else:
        buffer = 0
    leaves = get_module_leaves(module_sizes)
    module_sizes_leaves = {n: v for n, v in module_sizes.items() if n in leaves}
    mean_leaves = int(sum(module_sizes_leaves.values()) / max(len(leaves), 1))
    buffer = int(1.25 * max(buffer, mean_leaves))
    per_gpu += buffer
    gpus_idx_list = sorted(gpu_keys)
    for idx in gpus_idx_list[:-1]:
        max_memory[idx] = min(max_memory[0] if low_zero and idx == 0 else per_gpu, max_memory[idx])
    if low_zero:
        min_zero = max(0, module_sizes[""] - sum([max_memory[i] for i in range(1, num_devices)]))
        max_memory[0] = min(min_zero, max_memory[0])
    return max_memory


def get_module_leaves(module_sizes):
    module_children = {}
    for module in module_sizes:
        if module == "" or "." not in module:
            continue
        parent = module.rsplit(".", 1)[0]
        module_children[parent] = module_children.get(parent, 0) + 1
    return [module for module in module_sizes if module_children.get(module, 0) == 0 and module != ""]


def _module_size_with_ties(tied_params, module_size, module_sizes, modules_to_treat):
    if len(tied_params) < 1:
        return module_size, [], []
    tied_module_names, tied_modules = [], []
    for tied_param in tied_params:
        tied_module_index = [i for i, (n, _) in enumerate(modules_to_treat) if tied_param.startswith(n + ".")]
        if not tied_module_index:
            continue
        tied_module_names.append(modules_to_treat[tied_module_index[0]][0])
        tied_modules.append(modules_to_treat[tied_module_index[0]][1])
    module_size_with_ties = module_size
    for tied_param, tied_module_name in zip(tied_params, tied_module_names):
        module_size_with_ties += module_sizes[tied_module_name] - module_sizes[tied_param]
    return module_size_with_ties, tied_module_names, tied_modules


def infer_auto_device_map(
    model: nn.Module,
    max_memory: Optional[dict] = None,
    no_split_module_classes: Optional[list[str]] = None,
    dtype=None,
    special_dtypes=None,
    verbose: bool = False,
    clean_result: bool = True,
    offload_buffers: bool = False,
    fallback_allocation: bool = False,
):
    """Greedy device map: fill GPU 0, 1, ... then cpu, then disk, in module order (reference
    utils/modeling.py:1278-1583)."""
    max_memory = get_max_memory(max_memory)
    if no_split_module_classes is None:
        no_split_module_classes = []
    elif not isinstance(no_split_module_classes, (list, tuple)):
        no_split_module_classes = [no_split_module_classes]
    devices = list(max_memory.keys())
    if "disk" not in devices:
        devices.append("disk")
    gpus = [device for device in devices if device not in ["cpu", "disk"]]
    main_devices = [gpus[0], "cpu"] if len(gpus) > 0 else ["cpu"]
    module_sizes = compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes)
    tied_parameters = find_tied_parameters(model)
    device_map = OrderedDict()
    current_device = 0
    device_memory_used = {device: 0 for device in devices}
    modules_to_treat = list(model.named_parameters(recurse=False)) + list(model.named_children()) + list(model.named_buffers(recurse=False))
    max_layer_size, max_layer_names = get_max_layer_size(modules_to_treat, module_sizes, no_split_module_classes)
    while len(modules_to_treat) > 0:
        name, module = modules_to_treat.pop(0)
        if verbose:
            print(f"\nTreating module {name}.")
        max_layer_names = [n for n in max_layer_names if n != name and not n.startswith(name + ".")]
        if len(max_layer_names) == 0:
            max_layer_size, max_layer_names = get_max_layer_size(
                [(n, m) for n, m in modules_to_treat if isinstance(m, nn.Module)], module_sizes, no_split_module_classes
            )
        module_size = module_sizes[name]
        tied_param_groups = [
            tied_group for tied_group in tied_parameters if any(name + "." in k + "." for k in tied_group) and not all(name + "." in k + "." for k in tied_group)
        ]
        tied_params = sum([[p for p in tied_group if name + "." not in p + "."] for tied_group in tied_param_groups], [])
        device = devices[current_device]
        current_max_size = max_memory[device] if device != "disk" else None
        current_memory_reserved = 0
        if devices[current_device] in main_devices:
            current_max_size = current_max_size - max_layer_size if current_max_size is not None else None
            current_memory_reserved = max_layer_size
        module_size_with_ties, tied_module_names, tied_modules = _module_size_with_ties(tied_params, module_size, module_sizes, modules_to_treat)
        if current_max_size is not None and device_memory_used[device] + module_size_with_ties > current_max_size:
            if verbose:
                print(f"Not enough space on {devices[current_device]} to put {name} (space available {current_max_size - device_memory_used[device]}, module size {module_size_with_ties}).")
            modules_children = [] if isinstance(module, (nn.Parameter, torch.Tensor)) else list(module.named_children())
            if len(modules_children) == 0 or module.__class__.__name__ in no_split_module_classes:
                # cannot split: move to the next device
                device_memory_used[device] = device_memory_used[device] + current_memory_reserved
                current_device += 1
                modules_to_treat = [(name, module)] + modules_to_treat
                continue
            modules_children = list(module.named_parameters(recurse=False)) + modules_children
            modules_to_treat = [(f"{name}.{n}", v) for n, v in modules_children] + modules_to_treat
            max_layer_size, max_layer_names = get_max_layer_size(
                [(n, m) for n, m in modules_to_treat if isinstance(m, nn.Module)], module_sizes, no_split_module_classes
            )
            continue
        if verbose:
            print(f"Putting {name} (size={module_size}) on {devices[current_device]}.")
        device_map[name] = devices[current_device]
        device_memory_used[device] += module_size
        for tied_module_name, tied_module in zip(tied_module_names, tied_modules):
            if tied_module_name in [m[0] for m in modules_to_treat]:
                idx = [m[0] for m in modules_to_treat].index(tied_module_name)
                modules_to_treat.pop(idx)
            device_map[tied_module_name] = devices[current_device]
            device_memory_used[device] += module_sizes[tied_module_name]
    if clean_result:
        device_map = clean_device_map(device_map)
    non_gpu_buffer_size = 0
    if not offload_buffers:
        for name, dev in device_map.items():
            if dev in ("cpu", "disk"):
                try:
                    sub = model.get_submodule(name)
                    non_gpu_buffer_size += sum(b.numel() * b.element_size() for b in sub.buffers())
                except AttributeError:
                    pass
    return device_map


def check_device_map(model: nn.Module, device_map: dict):
    all_model_tensors = [name for name, _ in model.state_dict().items()]
    for module_name in device_map.keys():
        if module_name == "":
            all_model_tensors.clear()
            break
        all_model_tensors = [name for name in all_model_tensors if not name == module_name and not name.startswith(module_name + ".")]
    if len(all_model_tensors) > 0:
        non_covered_params = ", ".join(all_model_tensors)
        raise ValueError(f"The device_map provided does not give any device for the following parameters: {non_covered_params}")


# ---------------------------------------------------------------------------------------------------- loading
def load_state_dict(checkpoint_file, device_map=None):
    """Load a .safetensors (memory-mapped, lazy) or torch checkpoint (weights_only) file to CPU tensors."""
    if checkpoint_file.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(checkpoint_file, device="cpu")
    return torch.load(checkpoint_file, map_location=torch.device("cpu"), weights_only=True)


def _checkpoint_files(checkpoint):
    if os.path.isfile(checkpoint):
        if str(checkpoint).endswith(".json"):
            index_filename = checkpoint
            folder = os.path.dirname(checkpoint)
            with open(index_filename) as f:
                index = json.loads(f.read())
            if "weight_map" in index:
                index = index["weight_map"]
            return sorted({os.path.join(folder, f) for f in index.values()})
        return [checkpoint]
    if os.path.isdir(checkpoint):
        for idx_name in (SAFE_WEIGHTS_INDEX_NAME, WEIGHTS_INDEX_NAME):
            p = os.path.join(checkpoint, idx_name)
            if os.path.isfile(p):
                return _checkpoint_files(p)
        for name in (SAFE_WEIGHTS_NAME, WEIGHTS_NAME):
            p = os.path.join(checkpoint, name)
            if os.path.isfile(p):
                return [p]
        potential = [f for f in os.listdir(checkpoint) if f.endswith((".safetensors", ".bin"))]
        if len(potential) == 1:
            return [os.path.join(checkpoint, potential[0])]
        raise ValueError(f"{checkpoint} is not a folder containing a `.bin`/`.safetensors` file or an index.")
    raise ValueError(f"`checkpoint` should be the path to a file or a folder, got {checkpoint}.")


def _device_for(param_name, device_map):
    if device_map is None:
        return None
    module_name = param_name
    while len(module_name) > 0 and module_name not in device_map:
        module_name = ".".join(module_name.split(".")[:-1])
    if module_name == "" and "" not in device_map:
        raise ValueError(f"{param_name} doesn't have any device set.")
    return device_map[module_name]


_ENGINES = {}


def _h2d_engine(device_index):
    """Shared native async H2D engine per GPU (None when the extension is unavailable)."""
    from .ops import _ext

    if not _ext.available():
        return None
    if device_index not in _ENGINES:
        _ENGINES[device_index] = _ext.ext().H2DEngine(device_index, 4, 64 << 20, 4)
    return _ENGINES[device_index]


def load_checkpoint_in_model(
    model: nn.Module,
    checkpoint: Union[str, os.PathLike],
    device_map: Optional[dict] = None,
    offload_folder: Optional[Union[str, os.PathLike]] = None,
    dtype=None,
    offload_state_dict: bool = False,
    offload_buffers: bool = False,
    keep_in_fp32_modules: list[str] = None,
    offload_8bit_bnb: bool = False,
    strict: bool = False,
    full_state_dict: bool = True,
    broadcast_from_rank0: bool = False,
):
    """Load a (sharded) checkpoint into `model`, placing each tensor per `device_map` (GPU / cpu / disk)."""
    tied_params = find_tied_parameters(model)
    if offload_folder is None and device_map is not None and "disk" in device_map.values():
        raise ValueError("At least one of the model submodule will be offloaded to disk, please pass along an `offload_folder`.")
    elif offload_folder is not None and device_map is not None and "disk" in device_map.values():
        os.makedirs(offload_folder, exist_ok=True)
    if isinstance(dtype, str):
        dtype = getattr(torch, dtype.replace("torch.", ""))
    files = _checkpoint_files(str(checkpoint))
    offload_index = {}
    if offload_state_dict:
        state_dict_folder = tempfile.mkdtemp()
        state_dict_index = {}
    unexpected_keys = set()
    model_keys = set(model.state_dict().keys())
    engines_used = set()
    for checkpoint_file in files:
        loaded = load_state_dict(checkpoint_file, device_map=device_map)
        if device_map is None:
            model.load_state_dict(loaded, strict=strict)
            unexpected_keys.update(set(loaded.keys()) - model_keys)
        else:
            for param_name, param in loaded.items():
                if param_name not in model_keys:
                    unexpected_keys.add(param_name)
                    if not strict:
                        continue
                param_device = _device_for(param_name, device_map)
                new_dtype = dtype
                if dtype is not None and torch.is_floating_point(param):
                    if keep_in_fp32_modules is not None and any(m in param_name.split(".") for m in keep_in_fp32_modules):
                        new_dtype = torch.float32
                if param_device == "disk":
                    if offload_buffers or param_name not in dict(model.named_buffers()):
                        set_module_tensor_to_device(model, param_name, "meta")
                        offload_weight(param, param_name, offload_folder, index=offload_index)
                        continue
                elif param_device == "cpu" and offload_state_dict:
                    set_module_tensor_to_device(model, param_name, "meta")
                    offload_weight(param, param_name, state_dict_folder, index=state_dict_index)
                    continue
                dev = _device(param_device)
                if dev.type == "cuda":
                    eng = _h2d_engine(dev.index if dev.index is not None else 0)
                    if eng is not None and param.is_contiguous():
                        src = param if new_dtype is None or not torch.is_floating_point(param) else param.to(new_dtype)
                        old = recursive_getattr(model, param_name)
                        if new_dtype is None and torch.is_floating_point(src) and old.dtype != src.dtype:
                            src = src.to(old.dtype)
                        dst = torch.empty(src.shape, dtype=src.dtype, device=dev)
                        eng.copy(src.contiguous(), dst)
                        engines_used.add(eng)
                        set_module_tensor_to_device(model, param_name, dev, value=dst, dtype=None, clear_cache=False)
                        continue
                set_module_tensor_to_device(model, param_name, param_device, value=param, dtype=new_dtype, clear_cache=False)
        del loaded
        gc.collect()
    for eng in engines_used:
        eng.wait_on_current_stream()
    if len(unexpected_keys) > 0:
        logger.warning(f"Some weights of the model checkpoint at {checkpoint} were not used when initializing {model.__class__.__name__}: {sorted(unexpected_keys)[:10]}")
    save_offload_index(offload_index, offload_folder)
    if offload_state_dict:
        _load_offloaded_weights(model, state_dict_index, state_dict_folder)
        import shutil

        shutil.rmtree(state_dict_folder)
    retie_parameters(model, tied_params)


def _load_offloaded_weights(model, index, offload_folder):
    if index is None or len(index) == 0:
        return
    for param_name, metadata in index.items():
        tensor_file = os.path.join(offload_folder, f"{param_name}.dat")
        weight = load_offloaded_weight(tensor_file, metadata)
        set_module_tensor_to_device(model, param_name, "cpu", value=weight)


# ---------------------------------------------------------------------------------------------------- dispatch
def dispatch_model(
    model: nn.Module,
    device_map: dict,
    main_device: Optional[torch.device] = None,
    state_dict: Optional[dict] = None,
    offload_dir: Optional[Union[str, os.PathLike]] = None,
    offload_index: Optional[dict] = None,
    offload_buffers: bool = False,
    skip_keys=None,
    preload_module_classes=None,
    force_hooks: bool = False,
):
    """Place `model` per `device_map` and attach hooks moving activations between devices (a naive pipeline) and
    streaming offloaded weights in (with async prefetch on MI355X)."""
    check_device_map(model, device_map)
    if (len(set(device_map.values())) > 1) or force_hooks:
        if main_device is None:
            if set(device_map.values()) == {"cpu"} or set(device_map.values()) == {"cpu", "disk"}:
                main_device = "cpu"
            else:
                main_device = [d for d in device_map.values() if d not in ["cpu", "disk"]][0]
        if main_device != "cpu":
            cpu_modules = [name for name, device in device_map.items() if device == "cpu"]
            if state_dict is None and len(cpu_modules) > 0:
                state_dict = extract_submodules_state_dict(model.state_dict(), cpu_modules)
        disk_modules = [name for name, device in device_map.items() if device == "disk"]
        if offload_dir is None and offload_index is None and len(disk_modules) > 0:
            raise ValueError(
                "We need an `offload_dir` to dispatch this model according to this `device_map`, the following submodules "
                f"need to be offloaded: {', '.join(disk_modules)}."
            )
        if len(disk_modules) > 0 and offload_index is None and (
            not os.path.isdir(offload_dir) or not os.path.isfile(os.path.join(offload_dir, "index.json"))
        ):
            disk_state_dict = extract_submodules_state_dict(model.state_dict(), disk_modules)
            offload_state_dict(offload_dir, disk_state_dict)
        execution_device = {name: main_device if device in ["cpu", "disk"] else device for name, device in device_map.items()}
        execution_device[""] = main_device
        offloaded_devices = ["disk"] if main_device == "cpu" else ["cpu", "disk"]
        offload = {name: device in offloaded_devices for name, device in device_map.items()}
        save_folder = offload_dir if len(disk_modules) > 0 else None
        if state_dict is not None or save_folder is not None or offload_index is not None:
            device = main_device if offload_index is not None else None
            weights_map = OffloadedWeightsLoader(state_dict=state_dict, save_folder=save_folder, index=offload_index, device=device)
        else:
            weights_map = None
        tied_params = find_tied_parameters(model)
        tied_params_map = {}
        for group in tied_params:
            for param_name in group:
                data_ptr = recursive_getattr(model, param_name).data_ptr()
                tied_params_map[data_ptr] = {}
        attach_align_device_hook_on_blocks(
            model,
            execution_device=execution_device,
            offload=offload,
            offload_buffers=offload_buffers,
            weights_map=weights_map,
            skip_keys=skip_keys,
            preload_module_classes=preload_module_classes,
            tied_params_map=tied_params_map,
        )
        offloaded_devices_str = " and ".join([device for device in set(device_map.values()) if device in ("cpu", "disk")])
        if len(offloaded_devices_str) > 0:
            logger.warning(f"Some parameters are on the meta device because they were offloaded to the {offloaded_devices_str}.")
        retie_parameters(model, tied_params)

        def add_warning(fn, model):
            import functools

            @functools.wraps(fn)
            def wrapper(*args, **kwargs):
                warning_msg = "You shouldn't move a model that is dispatched using accelerate hooks."
                if str(fn.__name__) == "to":
                    to_device = torch._C._nn._parse_to(*args, **kwargs)[0]
                    if to_device is not None:
                        logger.warning(warning_msg)
                else:
                    logger.warning(warning_msg)
                for param in model.parameters():
                    if param.device == torch.device("meta"):
                        raise RuntimeError("You can't move a model that has some modules offloaded to cpu or disk.")
                return fn(*args, **kwargs)

            return wrapper

        model.to = add_warning(model.to, model)
        model.cuda = add_warning(model.cuda, model)
    else:
        device = list(device_map.values())[0]
        if device != "disk":
            model.to(_device(device) if not isinstance(device, str) or device not in ("cpu",) else device)
        else:
            raise ValueError("You are trying to offload the whole model to the disk. Please use the `disk_offload` function instead.")
    model.hf_device_map = dict(device_map)
    return model


def cpu_offload(model: nn.Module, execution_device=None, offload_buffers: bool = False, state_dict=None, preload_module_classes=None):
    """Keep all weights on CPU; upload each module's weights to `execution_device` just for its forward."""
    if execution_device is None:
        execution_device = next(iter(model.parameters())).device
    if state_dict is None:
        state_dict = {n: p.to("cpu") for n, p in model.state_dict().items()}
    add_hook_to_module(model, AlignDevicesHook(io_same_device=True), append=True)
    attach_align_device_hook(
        model,
        execution_device=execution_device,
        offload=True,
        offload_buffers=offload_buffers,
        weights_map=state_dict,
        preload_module_classes=preload_module_classes,
    )
    return model


def cpu_offload_with_hook(model: nn.Module, execution_device=None, prev_module_hook: Optional[UserCpuOffloadHook] = None):
    """Move the whole model to the device on forward and leave it there until `hook.offload()` (pipelines of models)."""
    hook = CpuOffload(execution_device=execution_device, prev_module_hook=prev_module_hook)
    add_hook_to_module(model, hook, append=True)
    user_hook = UserCpuOffloadHook(model, hook)
    return model, user_hook


def disk_offload(model: nn.Module, offload_dir, execution_device=None, offload_buffers: bool = False, preload_module_classes=None):
    if not os.path.isdir(offload_dir) or not os.path.isfile(os.path.join(offload_dir, "index.json")):
        offload_state_dict(offload_dir, model.state_dict())
    if execution_device is None:
        execution_device = next(iter(model.parameters())).device
    weights_map = OffloadedWeightsLoader(save_folder=offload_dir)
    add_hook_to_module(model, AlignDevicesHook(io_same_device=True), append=True)
    attach_align_device_hook(
        model,
        execution_device=execution_device,
        offload=True,
        offload_buffers=offload_buffers,
        weights_map=weights_map,
        preload_module_classes=preload_module_classes,
    )
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
    """Load a checkpoint into a (meta-initialised) model and dispatch it (`device_map` "auto" / "balanced" /
    "balanced_low_0" / "sequential" / explicit dict)."""
    if isinstance(device_map, str) and device_map not in ["auto", "balanced", "balanced_low_0", "sequential"]:
        raise ValueError("If passing a string for `device_map`, please choose 'auto', 'balanced', 'balanced_low_0' or 'sequential'.")
    if no_split_module_classes is None:
        no_split_module_classes = getattr(model, "_no_split_modules", None)
    if isinstance(device_map, str):
        if device_map != "sequential":
            max_memory = get_balanced_memory(
                model,
                max_memory=max_memory,
                no_split_module_classes=no_split_module_classes,
                dtype=dtype,
                low_zero=(device_map == "balanced_low_0"),
            )
        device_map = infer_auto_device_map(
            model,
            max_memory=max_memory,
            no_split_module_classes=no_split_module_classes,
            dtype=dtype,
            offload_buffers=offload_buffers,
        )
    if offload_state_dict is None and device_map is not None and "disk" in device_map.values():
        offload_state_dict = True
    load_checkpoint_in_model(
        model,
        checkpoint,
        device_map=device_map,
        offload_folder=offload_folder,
        dtype=dtype,
        offload_state_dict=bool(offload_state_dict),
        offload_buffers=offload_buffers,
        strict=strict,
        full_state_dict=full_state_dict,
        broadcast_from_rank0=broadcast_from_rank0,
    )
    if device_map is None:
        return model
    return dispatch_model(
        model,
        device_map=device_map,
        offload_dir=offload_folder,
        offload_buffers=offload_buffers,
        skip_keys=skip_keys,
        preload_module_classes=preload_module_classes,
        force_hooks=force_hooks,
    )


def attach_layerwise_casting_hooks(
    module: nn.Module,
    storage_dtype: torch.dtype,
    compute_dtype: torch.dtype,
    skip_modules_pattern=None,
    skip_modules_classes=None,
    non_blocking: bool = False,
):
    """Store weights in `storage_dtype` (e.g. fp8 e4m3) and compute in `compute_dtype` (reference big_modeling.py:654-750)."""
    _SUPPORTED = (nn.Linear, nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.Embedding, nn.LayerNorm, nn.GroupNorm)
    if skip_modules_pattern is None:
        skip_modules_pattern = ("pos_embed", "patch_embed", "norm", "^proj_in$", "^proj_out$")
    skip_modules_classes = tuple(skip_modules_classes or ())

    def _apply(m, name):
        should_skip = (skip_modules_classes and isinstance(m, skip_modules_classes)) or any(re.search(p, name) for p in skip_modules_pattern)
        if should_skip:
            return
        if isinstance(m, _SUPPORTED):
            add_hook_to_module(m, LayerwiseCastingHook(storage_dtype, compute_dtype, non_blocking), append=True)
            return
        for child_name, child in m.named_children():
            _apply(child, f"{name}.{child_name}" if name else child_name)

    _apply(module, "")


def has_offloaded_params(module: nn.Module) -> bool:
    from .hooks import AlignDevicesHook as _A

    return hasattr(module, "_hf_hook") and isinstance(module._hf_hook, _A) and module._hf_hook.offload


@contextlib.contextmanager
def align_module_device(module: nn.Module, execution_device=None):
    """Temporarily materialise an offloaded module's weights on `execution_device`."""
    if has_offloaded_params(module):
        if execution_device is not None:
            original_device = module._hf_hook.execution_device
            module._hf_hook.execution_device = execution_device
        try:
            module._hf_hook.pre_forward(module)
            yield
        finally:
            module._hf_hook.post_forward(module, None)
            if execution_device is not None:
                module._hf_hook.execution_device = original_device
    elif execution_device is not None:
        devices = {name: param.device for name, param in module.named_parameters(recurse=False)}
        try:
            for name in devices:
                set_module_tensor_to_device(module, name, execution_device)
            yield
        finally:
            for name, device in devices.items():
                set_module_tensor_to_device(module, name, device)
    else:
        yield
