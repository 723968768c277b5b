"""Device-map planning for big-model inference: which submodule lives on which GPU, on the host, or on disk.

Public functions keep the reference's names and results (`/root/reference/src/accelerate/utils/modeling.py:744-1583`:
`get_max_memory`, `get_balanced_memory`, `get_max_layer_size`, `calculate_maximum_sizes`, `clean_device_map`,
`infer_auto_device_map` with `fallback_allocation`, `check_device_map`); the placement results are pinned against the
installed upstream `accelerate` by `tests/test_device_map_parity.py` over a grid of models and budgets.

The planner itself is one object, `DeviceMapPlanner`, that walks a work list of *placement candidates* (a direct
parameter/buffer or a submodule, by dotted name) in module order and fills devices greedily: GPU 0, 1, ... then the
host, then disk. On the devices a spilled layer would be streamed back to (the first GPU and the host) it keeps room
for the largest layer still to be placed; a candidate that does not fit is split into its direct tensors and children
unless it is a no-split class; parameters tied across candidates are placed together. With `fallback_allocation` a
device that would otherwise stay empty receives the first candidate (searched depth first through splittable modules)
that fits its budget.

MI355X: the default budget of a GPU is its free HBM from `torch.cuda.mem_get_info` (288 GB per MI355X), so an 8-GPU
node holds a 70B bf16 model (~140 GB) on its first GPU alone without offload.
"""

from __future__ import annotations

import logging
import warnings
from collections import OrderedDict
from typing import Optional, Union

import torch
import torch.nn as nn

from .modeling import compute_module_sizes, compute_module_total_buffer_size, convert_file_size_to_int

logger = logging.getLogger(__name__)

_HOST_KEYS = ("mps", "cpu", "disk")


# ----------------------------------------------------------------------------------------------------- budgets
def get_max_memory(max_memory: Optional[dict] = None) -> dict:
    """Budget per device: given sizes are normalised to bytes and ordered GPUs first (ascending), then mps / cpu /
    disk; with nothing given, every visible GPU's free HBM and the host's available RAM."""
    import psutil

    if max_memory is None:
        budget = {}
        if torch.cuda.is_available():
            for idx in range(torch.cuda.device_count()):
                try:
                    torch.zeros(1, device=idx)
                    budget[idx] = torch.cuda.mem_get_info(idx)[0]
                except Exception:  # a device that cannot be touched is simply not offered
                    logger.info(f"GPU {idx} is not usable; skipping it in the memory budget.")
        budget["cpu"] = psutil.virtual_memory().available
        return budget
    sized = {k: convert_file_size_to_int(v) if isinstance(v, str) else v for k, v in max_memory.items()}
    visible = torch.cuda.device_count() if torch.cuda.is_available() else 0
    gpu_ids = sorted(k for k in sized if isinstance(k, int))
    for idx in gpu_ids:
        if not 0 <= idx < visible:
            logger.warning(f"Device {idx} is not available, available devices are {list(range(visible))}")
    unknown = [k for k in sized if not isinstance(k, int) and k not in _HOST_KEYS]
    if unknown:
        raise ValueError(
            f"Device {unknown[0]} is not recognized, available devices are integers(for GPU/XPU), 'mps', 'cpu' and 'disk'"
        )
    return {k: sized[k] for k in gpu_ids + [h for h in _HOST_KEYS if h in sized]}


def get_module_leaves(module_sizes: dict) -> list:
    """Names (in `module_sizes` order) that are nobody's parent."""
    parents = {name.rsplit(".", 1)[0] for name in module_sizes if name and "." in name}
    return [name for name in module_sizes if name and name not in parents]


def _class_names(classes) -> list:
    """`no_split_module_classes` as a list of class names: None, one name, or any collection of names (transformers 5
    declares `_no_split_modules` as a set)."""
    if classes is None:
        return []
    if isinstance(classes, str):
        return [classes]
    return sorted(classes) if isinstance(classes, (set, frozenset)) else list(classes)


def _class_sizes(model: nn.Module, module_sizes: dict, classes: list) -> dict:
    """Size of the first module of each class in `classes`, in `module_sizes` order."""
    wanted, found = set(classes), {}
    for name in module_sizes:
        if not name:
            continue
        cls = model.get_submodule(name).__class__.__name__ if _is_module_path(model, name) else None
        if cls in wanted and cls not in found:
            found[cls] = module_sizes[name]
            if len(found) == len(wanted):
                break
    return found


def _is_module_path(model: nn.Module, name: str) -> bool:
    try:
        model.get_submodule(name)
        return True
    except AttributeError:
        return False


def get_balanced_memory(
    model: nn.Module,
    max_memory: Optional[dict] = None,
    no_split_module_classes: Optional[list] = None,
    dtype=None,
    special_dtypes=None,
    low_zero: bool = False,
) -> dict:
    """Per-GPU budgets that spread the model evenly over the GPUs (the last GPU keeps its full budget as slack).

    Each GPU but the last is capped at model_size / n_gpus plus a margin of 1.25 x max(largest no-split block, mean
    size of the innermost *modules* — leaf tensors excluded); `low_zero` keeps GPU 0 as empty as the rest allows
    (generation buffers live there)."""
    user_budget = max_memory is not None
    budget = get_max_memory(max_memory)
    gpus = sorted(k for k, v in budget.items() if isinstance(k, int) and v > 0)
    if not gpus:
        return budget
    if len(gpus) == 1:
        low_zero = False
        if not user_budget:  # keep 10 % of the only GPU for activations
            first = next(k for k in budget if isinstance(k, int))
            budget[first] *= 0.9
    sizes = compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes)
    share = sizes[""] // (len(gpus) - 1 if low_zero else len(gpus))

    no_split_module_classes = _class_names(no_split_module_classes)
    block = max(_class_sizes(model, sizes, no_split_module_classes).values(), default=0)
    # innermost modules: drop the leaf tensors first, then the leaves of what remains are the last modules
    tensor_leaves = set(get_module_leaves(sizes))
    module_only = {n: v for n, v in sizes.items() if n not in tensor_leaves}
    inner = get_module_leaves(module_only)
    mean_inner = int(sum(module_only[n] for n in inner) / max(len(inner), 1))
    share += int(1.25 * max(block, mean_inner))

    for idx in gpus[:-1]:
        budget[idx] = min(budget[0] if (low_zero and idx == 0) else share, budget[idx])
    if low_zero:
        rest = sum(budget[i] for i in range(1, len(gpus)))
        budget[0] = min(max(0, sizes[""] - rest), budget[0])
    return budget


# ----------------------------------------------------------------------------------------------------- layer sizes
def _splittable(obj, no_split: list) -> bool:
    return isinstance(obj, nn.Module) and obj.__class__.__name__ not in no_split and next(obj.children(), None) is not None


def _expand(name: str, obj: nn.Module) -> list:
    """A module's placement candidates: its direct parameters, then its children (buffers stay with the module)."""
    return [(f"{name}.{n}", p) for n, p in obj.named_parameters(recurse=False)] + [
        (f"{name}.{n}", c) for n, c in obj.named_children()
    ]


def get_max_layer_size(modules: list, module_sizes: dict, no_split_module_classes: list):
    """(size, names) of the largest *layer* reachable from `modules`: a layer is a module without children (or a
    tensor), or a module of a no-split class. Depth-first in module order; ties keep discovery order."""
    best, names = 0, []
    stack = list(reversed(modules))
    while stack:
        name, obj = stack.pop()
        kids = list(obj.named_children()) if isinstance(obj, nn.Module) else []
        if kids and obj.__class__.__name__ not in no_split_module_classes:
            stack.extend(reversed([(f"{name}.{n}", c) for n, c in kids]))
            continue
        size = module_sizes[name]
        if size > best:
            best, names = size, [name]
        elif size == best:
            names.append(name)
    return best, names


def _top_level(model: nn.Module) -> list:
    return list(model.named_parameters(recurse=False)) + list(model.named_children()) + list(model.named_buffers(recurse=False))


def calculate_maximum_sizes(model: nn.Module):
    """(total size, (largest layer size, its names)) with the model's own `_no_split_modules`."""
    sizes = compute_module_sizes(model)
    no_split = getattr(model, "_no_split_modules", None) or []
    return sizes[""], get_max_layer_size(_top_level(model), sizes, no_split)


def clean_device_map(device_map: dict, module_name: str = "") -> dict:
    """Merge every subtree whose entries all share one device into a single entry for the subtree's root."""
    prefix = f"{module_name}." if module_name else ""
    entries = [k for k in device_map if k.startswith(prefix)]
    devices = {device_map[k] for k in entries}
    if len(entries) > 1 and len(devices) == 1:
        dev = device_map[entries[0]]
        for k in entries:
            del device_map[k]
        device_map[module_name] = dev
    depth = len(module_name.split(".")) + 1 if module_name else 1
    children = {".".join(k.split(".")[:depth]) for k in device_map if k.startswith(prefix) and len(k) > len(module_name)}
    for child in children:
        clean_device_map(device_map, child)
    return device_map


def find_tied_parameters(model: nn.Module, **kwargs) -> list:
    """Groups of parameter names that share one Parameter (e.g. tied embedding / LM head), each sorted; groups in the
    order their first name is registered."""
    first_name = {}
    groups = OrderedDict()
    for name, p in model.named_parameters(remove_duplicate=False):
        owner = first_name.setdefault(id(p), name)
        if owner != name:
            groups.setdefault(owner, {owner}).add(name)
    return [sorted(g) for g in groups.values()]


def _tied_outside(name: str, ties: list) -> list:
    """Names of parameters tied to something inside `name` but living outside it (a dotted-boundary test, so
    `lin.weight_extra` is outside `lin.weight`)."""
    inside = lambda p: (name + ".") in (p + ".")  # noqa: E731
    out = []
    for group in ties:
        if any(inside(p) for p in group) and not all(inside(p) for p in group):
            out.extend(p for p in group if not inside(p))
    return out


# ----------------------------------------------------------------------------------------------------- planner
class DeviceMapPlanner:
    """Greedy placement of a model's submodules over a device budget (see module docstring)."""

    def __init__(self, model, max_memory=None, no_split_module_classes=None, dtype=None, special_dtypes=None,
                 verbose=False, offload_buffers=False, fallback_allocation=False):
        self.model = model
        self.budget = get_max_memory(max_memory)
        self.no_split = _class_names(no_split_module_classes)
        self.devices = list(self.budget) + ([] if "disk" in self.budget else ["disk"])
        gpus = [d for d in self.devices if d not in ("cpu", "disk")]
        self.gpus = gpus
        # devices that must keep room to stream back the largest offloaded layer
        self.streaming_targets = {"mps"} if "mps" in gpus else ({gpus[0], "cpu"} if gpus else {"cpu"})
        self.dtype, self.special_dtypes = dtype, special_dtypes
        self.sizes = compute_module_sizes(model, dtype=dtype, special_dtypes=special_dtypes)
        self.ties = find_tied_parameters(model)
        self.verbose = verbose
        self.offload_buffers = offload_buffers
        self.fallback = fallback_allocation
        self.work = _top_level(model)
        self.used = {d: 0 for d in self.devices}
        self.buffers_on = {}
        self.unmet = {}
        self.cursor = 0
        self.plan = OrderedDict()

    # -- helpers --------------------------------------------------------------------------------------------
    def _say(self, msg):
        if self.verbose:
            print(msg)

    def _largest(self):
        return get_max_layer_size([(n, m) for n, m in self.work if isinstance(m, nn.Module)], self.sizes, self.no_split)

    def _with_ties(self, name: str, size: int, outside: list):
        """Size of `name` plus the work-list entries holding its tied partners (each counted without the shared
        tensor), and those entries."""
        total, names, objs = size, [], []
        for p in outside:
            hit = next(((n, o) for n, o in self.work if p.startswith(n + ".")), None)
            if hit is None:
                continue
            names.append(hit[0])
            objs.append(hit[1])
            total += self.sizes[hit[0]] - self.sizes[p]
        return total, names, objs

    def _first_fit(self, limit):
        """Fallback: the first candidate in depth-first order (splittable modules opened in place) whose size with
        ties is <= `limit`; the work list is re-expanded along its path and the candidate taken out of it."""
        try:
            limit = convert_file_size_to_int(limit)
        except ValueError:
            return None
        stack = list(reversed(self.work))
        found = None
        while stack:
            name, obj = stack.pop()
            size = self._with_ties_in(name, self.sizes[name], _tied_outside(name, self.ties), list(reversed(stack)))
            if size <= limit:
                found = name
                break
            if _splittable(obj, self.no_split):
                stack.extend(reversed(_expand(name, obj)))
        if found is None:
            return None
        parts = found.split(".")
        for depth in range(1, len(parts)):  # open every ancestor of `found` that is still one work-list entry
            parent = ".".join(parts[:depth])
            idx = next((i for i, (n, _) in enumerate(self.work) if n == parent), None)
            if idx is not None:
                self.work[idx : idx + 1] = _expand(parent, self.work[idx][1])
        idx = next(i for i, (n, _) in enumerate(self.work) if n == found)
        return self.work.pop(idx)

    def _with_ties_in(self, name, size, outside, pool):
        total = size
        for p in outside:
            hit = next((n for n, _ in pool if p.startswith(n + ".")), None)
            if hit is not None:
                total += self.sizes[hit] - self.sizes[p]
        return total

    # -- main loop ------------------------------------------------------------------------------------------
    def run(self) -> OrderedDict:
        largest, largest_names = get_max_layer_size(self.work, self.sizes, self.no_split)
        while self.work:
            name, obj = self.work.pop(0)
            self._say(f"\nTreating module {name}.")
            largest_names = [n for n in largest_names if n != name and not n.startswith(name + ".")]
            if not largest_names:
                largest, largest_names = self._largest()
            size = self.sizes[name]
            outside = _tied_outside(name, self.ties)
            dev = self.devices[self.cursor]
            cap = None if dev == "disk" else self.budget[dev]
            reserved = 0
            if dev in self.streaming_targets:
                cap -= largest
                reserved = largest
            total, tied_names, tied_objs = self._with_ties(name, size, outside)

            if cap is None or self.used[dev] + total <= cap:
                self._say(f"Putting {name} on {dev}.")
                self.used[dev] += total
                self.plan[name] = dev
                for t in tied_names:
                    self.work = [(n, o) for n, o in self.work if n != t]
                    self.plan[t] = dev
                if not self.offload_buffers and isinstance(obj, nn.Module):
                    self.buffers_on[dev] = self.buffers_on.get(dev, 0) + compute_module_total_buffer_size(
                        obj, dtype=self.dtype, special_dtypes=self.special_dtypes)
                continue

            if outside and self.used[dev] + size <= cap:
                # the module alone fits: try opening one of its tied partners instead of moving on
                opened = False
                for t_name, t_obj in zip(tied_names, tied_objs):
                    if not _splittable(t_obj, self.no_split):
                        continue
                    self._say(f"Splitting {t_name}.")
                    idx = next(i for i, (n, _) in enumerate(self.work) if n == t_name)
                    self.work = [(name, obj)] + self.work[:idx] + _expand(t_name, t_obj) + self.work[idx + 1 :]
                    largest, largest_names = self._largest()
                    opened = True
                    break
                if opened:
                    continue

            if self.used[dev] + size >= cap:
                if _splittable(obj, self.no_split):
                    self._say(f"Splitting {name}.")
                    self.work = _expand(name, obj) + self.work
                    largest, largest_names = self._largest()
                    continue

            if self.used[dev] == 0 and self.fallback and dev != "disk":
                hit = self._first_fit(self.budget[dev] - max(largest, total))
                if hit is not None:  # place the found candidate next, then retry the current one
                    self.work = [hit, (name, obj)] + self.work
                    continue

            if self.used[dev] == 0:
                self.unmet[dev] = total + reserved
            self.used[dev] += reserved
            self.cursor += 1
            self.work.insert(0, (name, obj))
        return self.plan


def infer_auto_device_map(
    model: nn.Module,
    max_memory: Optional[dict] = None,
    no_split_module_classes: Optional[list] = None,
    dtype=None,
    special_dtypes=None,
    verbose: bool = False,
    clean_result: bool = True,
    offload_buffers: bool = False,
    fallback_allocation: bool = False,
) -> OrderedDict:
    """Device map filling GPUs in order, then the host, then disk (see `DeviceMapPlanner`)."""
    planner = DeviceMapPlanner(model, max_memory, no_split_module_classes, dtype, special_dtypes, verbose,
                               offload_buffers, fallback_allocation)
    device_map = planner.run()
    if clean_result:
        device_map = clean_device_map(device_map)
    used = {d: m for d, m in planner.used.items() if m > 0}
    offloaded_buffers = planner.buffers_on.get("cpu", 0) + planner.buffers_on.get("disk", 0)
    if offloaded_buffers > 0 and not offload_buffers and planner.gpus:
        fits = any(mem >= offloaded_buffers + used.get(d, 0) for d, mem in planner.budget.items() if d not in ("cpu", "disk"))
        if not fits:
            warnings.warn(
                f"Current model requires {offloaded_buffers} bytes of buffer for offloaded layers, which seems does not "
                "fit any GPU's remaining memory. If you are experiencing a OOM later, please consider using "
                "offload_buffers=True."
            )
    if planner.unmet:
        detail = "\n".join(f"  - {d}: {m} bytes required" for d, m in planner.unmet.items())
        logger.info(f"No module could be assigned to these devices (insufficient memory):\n{detail}")
    return device_map


def check_device_map(model: nn.Module, device_map: dict):
    """Raise if some parameter/buffer of `model` is covered by no entry of `device_map`."""
    if "" in device_map:
        return
    covered = lambda t: any(t == k or t.startswith(k + ".") for k in device_map)  # noqa: E731
    missing = [name for name in model.state_dict() if not covered(name)]
    if missing:
        raise ValueError(f"The device_map provided does not give any device for the following parameters: {', '.join(missing)}")
