"""Collective and nested-structure operations (L2 of the layer map).

Parity: `/root/reference/src/accelerate/utils/operations.py:85-871` — same function names and semantics
(`gather`, `gather_object`, `broadcast`, `broadcast_object_list`, `reduce`, `pad_across_processes`,
`send_to_device`, `concatenate`, `slice_tensors`, `find_batch_size`, `convert_to_fp32`, debug-mode
`verify_operation`).

MI355X-specific design:
* On GPU every tensor collective goes to RCCL (`torch.distributed` "nccl" backend) on the current HIP
  stream. Each RCCL launch costs tens of microseconds, so nested structures of tensors are **coalesced**:
  `reduce`/`gather`/`broadcast` of a dict/list of same-dtype tensors flatten everything into one buffer
  and issue ONE collective (the reference issues one per leaf).
* Shape exchange for `pad_across_processes` / `copy_tensor_to_devices` all-gathers a tiny int64 vector
  instead of the reference's 4 MB int32 all-reduce (`operations.py:496-535`).
"""

from __future__ import annotations

import pickle
from collections.abc import Mapping
from contextlib import contextmanager, nullcontext
from functools import update_wrapper, wraps
from typing import Any

import torch

from .dataclasses import DistributedType, TensorInformation
from .fault_tolerance import record_collective


def PartialState():  # noqa: N802 - lazy accessor (utils is imported by state.py; avoid the import cycle)
    from ..state import PartialState as _PartialState

    return _PartialState()


class DistributedOperationException(Exception):
    """Raised (in debug mode) when ranks call a collective with mismatched shapes instead of hanging RCCL."""


def is_torch_tensor(tensor):
    return isinstance(tensor, torch.Tensor)


def is_tensor_information(tensor_info):
    return isinstance(tensor_info, TensorInformation)


def is_namedtuple(data):
    return isinstance(data, tuple) and hasattr(data, "_asdict") and hasattr(data, "_fields")


def honor_type(obj, generator):
    """Rebuild `obj`'s container type from `generator` (namedtuples need positional construction)."""
    items = list(generator)
    return type(obj)(*items) if is_namedtuple(obj) else type(obj)(items)


def _tree_map(leaf_fn, data, is_leaf, on_other=None):
    """Map `leaf_fn` over the leaves of a list / tuple / mapping tree, keeping every container's own type. Values that
    are neither containers nor leaves go through `on_other` (returned unchanged by default)."""
    if isinstance(data, (list, tuple)):
        return honor_type(data, (_tree_map(leaf_fn, x, is_leaf, on_other) for x in data))
    if isinstance(data, Mapping):
        return type(data)({k: _tree_map(leaf_fn, v, is_leaf, on_other) for k, v in data.items()})
    if is_leaf(data):
        return leaf_fn(data)
    return on_other(data) if on_other is not None else data


def _tree_first(data, pick):
    """First non-None `pick(leaf)` in depth-first order over lists / tuples / mappings (None if there is none)."""
    if isinstance(data, Mapping):
        data = list(data.values())
    if isinstance(data, (list, tuple)):
        for x in data:
            got = _tree_first(x, pick)
            if got is not None:
                return got
        return None
    return pick(data)


def recursively_apply(func, data, *args, test_type=is_torch_tensor, error_on_other_type=False, **kwargs):
    """Apply `func(leaf, *args, **kwargs)` to every leaf of a nested list / tuple / dict that passes `test_type`;
    other leaves are kept, or rejected with `error_on_other_type`."""

    def reject(x):
        raise TypeError(f"Unsupported types ({type(x)}) passed to `{func.__name__}`. Only nested list/tuple/dicts of "
                        f"objects that are valid for `{test_type.__name__}` should be passed.")

    return _tree_map(lambda x: func(x, *args, **kwargs), data, test_type, reject if error_on_other_type else None)


def send_to_device(tensor, device, non_blocking=False, skip_keys=None):
    """Move every tensor (and any object with a `.to`) in a nested structure to `device`; mapping entries named in
    `skip_keys` stay where they are. Objects whose `.to` takes no `non_blocking` are moved synchronously."""
    if hasattr(tensor, "to"):  # tensors, modules, BatchEncoding-like objects: the object moves itself
        try:
            return tensor.to(device, non_blocking=non_blocking)
        except TypeError:
            return tensor.to(device)
    skip = {skip_keys} if isinstance(skip_keys, str) else set(skip_keys or ())
    if isinstance(tensor, Mapping):
        return type(tensor)({k: v if k in skip else send_to_device(v, device, non_blocking, skip_keys)
                             for k, v in tensor.items()})
    if isinstance(tensor, (list, tuple)):
        return honor_type(tensor, (send_to_device(v, device, non_blocking, skip_keys) for v in tensor))
    return tensor


def get_data_structure(data):
    """The same structure with every tensor replaced by its `TensorInformation` (shape, dtype)."""
    return _tree_map(lambda t: TensorInformation(shape=t.shape, dtype=t.dtype), data, is_torch_tensor)


def get_shape(data):
    return _tree_map(lambda t: list(t.shape), data, is_torch_tensor)


def initialize_tensors(data_structure):
    """Uninitialised tensors for a structure of `TensorInformation` (the receive side of a structure broadcast)."""
    return _tree_map(lambda info: torch.empty(*info.shape, dtype=info.dtype), data_structure, is_tensor_information)


def find_batch_size(data):
    """Size of dim 0 of the first tensor in `data` (depth first)."""
    if isinstance(data, (tuple, list, Mapping)) and len(data) == 0:
        raise ValueError(f"Cannot find the batch size from empty {type(data)}.")
    while isinstance(data, (tuple, list, Mapping)):
        data = next(iter(data.values())) if isinstance(data, Mapping) else data[0]
        if isinstance(data, (tuple, list, Mapping)) and len(data) == 0:
            raise ValueError(f"Cannot find the batch size from empty {type(data)}.")
    if not isinstance(data, torch.Tensor):
        raise TypeError(f"Can only find the batch size of tensors but got {type(data)}.")
    return data.shape[0]


def ignorant_find_batch_size(data):
    try:
        return find_batch_size(data)
    except (ValueError, TypeError):
        return None


def listify(data):
    """Tensors -> Python lists / scalars (bf16 through fp32, which `tolist` needs)."""

    def to_list(t):
        t = t.detach().cpu()
        return (t.float() if t.dtype == torch.bfloat16 else t).tolist()

    return _tree_map(to_list, data, is_torch_tensor)


# ------------------------------------------------------------------------------------------------------
# Debug-mode cross-rank verification (enabled by `launch --debug` / ACCELERATE_DEBUG_MODE)
# ------------------------------------------------------------------------------------------------------
def _shape_report(name: str, per_rank: list) -> str:
    rows = "\n".join(f"  - Process {i}: {shape}" for i, shape in enumerate(per_rank))
    return (f"Cannot apply desired operation due to shape mismatches. All shapes across devices must be valid.\n\n"
            f"Operation: `{name}`\nInput shapes:\n{rows}")


def verify_operation(function):
    """Debug mode: before the collective, every rank's input shapes are all-gathered (one object gather) and a
    mismatch raises `DistributedOperationException` on all ranks — instead of RCCL hanging, or silently combining
    differently shaped buffers. Also refuses inputs on another device type than the process's. Outside debug mode
    (and in single-process runs) it is a plain call. Reference semantics: utils/operations.py:355-396."""

    name = f"{function.__module__}.{function.__name__}"

    @wraps(function)
    def wrapper(*args, **kwargs):
        state = PartialState()
        if not state.debug or state.distributed_type == DistributedType.NO:
            return function(*args, **kwargs)
        data = kwargs["tensor"] if "tensor" in kwargs else args[0]
        dev = find_device(data)
        if dev is not None and dev.type != state.device.type:
            raise DistributedOperationException(
                f"One or more of the tensors passed to {name} were not on the {dev.type} while the `Accelerator` is "
                f"configured for {state.device.type}. Please move it to the {state.device.type} before calling {name}.")
        per_rank = gather_object([get_shape(data)])
        if per_rank[0] is not None and any(s != per_rank[0] for s in per_rank[1:]):
            raise DistributedOperationException(_shape_report(name, per_rank))
        return function(*args, **kwargs)

    return wrapper


def chained_operation(function):
    """Calls made through another collective re-raise a debug-mode mismatch under the outer operation's name."""
    name = f"{function.__module__}.{function.__name__}"

    @wraps(function)
    def wrapper(*args, **kwargs):
        try:
            return function(*args, **kwargs)
        except DistributedOperationException as exc:
            raise DistributedOperationException(
                f"Error found while calling `{name}`. Please see the earlier error for more details.") from exc

    return wrapper


def find_device(data):
    """Device of the first tensor in a nested structure (None if it holds no tensor)."""
    return _tree_first(data, lambda x: x.device if isinstance(x, torch.Tensor) else None)


# ------------------------------------------------------------------------------------------------------
# Coalescing helpers: one collective for a whole nested structure
# ------------------------------------------------------------------------------------------------------
def _leaves(data, out):
    if isinstance(data, (tuple, list)):
        for d in data:
            _leaves(d, out)
    elif isinstance(data, Mapping):
        for v in data.values():
            _leaves(v, out)
    elif isinstance(data, torch.Tensor):
        out.append(data)
    return out


def _rebuild(data, it):
    if isinstance(data, (tuple, list)):
        return honor_type(data, (_rebuild(d, it) for d in data))
    elif isinstance(data, Mapping):
        return type(data)({k: _rebuild(v, it) for k, v in data.items()})
    elif isinstance(data, torch.Tensor):
        return next(it)
    return data


def _coalescable(leaves):
    if len(leaves) < 2:
        return False
    dev, dt = leaves[0].device, leaves[0].dtype
    return all(t.device == dev and t.dtype == dt for t in leaves)


# ------------------------------------------------------------------------------------------------------
# gather
# ------------------------------------------------------------------------------------------------------
def _gpu_gather_one(tensor: torch.Tensor) -> torch.Tensor:
    state = PartialState()
    if tensor.ndim == 0:
        tensor = tensor.clone()[None]
    if not tensor.is_contiguous():
        tensor = tensor.contiguous()
    if tensor.is_cuda and state.backend is not None and state.backend.startswith("gloo"):  # gloo: host-only tensor forms
        outs = [torch.empty_like(tensor) for _ in range(state.num_processes)]
        record_collective("all_gather", tensor)
        torch.distributed.all_gather(outs, tensor)
        return torch.cat(outs, dim=0)
    out = torch.empty(state.num_processes * tensor.numel(), dtype=tensor.dtype, device=tensor.device)
    record_collective("all_gather", tensor)
    torch.distributed.all_gather_into_tensor(out, tensor.reshape(-1))
    return out.view(-1, *tensor.size()[1:])


def _gpu_gather(tensor):
    leaves = _leaves(tensor, [])
    if not leaves:
        return tensor
    if _coalescable(leaves) and all(t.ndim > 0 for t in leaves):
        # One all-gather for the whole structure: flatten, gather, then de-interleave per rank.
        state = PartialState()
        flat = torch.cat([t.reshape(-1) for t in leaves])
        gathered = _gpu_gather_one(flat).view(state.num_processes, -1)
        outs, off = [], 0
        for t in leaves:
            n = t.numel()
            outs.append(gathered[:, off : off + n].reshape(state.num_processes * t.shape[0], *t.shape[1:]))
            off += n
        return _rebuild(tensor, iter(outs))
    return recursively_apply(_gpu_gather_one, tensor, error_on_other_type=True)


@verify_operation
def gather(tensor):
    """Concatenate `tensor` (nested) from all processes along dim 0."""
    if PartialState().distributed_type in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU, DistributedType.FSDP) and PartialState().num_processes > 1:
        return _gpu_gather(tensor)
    return tensor


def _gpu_gather_object(object: Any):
    output_objects = [None for _ in range(PartialState().num_processes)]
    torch.distributed.all_gather_object(output_objects, object)
    # all_gather_object returns a list of lists; flatten them.
    return [x for y in output_objects for x in y]


def gather_object(object: Any):
    """Gather picklable objects (lists are concatenated) from all processes."""
    if PartialState().distributed_type == DistributedType.NO or PartialState().num_processes == 1:
        return object
    return _gpu_gather_object(object)


# ------------------------------------------------------------------------------------------------------
# broadcast
# ------------------------------------------------------------------------------------------------------
def _gpu_broadcast(data, src=0):
    leaves = _leaves(data, [])
    if _coalescable(leaves):
        flat = torch.cat([t.reshape(-1) for t in leaves])
        record_collective("broadcast", flat)
        torch.distributed.broadcast(flat, src=src)
        outs, off = [], 0
        for t in leaves:
            n = t.numel()
            t.copy_(flat[off : off + n].view_as(t))
            outs.append(t)
            off += n
        return _rebuild(data, iter(outs))

    def _gpu_broadcast_one(tensor, src=0):
        record_collective("broadcast", tensor)
        torch.distributed.broadcast(tensor, src=src)
        return tensor

    return recursively_apply(_gpu_broadcast_one, data, error_on_other_type=True, src=src)


@verify_operation
def broadcast(tensor, from_process: int = 0):
    """In-place broadcast of (nested) tensors from `from_process`."""
    if PartialState().distributed_type in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU, DistributedType.FSDP) and PartialState().num_processes > 1:
        return _gpu_broadcast(tensor, src=from_process)
    return tensor


def broadcast_object_list(object_list, from_process: int = 0):
    if PartialState().distributed_type != DistributedType.NO and PartialState().num_processes > 1:
        torch.distributed.broadcast_object_list(object_list, src=from_process)
    return object_list


def slice_tensors(data, tensor_slice, process_index=None, num_processes=None):
    def _slice_tensor(tensor, tensor_slice):
        return tensor[tensor_slice]

    return recursively_apply(_slice_tensor, data, tensor_slice)


def concatenate(data, dim=0):
    """Concatenate a list of (nested, identically structured) tensors."""
    if isinstance(data[0], (tuple, list)):
        return honor_type(data[0], (concatenate([d[i] for d in data], dim=dim) for i in range(len(data[0]))))
    elif isinstance(data[0], Mapping):
        return type(data[0])({k: concatenate([d[k] for d in data], dim=dim) for k in data[0].keys()})
    elif not isinstance(data[0], torch.Tensor):
        raise TypeError(f"Can only concatenate tensors but got {type(data[0])}")
    return torch.cat(data, dim=dim)


class CannotPadNestedTensorWarning(UserWarning):
    pass


def _all_sizes(tensor) -> torch.Tensor:
    """All ranks' shapes as a [W, ndim] int64 tensor (one tiny all-gather)."""
    size = torch.tensor(tensor.shape, device=tensor.device, dtype=torch.int64)[None]
    return gather(size)


def _padded(tensor: torch.Tensor, dim: int, target: int, value, front: bool) -> torch.Tensor:
    """`tensor` extended along `dim` to length `target` with `value` (before the data when `front`)."""
    missing = target - tensor.shape[dim]
    if missing <= 0:
        return tensor
    shape = list(tensor.shape)
    shape[dim] = missing
    filler = tensor.new_full(shape, value)
    return torch.cat([filler, tensor] if front else [tensor, filler], dim=dim)


@chained_operation
def pad_across_processes(tensor, dim=0, pad_index=0, pad_first=False):
    """Pad every tensor along `dim` to the largest size any process holds (one shape all-gather per tensor), so the
    results can be gathered; nested tensors and out-of-range `dim`s are returned as they are."""

    def _one(t, dim=0, pad_index=0, pad_first=False):
        if getattr(t, "is_nested", False):
            import warnings

            warnings.warn("Cannot pad nested tensors without more information. Leaving unprocessed.", CannotPadNestedTensorWarning)
            return t
        nd = t.dim()
        if not -nd <= dim < nd:
            return t
        dim %= nd
        target = int(_all_sizes(t)[:, dim].max())
        return _padded(t, dim, target, pad_index, pad_first)

    return recursively_apply(_one, tensor, error_on_other_type=True, dim=dim, pad_index=pad_index, pad_first=pad_first)


def _split_padding(batch_size: int, num_processes: int) -> int:
    """Rows `pad_input_tensors` appends (the reference's rule, `utils/operations.py:700-717`, reproduced exactly):
    num_processes minus the per-process share (or minus the batch when smaller than the process count), and when that
    is < 1 while a remainder exists, remainder minus it."""
    per = batch_size // num_processes
    rest = batch_size - per * num_processes
    pad = num_processes - (batch_size if per == 0 else per)
    if pad < 1 and rest > pad:
        pad = rest - pad
    return pad


def pad_input_tensors(tensor, batch_size, num_processes, dim=0):
    """Zero-pad the batch dimension (for `split_between_processes` with `apply_padding`)."""

    def _one(t, batch_size, num_processes, dim=0):
        return _padded(t, dim, batch_size + _split_padding(batch_size, num_processes), 0, False)

    return recursively_apply(_one, tensor, error_on_other_type=True, batch_size=batch_size, num_processes=num_processes, dim=dim)


def gather_tensor_shape(tensor):
    """Shape of `tensor` on the process that holds it (others pass None) — used by `copy_tensor_to_devices`."""
    state = PartialState()
    shape = [-1] * 8
    if tensor is not None:
        shape[: tensor.ndim] = list(tensor.shape)
        shape.append(tensor.ndim)
    else:
        shape.append(-1)
    dev = state.device
    t = torch.tensor(shape, dtype=torch.int64, device=dev)
    allt = gather(t).view(state.num_processes, -1)
    for row in allt.tolist():
        if row[-1] >= 0:
            return row[: row[-1]]
    return None


def copy_tensor_to_devices(tensor=None) -> torch.Tensor:
    """Make the tensor held by exactly one process available on all (used by pipeline inference)."""
    state = PartialState()
    shape = gather_tensor_shape(tensor)
    if tensor is None:
        dtype_code = torch.tensor([-1], device=state.device)
    else:
        dtype_code = torch.tensor([_DTYPES.index(tensor.dtype)], device=state.device)
    codes = gather(dtype_code).tolist()
    dtype = _DTYPES[max(codes)]
    if tensor is None:
        tensor = torch.zeros(shape, dtype=dtype, device=state.device)
    return reduce(tensor, reduction="sum")


_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.int8, torch.uint8, torch.bool, torch.float64]


# ------------------------------------------------------------------------------------------------------
# reduce
# ------------------------------------------------------------------------------------------------------
@verify_operation
def reduce(tensor, reduction="mean", scale=1.0):
    """All-reduce (nested) tensors with `reduction` in {"sum", "mean"}; returns new tensors.

    Nested structures of same-dtype tensors are reduced with a single collective."""

    state = PartialState()
    if state.distributed_type == DistributedType.NO or state.num_processes == 1:
        def _scale_only(t):
            t = t.clone()
            if scale != 1.0:
                t *= scale
            return t

        return recursively_apply(_scale_only, tensor, error_on_other_type=True)

    def _finish(t):
        if reduction == "mean":
            t /= state.num_processes
        if scale != 1.0:
            t *= scale
        return t

    leaves = _leaves(tensor, [])
    if _coalescable(leaves):
        flat = torch.cat([t.reshape(-1) for t in leaves])
        record_collective("all_reduce", flat)
        # small (loss / metric / trigger-flag) reductions take the IPC one-shot kernel (parallel/small_allreduce.py)
        from ..parallel import small_allreduce

        small_allreduce.all_reduce_(flat, torch.distributed.ReduceOp.SUM)
        _finish(flat)
        outs, off = [], 0
        for t in leaves:
            n = t.numel()
            outs.append(flat[off : off + n].view_as(t).clone())
            off += n
        return _rebuild(tensor, iter(outs))

    def _reduce_across_processes(t):
        cloned = t.clone()
        record_collective("all_reduce", cloned)
        torch.distributed.all_reduce(cloned, torch.distributed.ReduceOp.SUM)
        return _finish(cloned)

    return recursively_apply(_reduce_across_processes, tensor, error_on_other_type=True)


# ------------------------------------------------------------------------------------------------------
# fp32 conversion of model outputs under mixed precision
# ------------------------------------------------------------------------------------------------------
def convert_to_fp32(tensor):
    def _convert_to_fp32(tensor):
        return tensor.float()

    def _is_fp16_bf16_tensor(tensor):
        return (is_torch_tensor(tensor) or hasattr(tensor, "dtype")) and tensor.dtype in (torch.float16, torch.bfloat16)

    return recursively_apply(_convert_to_fp32, tensor, test_type=_is_fp16_bf16_tensor)


class ConvertOutputsToFp32:
    """Picklable wrapper casting a forward's fp16/bf16 outputs to fp32."""

    def __init__(self, model_forward):
        self.model_forward = model_forward
        update_wrapper(self, model_forward)

    def __call__(self, *args, **kwargs):
        return convert_to_fp32(self.model_forward(*args, **kwargs))

    def __getstate__(self):
        raise pickle.PicklingError(
            "Cannot pickle a prepared model with automatic mixed precision, please unwrap the model with "
            "`Accelerator.unwrap_model(model)` before pickling it."
        )


def convert_outputs_to_fp32(model_forward):
    model_forward = ConvertOutputsToFp32(model_forward)

    def forward(*args, **kwargs):
        return model_forward(*args, **kwargs)

    forward.__wrapped__ = model_forward
    return forward


@contextmanager
def GatheredParameters(params, modifier_rank=None, fwd_module=None, enabled=True):
    """No-op context (the reference uses it for DeepSpeed ZeRO-3). Our FSDP engine exposes
    `summon_full_params` for the equivalent purpose."""
    yield


def get_grad_scaler(distributed_type: DistributedType = None, **kwargs):
    """fp16 GradScaler (bf16 needs none)."""
    if torch.cuda.is_available():
        return torch.amp.GradScaler("cuda", **kwargs)
    return torch.amp.GradScaler("cpu", **kwargs)
