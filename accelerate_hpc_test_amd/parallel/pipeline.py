"""Pipeline-parallel inference (GPipe micro-batching) for `prepare_pippy`.

Parity target: `/root/reference/src/accelerate/inference.py:31-186` — `split_points="auto"` balances the layers over
the ranks, inputs are cut into `num_chunks` micro-batches, the last stage holds the real output and
`gather_output=True` broadcasts it to every rank; other ranks return `None`.

Design (no graph tracer): the reference traces the model with `torch.export` into stage sub-graphs. Here every rank
runs the model's *own* forward, but the units it does not own live on the **meta device**: they execute as pure
shape propagation (zero FLOPs, zero memory). The first owned block of stage s finds meta tensors among its inputs
and receives the real activations into buffers of exactly those shapes from stage s-1 (no shape handshake); the
last owned block sends its tensor outputs to stage s+1 with async RCCL P2P (`isend`), so micro-batch m+1 is
computed while m is in flight — the GPipe forward schedule falls out of the program order.

Units: the blocks of the model's repeated `ModuleList` (its `_no_split_modules` class), plus every parameter-owning
module outside it (pre-block modules → stage 0, post-block modules → last stage, by registration order).
Parameterless modules (rotary embeddings, activations) run everywhere.
"""

from __future__ import annotations

import dataclasses
from typing import Any, Optional, Union

import torch
import torch.distributed as dist
import torch.nn as nn

from ..state import PartialState


# ------------------------------------------------------------------------------------------------ structure
def _find_block_list(model: nn.Module, no_split_module_classes=None):
    names = set(no_split_module_classes or getattr(model, "_no_split_modules", None) or [])
    best, best_n = None, -1
    for name, m in model.named_modules():
        if isinstance(m, nn.ModuleList) and len(m) > 0:
            if names and not any(type(c).__name__ in names for c in m):
                continue
            n = sum(p.numel() for p in m.parameters())
            if n > best_n:
                best, best_n = (name, m), n
    if best is None:
        raise ValueError("prepare_pippy: could not find the model's repeated block list (pass no_split_module_classes)")
    return best


def _param_bytes(m: nn.Module) -> int:
    return sum(p.numel() * p.element_size() for p in m.parameters())


def _plan(model, stages, split_points, no_split_module_classes):
    list_name, blocks = _find_block_list(model, no_split_module_classes)
    block_names = [f"{list_name}.{i}" if list_name else str(i) for i in range(len(blocks))]
    if stages > len(blocks):
        raise ValueError(f"prepare_pippy: {stages} stages but only {len(blocks)} blocks")
    if split_points == "auto":
        sizes = [_param_bytes(b) for b in blocks]
        total = sum(sizes)
        bounds, acc = [], 0
        for i, s in enumerate(sizes):
            acc += s
            if len(bounds) < stages - 1 and acc >= total * (len(bounds) + 1) / stages and i + 1 < len(blocks):
                bounds.append(i + 1)
        while len(bounds) < stages - 1:  # degenerate sizes: fill remaining boundaries evenly
            bounds.append(min(len(blocks) - (stages - 1 - len(bounds)), (bounds[-1] + 1) if bounds else 1))
        starts = bounds
    else:
        if len(split_points) != stages - 1:
            raise ValueError(f"prepare_pippy: need {stages - 1} split points, got {len(split_points)}")
        starts = [block_names.index(s) for s in split_points]
    stage_of_block = []
    s = 0
    for i in range(len(blocks)):
        while s < len(starts) and i >= starts[s]:
            s += 1
        stage_of_block.append(s)
    units = {}  # module -> stage
    for b, st in zip(blocks, stage_of_block):
        units[b] = st
    seen_list = False
    block_ids = {id(x) for x in blocks.modules()}
    for name, m in model.named_modules():
        if m is blocks:
            seen_list = True
            continue
        if id(m) in block_ids or not any(True for _ in m.parameters(recurse=False)):
            continue
        units[m] = (stages - 1) if seen_list else 0
    split_names = [block_names[i] for i in starts]
    return units, list(blocks), stage_of_block, split_names


# ------------------------------------------------------------------------------------------------ tree helpers
def _flatten(obj):
    if torch.is_tensor(obj):
        return [obj]
    if isinstance(obj, (list, tuple)):
        return [t for x in obj for t in _flatten(x)]
    if isinstance(obj, dict):
        return [t for x in obj.values() for t in _flatten(x)]
    if dataclasses.is_dataclass(obj) and not isinstance(obj, type):
        return [t for f in dataclasses.fields(obj) for t in _flatten(getattr(obj, f.name))]
    return []


def _map(obj, fn):
    if torch.is_tensor(obj):
        return fn(obj)
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):
        return type(obj)(*[_map(x, fn) for x in obj])
    if isinstance(obj, (list, tuple)):
        return type(obj)(_map(x, fn) for x in obj)
    if isinstance(obj, dict):
        out = {k: _map(v, fn) for k, v in obj.items()}
        try:
            return type(obj)(**out) if type(obj) is not dict else out
        except TypeError:
            return out
    if dataclasses.is_dataclass(obj) and not isinstance(obj, type):
        return dataclasses.replace(obj, **{f.name: _map(getattr(obj, f.name), fn) for f in dataclasses.fields(obj)})
    return obj


def _concat_outputs(outs):
    first = outs[0]
    if torch.is_tensor(first):
        return torch.cat(outs, 0) if first.dim() > 0 else first
    if isinstance(first, (list, tuple)) and not hasattr(first, "_fields"):
        return type(first)(_concat_outputs([o[i] for o in outs]) for i in range(len(first)))
    if isinstance(first, dict):
        merged = {k: _concat_outputs([o[k] for o in outs]) for k in first}
        try:
            return type(first)(**merged) if type(first) is not dict else merged
        except TypeError:
            return merged
    if dataclasses.is_dataclass(first) and not isinstance(first, type):
        return dataclasses.replace(first, **{f.name: _concat_outputs([getattr(o, f.name) for o in outs]) for f in dataclasses.fields(first)})
    return first


def _split_batch(obj, n, B):
    if torch.is_tensor(obj) and obj.dim() > 0 and obj.shape[0] == B:
        return list(obj.chunk(n, 0))
    if isinstance(obj, (list, tuple)):
        parts = [_split_batch(x, n, B) for x in obj]
        return [type(obj)(p[i] for p in parts) for i in range(n)]
    if isinstance(obj, dict):
        parts = {k: _split_batch(v, n, B) for k, v in obj.items()}
        return [{k: parts[k][i] for k in obj} for i in range(n)]
    return [obj] * n


def _find_batch(args, kwargs):
    for t in _flatten(list(args) + list(kwargs.values())):
        if t.dim() > 0:
            return t.shape[0]
    return None


# ------------------------------------------------------------------------------------------------ runtime
class _PipelineRuntime:
    def __init__(self, model, units, blocks, stage_of_block, stage, stages, device, group=None):
        self.model, self.stage, self.stages, self.device, self.group = model, stage, stages, device, group
        self.owned = [m for m, s in units.items() if s == stage]
        my_blocks = [b for b, s in zip(blocks, stage_of_block) if s == stage]
        self.first_block = my_blocks[0] if my_blocks else None
        self.last_block = my_blocks[-1] if my_blocks else None
        self.pending = []
        for m, s in units.items():
            if s != stage:
                m.register_forward_pre_hook(self._to_meta_hook, with_kwargs=True)
        if stage > 0 and self.first_block is not None:
            self.first_block.register_forward_pre_hook(self._recv_hook, with_kwargs=True)
        if stage < stages - 1 and self.last_block is not None:
            self.last_block.register_forward_hook(self._send_hook)

    def _peer(self, s):
        return s if self.group is None else dist.get_global_rank(self.group, s)

    @staticmethod
    def _to_meta_hook(mod, args, kwargs):
        conv = lambda t: t.to("meta") if t.device.type != "meta" else t  # noqa: E731
        return _map(args, conv), _map(kwargs, conv)

    def _recv_hook(self, mod, args, kwargs):
        src = self._peer(self.stage - 1)

        def fill(t):
            if t.device.type == "meta" and t.is_floating_point():
                buf = torch.empty(t.shape, dtype=t.dtype, device=self.device)
                dist.recv(buf, src=src, group=self.group)
                return buf
            return t

        return _map(args, fill), _map(kwargs, fill)

    def _send_hook(self, mod, args, out):
        dst = self._peer(self.stage + 1)
        for t in _flatten(out):
            if t.is_floating_point() and t.device.type != "meta":
                t = t.contiguous()
                self.pending.append((dist.isend(t, dst=dst, group=self.group), t))
        return out

    def drain(self):
        for work, _ in self.pending:
            work.wait()
        self.pending.clear()


def _place(model, units, stage, device):
    """Owned parameters → `device`; every other parameter → meta (tied weights follow their owners)."""
    owned_ids = {id(p) for m, s in units.items() if s == stage for p in m.parameters()}
    memo = {}
    for m in model.modules():
        for name, p in list(m._parameters.items()):
            if p is None:
                continue
            if id(p) not in memo:
                tgt = device if id(p) in owned_ids else torch.device("meta")
                memo[id(p)] = nn.Parameter(p.data.to(tgt), requires_grad=p.requires_grad)
            m._parameters[name] = memo[id(p)]
        for name, b in list(m._buffers.items()):
            if b is not None:
                m._buffers[name] = b.to(device)


def prepare_pippy(
    model: nn.Module,
    split_points: Optional[Union[str, list]] = "auto",
    no_split_module_classes: Optional[list] = None,
    example_args: Optional[tuple] = (),
    example_kwargs: Optional[dict] = None,
    num_chunks: Optional[int] = None,
    gather_output: Optional[bool] = False,
):
    """Wrap `model` for pipeline-parallel inference over all processes (one stage per rank).

    `example_args`/`example_kwargs` are accepted for API parity; no tracing is needed. `num_chunks` is the number of
    micro-batches per call (default: number of stages)."""
    state = PartialState()
    stages = state.num_processes
    if num_chunks is None:
        num_chunks = stages
    units, blocks, stage_of_block, split_names = _plan(model, stages, split_points, no_split_module_classes)
    stage = state.process_index
    device = state.device
    if stages > 1:
        _place(model, units, stage, device)
    else:
        model.to(device)
    runtime = _PipelineRuntime(model, units, blocks, stage_of_block, stage, stages, device) if stages > 1 else None
    model.hf_split_points = split_names
    model._original_forward = model.forward
    orig = model.forward

    def forward(*args, **kwargs):
        if runtime is None:
            return orig(*args, **kwargs)
        B = _find_batch(args, kwargs)
        if B is None:
            raise ValueError("prepare_pippy: could not find the batch size from the inputs")
        n = max(1, min(num_chunks, B))
        mb_args, mb_kwargs = _split_batch(list(args), n, B), _split_batch(kwargs, n, B)
        outs = []
        with torch.no_grad():
            for i in range(n):
                outs.append(orig(*mb_args[i], **mb_kwargs[i]))
        runtime.drain()
        out = _concat_outputs(outs)
        last = stages - 1
        if gather_output:
            def bcast(t):
                buf = t if t.device.type != "meta" else torch.empty(t.shape, dtype=t.dtype, device=device)
                dist.broadcast(buf, src=last)
                return buf

            return _map(out, bcast)
        return out if stage == last else None

    forward.__wrapped__ = orig
    model.forward = forward
    model.pippy_stage = runtime
    return model
