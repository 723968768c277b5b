"""Pipeline-parallel inference runtime (GPipe micro-batching): stage placement, activation transport and output
pytree helpers. The user entry point, stage planning and micro-batching are `accelerate_hpc_test_amd/inference.py`.

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

import torch
import torch.distributed as dist
import torch.nn as nn


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
