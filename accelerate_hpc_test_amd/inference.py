"""Pipeline-parallel inference: `prepare_pippy` (reference `/root/reference/src/accelerate/inference.py:31-186`).

Semantics kept: one pipeline stage per process; `split_points="auto"` balances the decoder blocks over the stages by
parameter bytes (or names the first block of every stage after the first); each call is cut into `num_chunks`
micro-batches; the last stage holds the real output and `gather_output=True` broadcasts it to every rank, other ranks
return `None`; `model.hf_split_points` records the cut.

What differs: there is no `torch.export` tracing into stage sub-graphs. Every rank runs the model's own forward, with
the units it does not own on the meta device (pure shape propagation); the runtime in `parallel/pipeline.py` moves the
activations between neighbouring stages with RCCL point-to-point sends over xGMI.
"""

from __future__ import annotations

from typing import Optional, Union

import torch
import torch.distributed as dist
import torch.nn as nn

from .parallel.pipeline import _concat_outputs, _flatten, _map, _PipelineRuntime, _place
from .state import PartialState


# ------------------------------------------------------------------------------------------------ structure
def _find_block_lists(model: nn.Module, no_split_module_classes=None):
    """The model's repeated block lists, in registration order: every `ModuleList` of the no-split class (HF
    `_no_split_modules`), e.g. T5's `encoder.block` and `decoder.block`; without class names, the largest list."""
    names = set(no_split_module_classes or getattr(model, "_no_split_modules", None) or [])
    lists, best, best_n = [], None, -1
    for name, m in model.named_modules():
        if isinstance(m, nn.ModuleList) and len(m) > 0:
            if names:
                if any(type(c).__name__ in names for c in m):
                    lists.append((name, m))
                continue
            n = sum(p.numel() for p in m.parameters())
            if n > best_n:
                best, best_n = (name, m), n
    if not names and best is not None:
        lists = [best]
    if not lists:
        raise ValueError("prepare_pippy: could not find the model's repeated block list (pass no_split_module_classes)")
    return lists


def _param_bytes(m: nn.Module) -> int:
    return sum(p.numel() * p.element_size() for p in m.parameters())


def _plan(model, stages, split_points, no_split_module_classes):
    """Stage of every unit. Units = the blocks of all block lists (concatenated in registration order, which is their
    execution order for encoder -> decoder models) + every parameter-owning module outside them, which goes to the
    stage of the block registered just before it (stage 0 before the first block). Modules registered under more
    than one parent (T5's `shared` embedding = encoder / decoder `embed_tokens`) are used by several stages: they are
    returned as `replicated`, real on every stage."""
    lists = _find_block_lists(model, no_split_module_classes)
    blocks, block_names = [], []
    for list_name, ml in lists:
        for i, b in enumerate(ml):
            blocks.append(b)
            block_names.append(f"{list_name}.{i}" if list_name else str(i))
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
    units = dict(zip(blocks, stage_of_block))
    block_stage = {id(b): st for b, st in units.items()}
    in_block = {id(x) for b in blocks for x in b.modules()}
    list_ids = {id(ml) for _, ml in lists}
    uses = {}
    for _, m in model.named_modules(remove_duplicate=False):
        uses[id(m)] = uses.get(id(m), 0) + 1
    replicated = set()
    cur = 0
    for name, m in model.named_modules():
        if id(m) in block_stage:
            cur = block_stage[id(m)]
            continue
        if id(m) in list_ids or id(m) in in_block or not any(True for _ in m.parameters(recurse=False)):
            continue
        units[m] = cur
        if uses.get(id(m), 1) > 1:
            replicated.add(m)
    split_names = [block_names[i] for i in starts]
    return units, blocks, stage_of_block, split_names, replicated


# ------------------------------------------------------------------------------------------------ micro-batching
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



# ------------------------------------------------------------------------------------------------ entry point
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
    units, blocks, stage_of_block, split_names, replicated = _plan(model, stages, split_points, no_split_module_classes)
    stage = state.process_index
    device = state.device
    if stages > 1:
        _place(model, units, stage, device, replicated)
        for m in replicated:  # real on every stage: neither sent nor turned into meta
            units[m] = stage
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
                runtime.reset()
                outs.append(orig(*mb_args[i], **mb_kwargs[i]))
            runtime.reset()
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
