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
