"""Seeding and cross-rank RNG synchronisation.

Parity: `/root/reference/src/accelerate/utils/random.py:39-156` (`set_seed`, `synchronize_rng_state(s)`).
All RNG states are broadcast from rank 0 in ONE collective per call (the states are packed into a single
uint8 buffer) instead of one broadcast per generator. Also fixes the reference quirk at
`random.py:146` (compares the state tensor with an enum instead of the RNG type).
"""

from __future__ import annotations

import random
from typing import Optional, Union

import numpy as np
import torch

from .dataclasses import DistributedType, RNGType


def AcceleratorState():  # noqa: N802 - lazy accessor (avoids the utils <-> state import cycle)
    from ..state import AcceleratorState as _AcceleratorState

    return _AcceleratorState()


def set_seed(seed: int, device_specific: bool = False, deterministic: bool = False):
    """Seed python, numpy and torch (CPU + every HIP device). `device_specific` offsets by the rank."""
    if device_specific:
        seed += AcceleratorState().process_index
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    if deterministic:
        torch.use_deterministic_algorithms(True)


def _get_state(rng_type: RNGType, generator: Optional[torch.Generator]):
    if rng_type == RNGType.TORCH:
        return torch.get_rng_state()
    if rng_type == RNGType.CUDA:
        return torch.cuda.get_rng_state()
    if rng_type == RNGType.GENERATOR:
        if generator is None:
            raise ValueError("Need a generator to synchronize its seed.")
        return generator.get_state()
    raise ValueError(f"RNG type {rng_type} is not supported on MI355X")


def _set_state(rng_type: RNGType, generator, state: torch.Tensor):
    if rng_type == RNGType.TORCH:
        torch.set_rng_state(state)
    elif rng_type == RNGType.CUDA:
        torch.cuda.set_rng_state(state)
    elif rng_type == RNGType.GENERATOR:
        generator.set_state(state)


def synchronize_rng_state(rng_type: Optional[RNGType] = None, generator: Optional[torch.Generator] = None):
    synchronize_rng_states([rng_type], generator=generator)


def synchronize_rng_states(rng_types: list[Union[str, RNGType]], generator: Optional[torch.Generator] = None):
    """Broadcast the given RNG states from process 0 (one packed collective)."""
    state = AcceleratorState()
    types = []
    for t in rng_types:
        if t is None:
            continue
        t = RNGType(t)
        if t == RNGType.CUDA and not torch.cuda.is_available():
            continue
        if t == RNGType.GENERATOR and generator is None:
            continue
        if t in (RNGType.XLA, RNGType.NPU, RNGType.XPU, RNGType.HPU):
            continue
        types.append(t)
    if not types or state.distributed_type == DistributedType.NO or state.num_processes == 1:
        return
    states = [_get_state(t, generator).to(torch.uint8) for t in types]
    sizes = [s.numel() for s in states]
    flat = torch.cat(states)
    dev = state.device if state.backend and "nccl" in state.backend else torch.device("cpu")
    flat = flat.to(dev)
    torch.distributed.broadcast(flat, 0)
    flat = flat.cpu()
    off = 0
    for t, n in zip(types, sizes):
        _set_state(t, generator, flat[off : off + n].clone())
        off += n
