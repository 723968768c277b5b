"""Accelerator state checkpoints: model / optimizer / scheduler / sampler / dataloader / scaler / RNG / custom objects.

File names and layout follow the reference (`/root/reference/src/accelerate/checkpointing.py:62-331`) so checkpoints
move between the two: the k-th object of a kind gets the kind's name with `_k` before the extension from k = 1 on
(`model.safetensors`, `model_1.safetensors` or `pytorch_model.bin`, `optimizer.bin`, `scheduler_1.bin`,
`sampler.bin`, `dl_state_dict.bin`, `scaler.pt`, `random_states_<rank>.pkl`, `custom_checkpoint_<k>.pkl`).

Design: `CheckpointLayout` is the one place that knows the names; `save_accelerator_state` / `load_accelerator_state`
walk the object lists through it. RNG states hold only tensors, numbers and lists, so they are written with
`torch.save` and read back with `weights_only=True` (nothing in a checkpoint is unpickled as code).
"""

from __future__ import annotations

import random
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from .logging import get_logger
from .state import PartialState
from .utils.constants import (
    DATALOADER_STATE_NAME,
    OPTIMIZER_NAME,
    RNG_STATE_NAME,
    SAFE_MODEL_NAME,
    SAFE_WEIGHTS_NAME,
    SAMPLER_NAME,
    SCALER_NAME,
    SCHEDULER_NAME,
    WEIGHTS_NAME,
)
from .utils.other import load, save

logger = get_logger(__name__)


class CheckpointLayout:
    """File names of every piece of an accelerator checkpoint inside `root`."""

    def __init__(self, root):
        self.root = Path(root)

    @staticmethod
    def _nth(stem: str, ext: str, k: int) -> str:
        return f"{stem}{'' if k == 0 else f'_{k}'}{ext}"

    def model(self, k: int, safe: bool) -> Path:
        base = SAFE_WEIGHTS_NAME if safe else WEIGHTS_NAME  # "model.safetensors" / "pytorch_model.bin"
        stem, ext = base.rsplit(".", 1)
        return self.root / self._nth(stem, "." + ext, k)

    def model_candidates(self, k: int):
        yield self.root / self._nth(SAFE_MODEL_NAME, ".safetensors", k)
        yield self.root / self._nth(WEIGHTS_NAME.replace(".bin", ""), ".bin", k)

    def optimizer(self, k):
        return self.root / self._nth(OPTIMIZER_NAME, ".bin", k)

    def scheduler(self, k):
        return self.root / self._nth(SCHEDULER_NAME, ".bin", k)

    def sampler(self, k):
        return self.root / self._nth(SAMPLER_NAME, ".bin", k)

    def dataloader(self, k):
        return self.root / self._nth(DATALOADER_STATE_NAME, ".bin", k)

    def scaler(self):
        return self.root / SCALER_NAME

    def rng(self, rank: int):
        return self.root / f"{RNG_STATE_NAME}_{rank}.pkl"

    def custom(self, k: int):
        return self.root / f"custom_checkpoint_{k}.pkl"


# ------------------------------------------------------------------------------------------------ RNG
def _rng_snapshot(step: int) -> dict:
    py = random.getstate()
    npst = np.random.get_state()
    snap = {
        "step": step,
        "random_state": [py[0], list(py[1]), py[2]],
        "numpy_random_seed": [npst[0], torch.from_numpy(np.asarray(npst[1]).astype(np.int64)), int(npst[2]),
                              int(npst[3]), float(npst[4])],
        "torch_manual_seed": torch.get_rng_state(),
    }
    if torch.cuda.is_available():
        snap["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    return snap


def _rng_restore(snap: dict):
    version, internal, gauss = snap["random_state"]
    random.setstate((version, tuple(internal), gauss))
    kind, keys, pos, has_gauss, cached = snap["numpy_random_seed"]
    np.random.set_state((kind, keys.numpy().astype(np.uint32), pos, has_gauss, cached))
    torch.set_rng_state(snap["torch_manual_seed"])
    if torch.cuda.is_available() and "torch_cuda_manual_seed" in snap:
        torch.cuda.set_rng_state_all(snap["torch_cuda_manual_seed"])


def _seedable_sampler(dataloader):
    from .data_loader import IterableDatasetShard, SeedableRandomSampler

    if not isinstance(dataloader.dataset, IterableDatasetShard):
        return None
    sampler = dataloader.get_sampler()
    return sampler if isinstance(sampler, SeedableRandomSampler) else None


# ------------------------------------------------------------------------------------------------ save / load
def save_accelerator_state(output_dir, model_states: list, optimizers: list, schedulers: list, dataloaders: list,
                           process_index: int, step: int, scaler=None, save_on_each_node: bool = False,
                           safe_serialization: bool = True):
    """Write every piece of the training state under `output_dir` (see `CheckpointLayout`)."""
    lay = CheckpointLayout(output_dir)
    node_kw = {"save_on_each_node": save_on_each_node}
    for k, state in enumerate(model_states):
        path = lay.model(k, safe_serialization)
        save(state, path, safe_serialization=safe_serialization, **node_kw)
        logger.info(f"Model weights saved in {path}")
    for kind, objs, namer in (("Optimizer", optimizers, lay.optimizer), ("Scheduler", schedulers, lay.scheduler)):
        for k, obj in enumerate(objs):
            save(obj.state_dict(), namer(k), safe_serialization=False, **node_kw)
            logger.info(f"{kind} state saved in {namer(k)}")
    for k, dl in enumerate(dataloaders):
        sampler = _seedable_sampler(dl)
        if sampler is not None:
            save({"epoch": sampler.epoch, "initial_seed": sampler.initial_seed}, lay.sampler(k), **node_kw)
        if getattr(dl, "use_stateful_dataloader", False):  # position within the epoch: only for stateful loaders
            save(dl.state_dict(), lay.dataloader(k), **node_kw)
    if scaler is not None:
        torch.save(scaler.state_dict(), lay.scaler())
        logger.info(f"Gradient scaler state saved in {lay.scaler()}")
    torch.save(_rng_snapshot(step), lay.rng(process_index))
    logger.info(f"Random states saved in {lay.rng(process_index)}")
    return Path(output_dir)


def load_accelerator_state(input_dir, models, optimizers, schedulers, dataloaders, process_index, scaler=None,
                           map_location=None, load_kwargs: Optional[dict] = None, **load_model_func_kwargs) -> dict:
    """Restore what `save_accelerator_state` wrote; returns attributes to override on the Accelerator (`step`)."""
    if map_location not in (None, "cpu", "on_device"):
        raise TypeError("Unsupported optimizer map location passed, please choose one of `None`, `'cpu'`, or `'on_device'`.")
    where = PartialState().device if map_location == "on_device" else "cpu"
    load_kwargs = load_kwargs or {}
    lay = CheckpointLayout(input_dir)
    for k, model in enumerate(models):
        safe_path, bin_path = lay.model_candidates(k)
        if safe_path.exists():
            from safetensors.torch import load_file

            state = load_file(safe_path, device=str(where))
        else:
            state = load(bin_path, map_location=where)
        model.load_state_dict(state, **load_model_func_kwargs)
    logger.info("All model weights loaded successfully")
    for k, opt in enumerate(optimizers):
        opt.load_state_dict(load(lay.optimizer(k), map_location=where, **load_kwargs))
    logger.info("All optimizer states loaded successfully")
    for k, sched in enumerate(schedulers):
        sched.load_state_dict(load(lay.scheduler(k), **load_kwargs))
    logger.info("All scheduler states loaded successfully")
    for k, dl in enumerate(dataloaders):
        sampler = _seedable_sampler(dl)
        if sampler is not None and lay.sampler(k).exists():
            saved = load(lay.sampler(k))
            sampler.epoch, sampler.initial_seed = saved["epoch"], saved["initial_seed"]
        if getattr(dl, "use_stateful_dataloader", False) and lay.dataloader(k).exists():
            dl.load_state_dict(load(lay.dataloader(k)))
    logger.info("All dataloader sampler states loaded successfully")
    if scaler is not None:
        scaler.load_state_dict(torch.load(lay.scaler(), weights_only=True))
        logger.info("GradScaler state loaded successfully")
    overrides = {}
    try:
        snap = torch.load(lay.rng(process_index), weights_only=True)
        if "step" in snap:
            overrides["step"] = snap["step"]
        _rng_restore(snap)
        logger.info("All random states loaded successfully")
    except Exception:
        logger.info("Could not load random states")
    return overrides


def save_custom_state(obj, path, index: int = 0, save_on_each_node: bool = False):
    target = CheckpointLayout(path).custom(index)
    logger.info(f"Saving the state of {obj.__class__.__name__} to {target}")
    save(obj.state_dict(), target, save_on_each_node=save_on_each_node)


def load_custom_state(obj, path, index: int = 0):
    source = CheckpointLayout(path).custom(index)
    logger.info(f"Loading the state of {obj.__class__.__name__} from {source}")
    obj.load_state_dict(load(source, map_location="cpu"))
