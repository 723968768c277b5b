"""Accelerator state checkpoint writer/reader (model, optimizer, scheduler, sampler, scaler, RNG, custom objects).

Parity: `/root/reference/src/accelerate/checkpointing.py:62-331`. File names and layout are identical
(`model.safetensors`/`model_{i}.safetensors` or `pytorch_model{_i}.bin`, `optimizer{_i}.bin`, `scheduler{_i}.bin`,
`sampler{_i}.bin`, `dl_state_dict{_i}.bin`, `scaler.pt`, `random_states_{rank}.pkl`, `custom_checkpoint_{i}.pkl`).
RNG state files are written with `torch.save` of plain tensors/lists and read with `weights_only=True`.
"""

from __future__ import annotations

import os
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
from .utils.dataclasses import DistributedType
from .utils.other import load, save

logger = get_logger(__name__)


def _suffix(i: int) -> str:
    return "" if i == 0 else f"_{i}"


def save_accelerator_state(
    output_dir: str,
    model_states: list[dict],
    optimizers: list,
    schedulers: list,
    dataloaders: list,
    process_index: int,
    step: int,
    scaler=None,
    save_on_each_node: bool = False,
    safe_serialization: bool = True,
):
    output_dir = Path(output_dir)
    for i, state in enumerate(model_states):
        weights_name = WEIGHTS_NAME if not safe_serialization else SAFE_WEIGHTS_NAME
        if i > 0:
            weights_name = weights_name.replace(".", f"_{i}.")
        output_model_file = output_dir.joinpath(weights_name)
        save(state, output_model_file, save_on_each_node=save_on_each_node, safe_serialization=safe_serialization)
        logger.info(f"Model weights saved in {output_model_file}")
    for i, opt in enumerate(optimizers):
        state = opt.state_dict()
        optimizer_name = f"{OPTIMIZER_NAME}.bin" if i == 0 else f"{OPTIMIZER_NAME}_{i}.bin"
        output_optimizer_file = output_dir.joinpath(optimizer_name)
        save(state, output_optimizer_file, save_on_each_node=save_on_each_node, safe_serialization=False)
        logger.info(f"Optimizer state saved in {output_optimizer_file}")
    for i, scheduler in enumerate(schedulers):
        state = scheduler.state_dict()
        scheduler_name = f"{SCHEDULER_NAME}.bin" if i == 0 else f"{SCHEDULER_NAME}_{i}.bin"
        output_scheduler_file = output_dir.joinpath(scheduler_name)
        save(state, output_scheduler_file, save_on_each_node=save_on_each_node, safe_serialization=False)
        logger.info(f"Scheduler state saved in {output_scheduler_file}")
    from .data_loader import IterableDatasetShard, SeedableRandomSampler

    for i, dataloader in enumerate(dataloaders):
        sampler_name = f"{SAMPLER_NAME}.bin" if i == 0 else f"{SAMPLER_NAME}_{i}.bin"
        output_sampler_file = output_dir.joinpath(sampler_name)
        if isinstance(dataloader.dataset, IterableDatasetShard):
            sampler = dataloader.get_sampler()
            if isinstance(sampler, SeedableRandomSampler):
                save({"epoch": sampler.epoch, "initial_seed": sampler.initial_seed}, output_sampler_file, save_on_each_node=save_on_each_node)
        if hasattr(dataloader, "state_dict"):
            dl_name = f"{DATALOADER_STATE_NAME}.bin" if i == 0 else f"{DATALOADER_STATE_NAME}_{i}.bin"
            save(dataloader.state_dict(), output_dir.joinpath(dl_name), save_on_each_node=save_on_each_node)
    if scaler is not None:
        state = scaler.state_dict()
        output_scaler_file = output_dir.joinpath(SCALER_NAME)
        torch.save(state, output_scaler_file)
        logger.info(f"Gradient scaler state saved in {output_scaler_file}")
    # RNG states (per process): only tensors / python lists so they load with weights_only=True.
    states = {"step": step}
    py_state = random.getstate()
    states["random_state"] = [py_state[0], list(py_state[1]), py_state[2]]
    np_state = np.random.get_state()
    states["numpy_random_seed"] = [np_state[0], torch.from_numpy(np.asarray(np_state[1]).astype(np.int64)), int(np_state[2]), int(np_state[3]), float(np_state[4])]
    states["torch_manual_seed"] = torch.get_rng_state()
    if torch.cuda.is_available():
        states["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    output_states_file = output_dir.joinpath(f"{RNG_STATE_NAME}_{process_index}.pkl")
    torch.save(states, output_states_file)
    logger.info(f"Random states saved in {output_states_file}")
    return output_dir


def load_accelerator_state(
    input_dir,
    models,
    optimizers,
    schedulers,
    dataloaders,
    process_index,
    scaler=None,
    map_location=None,
    load_kwargs=None,
    **load_model_func_kwargs,
):
    override_attributes = dict()
    if map_location not in [None, "cpu", "on_device"]:
        raise TypeError("Unsupported optimizer map location passed, please choose one of `None`, `'cpu'`, or `'on_device'`.")
    if map_location is None:
        map_location = "cpu"
    elif map_location == "on_device":
        map_location = PartialState().device
    if load_kwargs is None:
        load_kwargs = {}
    input_dir = Path(input_dir)
    for i, model in enumerate(models):
        ending = f"_{i}" if i > 0 else ""
        input_model_file = input_dir.joinpath(f"{SAFE_MODEL_NAME}{ending}.safetensors")
        if input_model_file.exists():
            from safetensors.torch import load_file

            state_dict = load_file(input_model_file, device=str(map_location))
        else:
            input_model_file = input_dir.joinpath(f"{WEIGHTS_NAME.replace('.bin', '')}{ending}.bin")
            state_dict = load(input_model_file, map_location=map_location)
        model.load_state_dict(state_dict, **load_model_func_kwargs)
    logger.info("All model weights loaded successfully")
    for i, opt in enumerate(optimizers):
        optimizer_name = f"{OPTIMIZER_NAME}.bin" if i == 0 else f"{OPTIMIZER_NAME}_{i}.bin"
        input_optimizer_file = input_dir.joinpath(optimizer_name)
        optimizer_state = load(input_optimizer_file, map_location=map_location, **load_kwargs)
        optimizers[i].load_state_dict(optimizer_state)
    logger.info("All optimizer states loaded successfully")
    for i, scheduler in enumerate(schedulers):
        scheduler_name = f"{SCHEDULER_NAME}.bin" if i == 0 else f"{SCHEDULER_NAME}_{i}.bin"
        input_scheduler_file = input_dir.joinpath(scheduler_name)
        scheduler_state = load(input_scheduler_file, **load_kwargs)
        scheduler.load_state_dict(scheduler_state)
    logger.info("All scheduler states loaded successfully")
    from .data_loader import IterableDatasetShard, SeedableRandomSampler

    for i, dataloader in enumerate(dataloaders):
        sampler_name = f"{SAMPLER_NAME}.bin" if i == 0 else f"{SAMPLER_NAME}_{i}.bin"
        input_sampler_file = input_dir.joinpath(sampler_name)
        if isinstance(dataloader.dataset, IterableDatasetShard) and input_sampler_file.exists():
            sampler = dataloader.get_sampler()
            if isinstance(sampler, SeedableRandomSampler):
                st = load(input_sampler_file)
                sampler.epoch, sampler.initial_seed = st["epoch"], st["initial_seed"]
        dl_name = f"{DATALOADER_STATE_NAME}.bin" if i == 0 else f"{DATALOADER_STATE_NAME}_{i}.bin"
        dl_file = input_dir.joinpath(dl_name)
        if dl_file.exists() and hasattr(dataloader, "load_state_dict"):
            dataloader.load_state_dict(load(dl_file))
    logger.info("All dataloader sampler states loaded successfully")
    if scaler is not None:
        input_scaler_file = input_dir.joinpath(SCALER_NAME)
        scaler_state = torch.load(input_scaler_file, weights_only=True)
        scaler.load_state_dict(scaler_state)
        logger.info("GradScaler state loaded successfully")
    try:
        states = torch.load(input_dir.joinpath(f"{RNG_STATE_NAME}_{process_index}.pkl"), weights_only=True)
        if "step" in states:
            override_attributes["step"] = states["step"]
        rs = states["random_state"]
        random.setstate((rs[0], tuple(rs[1]), rs[2]))
        ns = states["numpy_random_seed"]
        np.random.set_state((ns[0], ns[1].numpy().astype(np.uint32), ns[2], ns[3], ns[4]))
        torch.set_rng_state(states["torch_manual_seed"])
        if torch.cuda.is_available() and "torch_cuda_manual_seed" in states:
            torch.cuda.set_rng_state_all(states["torch_cuda_manual_seed"])
        logger.info("All random states loaded successfully")
    except Exception:
        logger.info("Could not load random states")
    return override_attributes


def save_custom_state(obj, path, index: int = 0, save_on_each_node: bool = False):
    save_location = Path(path) / f"custom_checkpoint_{index}.pkl"
    logger.info(f"Saving the state of {obj.__class__.__name__} to {save_location}")
    save(obj.state_dict(), save_location, save_on_each_node=save_on_each_node)


def load_custom_state(obj, path, index: int = 0):
    load_location = f"{path}/custom_checkpoint_{index}.pkl"
    logger.info(f"Loading the state of {obj.__class__.__name__} from {load_location}")
    obj.load_state_dict(load(load_location, map_location="cpu"))
