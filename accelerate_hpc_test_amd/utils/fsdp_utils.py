"""Checkpointing for models sharded by the native FSDP engine.

Parity: `/root/reference/src/accelerate/utils/fsdp_utils.py:56-418`. Same directory / file names as the reference:
  FULL_STATE_DICT    → `pytorch_model_fsdp{_i}.bin` (rank 0), `optimizer{_i}.bin` (rank 0)
  SHARDED_STATE_DICT → `pytorch_model_fsdp_{i}/` and `optimizer_{i}/` directories with one file per rank.
The reference uses torch DCP for sharded dirs; ours writes `shard_{rank}.safetensors` + `meta_{rank}.json` (model)
and `shard_{rank}.pt` (optimizer) with the flat-slice layout, which lets a checkpoint written on N ranks be loaded on
M ranks (each rank reads the pieces overlapping its new slice). `merge_fsdp_weights` turns a sharded dir into one
`model.safetensors` / `pytorch_model.bin` (the `accelerate merge-weights` command).
"""

from __future__ import annotations

import glob
import json
import os
from collections import OrderedDict

import torch
import torch.distributed as dist

from ..logging import get_logger
from .constants import FSDP_MODEL_NAME, OPTIMIZER_NAME, SAFE_WEIGHTS_NAME, WEIGHTS_NAME

logger = get_logger(__name__)


def _engine(model):
    from ..parallel.fsdp import FullyShardedModule

    if isinstance(model, FullyShardedModule):
        return model.engine
    eng = getattr(model, "engine", None)
    if eng is None:
        raise ValueError("Model is not sharded by the native FSDP engine.")
    return eng


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _barrier():
    if dist.is_available() and dist.is_initialized():
        from ..state import PartialState

        PartialState().wait_for_everyone()


def save_fsdp_model(fsdp_plugin, accelerator, model, output_dir, model_index=0, adapter_only=False):
    os.makedirs(output_dir, exist_ok=True)
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        sd = eng.full_state_dict(rank0_only=True)
        if _rank() == 0:
            name = f"{FSDP_MODEL_NAME}.bin" if model_index == 0 else f"{FSDP_MODEL_NAME}_{model_index}.bin"
            path = os.path.join(output_dir, name)
            torch.save(sd, path)
            logger.info(f"Model saved to {path}")
    else:
        ckpt_dir = os.path.join(output_dir, f"{FSDP_MODEL_NAME}_{model_index}")
        os.makedirs(ckpt_dir, exist_ok=True)
        shard = eng.sharded_state_dict()
        from safetensors.torch import save_file

        r = eng.rank
        if getattr(eng, "replicate_rank", 0) != 0:  # HSDP / NO_SHARD replicas hold identical shards: replica 0 writes
            _barrier()
            return
        save_file({k: v.contiguous() for k, v in shard["tensors"].items()}, os.path.join(ckpt_dir, f"shard_{r}.safetensors"))
        with open(os.path.join(ckpt_dir, f"meta_{r}.json"), "w") as f:
            json.dump(shard["meta"], f)
        logger.info(f"Model shard saved to {ckpt_dir}")
    _barrier()


def _read_sharded_dir(ckpt_dir):
    from safetensors.torch import load_file

    pieces = []
    for meta_path in sorted(glob.glob(os.path.join(ckpt_dir, "meta_*.json"))):
        r = int(os.path.basename(meta_path)[5:-5])
        with open(meta_path) as f:
            meta = json.load(f)
        tensors = load_file(os.path.join(ckpt_dir, f"shard_{r}.safetensors"))
        pieces.append((tensors, meta))
    return pieces


def load_fsdp_model(fsdp_plugin, accelerator, model, input_dir, model_index=0, adapter_only=False):
    _barrier()
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        name = f"{FSDP_MODEL_NAME}.bin" if model_index == 0 else f"{FSDP_MODEL_NAME}_{model_index}.bin"
        path = os.path.join(input_dir, name)
        # every rank reads the full file (host RAM is plentiful on MI355X nodes) and keeps its slice
        sd = torch.load(path, map_location="cpu", weights_only=True)
        eng.load_full_state_dict(sd)
    else:
        ckpt_dir = input_dir if os.path.basename(os.path.normpath(input_dir)).startswith(FSDP_MODEL_NAME) else os.path.join(input_dir, f"{FSDP_MODEL_NAME}_{model_index}")
        eng.load_sharded_pieces(_read_sharded_dir(ckpt_dir))
    _barrier()


# ---------------------------------------------------------------------------------------------- optimizer
def _optim_full_state(eng, optimizer):
    """Gather optimizer state into {fqn: {key: full tensor}} (one all-gather per unit per state key)."""
    opt = getattr(optimizer, "optimizer", optimizer)
    out, step_val = OrderedDict(), None
    for unit in eng.units:
        keys = set()
        for info in unit.infos:
            keys.update(k for k, v in opt.state.get(info.shard_param, {}).items() if torch.is_tensor(v) and v.dim() > 0)
            st = opt.state.get(info.shard_param, {})
            if "step" in st:
                step_val = st["step"]
        for key in sorted(keys):
            local = torch.zeros(unit.shard_numel, dtype=torch.float32, device=eng.device)
            for info in unit.infos:
                t = opt.state.get(info.shard_param, {}).get(key)
                if t is not None and info.local_hi > info.local_lo:
                    local[info.local_lo : info.local_hi].copy_(t.reshape(-1).float())
            full = eng.gather_full(unit, local)
            for info in unit.infos:
                out.setdefault(info.fqn, {})[key] = full[info.offset : info.offset + info.numel].view(info.shape).cpu().clone()
    groups = []
    fqn_of = {id(info.shard_param): info.fqn for unit in eng.units for info in unit.infos}
    for g in opt.param_groups:
        gg = {k: v for k, v in g.items() if k != "params"}
        gg["params"] = [fqn_of.get(id(p)) for p in g["params"]]
        groups.append(gg)
    return {"state": out, "param_groups": groups, "step": step_val}


def _optim_load_full(eng, optimizer, sd):
    opt = getattr(optimizer, "optimizer", optimizer)
    info_of = {info.fqn: info for unit in eng.units for info in unit.infos}
    for fqn, st in sd["state"].items():
        info = info_of.get(fqn)
        if info is None:
            continue
        n = info.local_hi - info.local_lo
        new = {}
        for k, v in st.items():
            new[k] = v.reshape(-1)[info.param_lo : info.param_lo + n].to(eng.device, torch.float32).clone()
        if sd.get("step") is not None:
            new["step"] = torch.as_tensor(sd["step"], dtype=torch.float32).clone()
        opt.state[info.shard_param] = new
    for g, gs in zip(opt.param_groups, sd.get("param_groups", [])):
        for k, v in gs.items():
            if k != "params":
                g[k] = v


def save_fsdp_optimizer(fsdp_plugin, accelerator, optimizer, model, output_dir, optimizer_index=0):
    os.makedirs(output_dir, exist_ok=True)
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        sd = _optim_full_state(eng, optimizer)
        if _rank() == 0:
            name = f"{OPTIMIZER_NAME}.bin" if optimizer_index == 0 else f"{OPTIMIZER_NAME}_{optimizer_index}.bin"
            torch.save(sd, os.path.join(output_dir, name))
    else:
        d = os.path.join(output_dir, f"{OPTIMIZER_NAME}_{optimizer_index}")
        os.makedirs(d, exist_ok=True)
        opt = getattr(optimizer, "optimizer", optimizer)
        local = {}
        for unit in eng.units:
            for info in unit.infos:
                st = opt.state.get(info.shard_param)
                if st:
                    local[info.fqn] = {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in st.items()}
        fqn_of = {id(info.shard_param): info.fqn for unit in eng.units for info in unit.infos}
        groups = [{**{k: v for k, v in g.items() if k != "params"}, "params": [fqn_of.get(id(p)) for p in g["params"]]} for g in opt.param_groups]
        meta = {info.fqn: {"param_lo": info.param_lo, "numel": info.local_hi - info.local_lo} for unit in eng.units for info in unit.infos}
        if getattr(eng, "replicate_rank", 0) == 0:  # replicas hold identical optimizer shards
            torch.save({"state": local, "param_groups": groups, "meta": meta}, os.path.join(d, f"shard_{eng.rank}.pt"))
    _barrier()


def load_fsdp_optimizer(fsdp_plugin, accelerator, optimizer, model, input_dir, optimizer_index=0, adapter_only=False):
    _barrier()
    eng = _engine(model)
    opt = getattr(optimizer, "optimizer", optimizer)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        name = f"{OPTIMIZER_NAME}.bin" if optimizer_index == 0 else f"{OPTIMIZER_NAME}_{optimizer_index}.bin"
        sd = torch.load(os.path.join(input_dir, name), map_location="cpu", weights_only=True)
        _optim_load_full(eng, optimizer, sd)
    else:
        d = input_dir if os.path.basename(os.path.normpath(input_dir)).startswith(OPTIMIZER_NAME) else os.path.join(input_dir, f"{OPTIMIZER_NAME}_{optimizer_index}")
        files = sorted(glob.glob(os.path.join(d, "shard_*.pt")))
        saved = [torch.load(f, map_location="cpu", weights_only=True) for f in files]
        for unit in eng.units:
            for info in unit.infos:
                lo_need, hi_need = info.param_lo, info.param_lo + (info.local_hi - info.local_lo)
                new = {}
                for s in saved:
                    st, m = s["state"].get(info.fqn), s["meta"].get(info.fqn)
                    if st is None or m is None:
                        continue
                    a, b = max(lo_need, m["param_lo"]), min(hi_need, m["param_lo"] + m["numel"])
                    for k, v in st.items():
                        if torch.is_tensor(v) and v.dim() > 0:
                            dst = new.setdefault(k, torch.zeros(hi_need - lo_need, dtype=torch.float32))
                            if b > a:
                                dst[a - lo_need : b - lo_need].copy_(v[a - m["param_lo"] : b - m["param_lo"]])
                        else:
                            new[k] = v.clone() if torch.is_tensor(v) else v
                if new:
                    opt.state[info.shard_param] = {k: (v.to(eng.device) if torch.is_tensor(v) and v.dim() > 0 else v) for k, v in new.items()}
        if saved:
            for g, gs in zip(opt.param_groups, saved[0]["param_groups"]):
                for k, v in gs.items():
                    if k != "params":
                        g[k] = v
    _barrier()


def merge_fsdp_weights(checkpoint_dir: str, output_path: str, safe_serialization: bool = True, remove_checkpoint_dir: bool = False):
    """Merge a SHARDED_STATE_DICT model dir into a single weights file (reference fsdp_utils.py:366-418)."""
    pieces = _read_sharded_dir(checkpoint_dir)
    if not pieces:
        raise ValueError(f"No shards found in {checkpoint_dir}")
    full = OrderedDict()
    for tensors, meta in pieces:
        for fqn, pm in meta["params"].items():
            if fqn not in full:
                shape = pm["shape"]
                n = 1
                for s in shape:
                    n *= s
                full[fqn] = (torch.zeros(n, dtype=tensors[fqn].dtype), shape)
            buf, _ = full[fqn]
            if pm["numel"] > 0:
                buf[pm["param_lo"] : pm["param_lo"] + pm["numel"]].copy_(tensors[fqn])
    sd = OrderedDict((k, v.view(shape)) for k, (v, shape) in full.items())
    os.makedirs(output_path, exist_ok=True)
    if safe_serialization:
        from safetensors.torch import save_file

        path = os.path.join(output_path, SAFE_WEIGHTS_NAME)
        save_file(dict(sd), path, metadata={"format": "pt"})
    else:
        path = os.path.join(output_path, WEIGHTS_NAME)
        torch.save(sd, path)
    if remove_checkpoint_dir:
        import shutil

        shutil.rmtree(checkpoint_dir)
    logger.info(f"Merged weights written to {path}")
    return path
