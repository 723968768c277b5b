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
from .async_checkpoint import writer as async_writer
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


# bytes of tensor data this process read from checkpoint files (sharded / full loads): the per-rank IO bound test
# (tests/test_multiprocess_cpu.py::test_fsdp_checkpoint_io_is_per_rank_bounded) reads and resets it
IO_STATS = {"bytes_read": 0}


def _count(t: torch.Tensor) -> torch.Tensor:
    IO_STATS["bytes_read"] += t.numel() * t.element_size()
    return t


def _tp_info(eng):
    group, size = eng._tp_group() if hasattr(eng, "_tp_group") else (None, 1)
    return (dist.get_rank(group) if size > 1 else 0), size


def _shard_stem(eng):
    """File stem of this rank's shard: `shard_{dp_shard rank}`, plus `_tp{t}` when tensor parallel ranks hold
    different slices of the same FSDP shard position."""
    t, tp = _tp_info(eng)
    return f"shard_{eng.rank}" + (f"_tp{t}" if tp > 1 else "")


def save_fsdp_model(fsdp_plugin, accelerator, model, output_dir, model_index=0, adapter_only=False):
    os.makedirs(output_dir, exist_ok=True)
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        sd = eng.full_state_dict(rank0_only=True)  # gathered unit by unit; only rank 0 keeps host copies
        if _rank() == 0:
            name = f"{FSDP_MODEL_NAME}.bin" if model_index == 0 else f"{FSDP_MODEL_NAME}_{model_index}.bin"
            path = os.path.join(output_dir, name)
            torch.save(sd, path)
            logger.info(f"Model saved to {path}")
    else:
        ckpt_dir = os.path.join(output_dir, f"{FSDP_MODEL_NAME}_{model_index}")
        os.makedirs(ckpt_dir, exist_ok=True)
        if getattr(eng, "replicate_rank", 0) != 0:  # HSDP / NO_SHARD replicas hold identical shards: replica 0 writes
            _barrier()
            return
        # device views of the live shards: the non-blocking writer snapshots them in HBM and streams them to the file
        # (utils/async_checkpoint.py); CPU shards are written synchronously in the same safetensors layout
        shard = eng.sharded_state_dict(to_cpu=False)
        t, tp = _tp_info(eng)
        shard["meta"].update(tp_rank=t, tp_size=tp)
        stem = _shard_stem(eng)
        async_writer().save_file({k: v.contiguous() for k, v in shard["tensors"].items()},
                                 os.path.join(ckpt_dir, f"{stem}.safetensors"))
        with open(os.path.join(ckpt_dir, stem.replace("shard_", "meta_") + ".json"), "w") as f:
            json.dump(shard["meta"], f)
        logger.info(f"Model shard saved to {ckpt_dir}")
    _barrier()


def _saved_metas(ckpt_dir, tp_rank=None):
    """[(shard file, meta)] of a sharded model dir, from the small JSON files only (no tensor data read). With
    `tp_rank`, only the shards written by that tensor-parallel rank."""
    out = []
    for meta_path in sorted(glob.glob(os.path.join(ckpt_dir, "meta_*.json"))):
        with open(meta_path) as f:
            meta = json.load(f)
        if tp_rank is not None and meta.get("tp_size", 1) > 1 and meta.get("tp_rank", 0) != tp_rank:
            continue
        stem = os.path.basename(meta_path)[len("meta_") : -len(".json")]
        out.append((os.path.join(ckpt_dir, f"shard_{stem}.safetensors"), meta))
    return out


def _check_tp_layout(metas, eng, what):
    """A sharded checkpoint holds TP-local slices: it loads only into the same tensor-parallel layout."""
    _, tp = _tp_info(eng)
    saved = {m.get("tp_size", 1) if "tp_size" in m else m.get("meta", {}).get("tp_size", 1) for _, m in metas}
    saved = {s for s in saved if s is not None} or {1}
    if saved != {tp}:
        raise ValueError(f"{what} was saved with tensor-parallel size {sorted(saved)} and is being loaded with tp={tp}: "
                         "a sharded checkpoint holds TP-local slices. Merge it (`merge_fsdp_weights` / "
                         "`accelerate merge-weights`) and load the full weights instead.")


def _read_sharded_dir(ckpt_dir):
    """Every saved shard in full: (tensors, meta) per saved rank (the merge tool; loads use `_load_sharded_model`)."""
    from safetensors.torch import load_file

    return [(load_file(path), meta) for path, meta in _saved_metas(ckpt_dir)]


class _ShardReader:
    """Lazily opened safetensors shards; `read(path, key, a, b)` returns elements [a, b) of a 1-D tensor through the
    file's mmap, so only the overlapping byte range is read."""

    def __init__(self):
        self.handles = {}

    def read(self, path, key, a=None, b=None):
        from safetensors import safe_open

        h = self.handles.get(path)
        if h is None:
            h = self.handles[path] = safe_open(path, framework="pt")
        sl = h.get_slice(key)
        return _count(sl[a:b] if a is not None else sl[:])

    def shape(self, path, key):
        from safetensors import safe_open

        h = self.handles.get(path)
        if h is None:
            h = self.handles[path] = safe_open(path, framework="pt")
        return tuple(h.get_slice(key).get_shape())


@torch.no_grad()
def _load_sharded_model(eng, ckpt_dir):
    """SHARDED_STATE_DICT load that reads only the saved pieces overlapping this rank's flat slice (reference: DCP's
    planned per-rank reads, /root/reference/src/accelerate/utils/fsdp_utils.py:221-225). Same world size: one file
    per rank; any other world size: the few files whose [param_lo, param_lo + numel) ranges intersect."""
    t, _ = _tp_info(eng)
    metas = _saved_metas(ckpt_dir, tp_rank=t)
    if not metas:
        raise FileNotFoundError(f"No model shards in {ckpt_dir}")
    _check_tp_layout(metas, eng, f"The sharded model in {ckpt_dir}")
    rd = _ShardReader()
    for unit in eng.units:
        for info in unit.infos:
            lo_need, hi_need = info.param_lo, info.param_lo + (info.local_hi - info.local_lo)
            if hi_need <= lo_need:
                continue
            for path, meta in metas:
                pm = meta["params"].get(info.fqn)
                if pm is None or pm["numel"] <= 0:
                    continue
                s_lo = pm["param_lo"]
                a, b = max(lo_need, s_lo), min(hi_need, s_lo + pm["numel"])
                if b > a:
                    src = rd.read(path, info.fqn, a - s_lo, b - s_lo)
                    unit.master[info.local_lo + (a - lo_need) : info.local_lo + (b - lo_need)].copy_(src.to(unit.master.device))
        if unit.shard_lp is not unit.master:
            unit.shard_lp.copy_(unit.master.to(unit.shard_lp.device))
    eng.refresh_fp8()
    for name, p in eng._extras():
        found = [(path, m["extra"][name]) for path, m in metas if name in m.get("extra", {})]
        if not found:
            continue
        if not found[0][1]["ep"]:
            p.copy_(rd.read(found[0][0], name).to(p.device, p.dtype))
            continue
        # expert-parallel stack: this rank's rows [r n, (r + 1) n) of the saved ranks' stacks in rank order
        group, W = p._ep_spec
        n = p.shape[0]
        lo = dist.get_rank(group) * n
        pos = 0
        for path, em in sorted(found, key=lambda x: x[1]["rank"]):
            rows = rd.shape(path, name)[0]
            a, b = max(lo, pos), min(lo + n, pos + rows)
            if b > a:
                p[a - lo : b - lo].copy_(rd.read(path, name, a - pos, b - pos).to(p.device, p.dtype))
            pos += rows


@torch.no_grad()
def _load_full_model_rank0(eng, path):
    """FULL_STATE_DICT load: global rank 0 reads the file (memory-mapped), every unit reaches the other ranks as one
    broadcast of its flat fp32 buffer (reference fsdp2_load_full_state_dict: rank 0 reads, broadcasts,
    /root/reference/src/accelerate/utils/fsdp_utils.py:467-554)."""
    sd = None
    if _rank() == 0:
        sd = torch.load(path, map_location="cpu", weights_only=True, mmap=True)
    eng.load_full_state_dict_broadcast(sd)


def load_fsdp_model(fsdp_plugin, accelerator, model, input_dir, model_index=0, adapter_only=False):
    _barrier()
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        name = f"{FSDP_MODEL_NAME}.bin" if model_index == 0 else f"{FSDP_MODEL_NAME}_{model_index}.bin"
        path = os.path.join(input_dir, name)
        if _tp_info(eng)[1] > 1 or not (dist.is_available() and dist.is_initialized()):
            sd = torch.load(path, map_location="cpu", weights_only=True, mmap=True)  # tp slices: every rank keeps its own
            eng.load_full_state_dict(sd)
        else:
            _load_full_model_rank0(eng, path)
    else:
        ckpt_dir = input_dir if os.path.basename(os.path.normpath(input_dir)).startswith(FSDP_MODEL_NAME) else os.path.join(input_dir, f"{FSDP_MODEL_NAME}_{model_index}")
        _load_sharded_model(eng, ckpt_dir)
    _barrier()


# ---------------------------------------------------------------------------------------------- optimizer
def _optim_full_state(eng, optimizer):
    """Gather optimizer state into {fqn: {key: full tensor}} (one all-gather per unit per state key); only global rank
    0 keeps host copies."""
    opt = getattr(optimizer, "optimizer", optimizer)
    keep = _rank() == 0
    out, step_val = OrderedDict(), None
    for unit in eng.units:
        keys = set()
        for info in unit.infos:
            keys.update(k for k, v in opt.state.get(info.shard_param, {}).items() if torch.is_tensor(v) and v.dim() > 0)
            st = opt.state.get(info.shard_param, {})
            if "step" in st:
                step_val = st["step"]
        keys = _agree_keys(keys)
        for key in keys:
            local = torch.zeros(unit.shard_numel, dtype=torch.float32, device=eng.device)
            for info in unit.infos:
                t = opt.state.get(info.shard_param, {}).get(key)
                if t is not None and info.local_hi > info.local_lo:
                    local[info.local_lo : info.local_hi].copy_(t.reshape(-1).float())
            full = eng.gather_full(unit, local)
            if keep:
                for info in unit.infos:
                    out.setdefault(info.fqn, {})[key] = full[info.offset : info.offset + info.numel].view(info.shape).cpu().clone()
            del full, local
    groups = []
    fqn_of = {id(info.shard_param): info.fqn for unit in eng.units for info in unit.infos}
    for g in opt.param_groups:
        gg = {k: v for k, v in g.items() if k != "params"}
        gg["params"] = [fqn_of.get(id(p)) for p in g["params"]]
        groups.append(gg)
    return {"state": out, "param_groups": groups, "step": step_val}


def _agree_keys(keys):
    """The sorted union of state keys over all ranks (a rank whose shard of a unit is empty has none)."""
    keys = sorted(keys)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        allk = [None] * dist.get_world_size()
        dist.all_gather_object(allk, keys)
        keys = sorted(set().union(*[set(k) for k in allk]))
    return keys


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
    _apply_groups(opt, sd.get("param_groups", []))


def _apply_groups(opt, saved_groups):
    for g, gs in zip(opt.param_groups, saved_groups):
        for k, v in gs.items():
            if k != "params":
                g[k] = v


@torch.no_grad()
def _optim_load_full_rank0(eng, optimizer, path):
    """FULL optimizer load: rank 0 reads the file, each unit's state key is broadcast as one flat fp32 buffer."""
    opt = getattr(optimizer, "optimizer", optimizer)
    sd = torch.load(path, map_location="cpu", weights_only=True, mmap=True) if _rank() == 0 else None
    head = [None]
    if _rank() == 0:
        keys = {fqn: sorted(k for k, v in st.items() if torch.is_tensor(v) and v.dim() > 0) for fqn, st in sd["state"].items()}
        head = [{"keys": keys, "step": sd.get("step"), "param_groups": sd.get("param_groups", [])}]
    dist.broadcast_object_list(head, src=0)
    head = head[0]
    step = head["step"]
    for unit in eng.units:
        ukeys = sorted({k for info in unit.infos for k in head["keys"].get(info.fqn, [])})
        for key in ukeys:
            full = torch.zeros(unit.padded, dtype=torch.float32, device=eng.device)
            if _rank() == 0:
                for info in unit.infos:
                    v = sd["state"].get(info.fqn, {}).get(key)
                    if v is not None:
                        full[info.offset : info.offset + info.numel].copy_(_count(v.reshape(-1)).to(eng.device, torch.float32))
            eng.broadcast_full(full)
            for info in unit.infos:
                if key not in head["keys"].get(info.fqn, []):
                    continue
                st = opt.state.setdefault(info.shard_param, {})
                st[key] = full[info.offset + info.param_lo : info.offset + info.param_lo + (info.local_hi - info.local_lo)].clone()
                if step is not None:
                    st["step"] = torch.as_tensor(step, dtype=torch.float32).clone()
            del full
    _apply_groups(opt, head["param_groups"])


def _jsonable(v):
    if torch.is_tensor(v):
        return {"__tensor__": v.item(), "dtype": str(v.dtype).replace("torch.", "")}
    if isinstance(v, tuple):
        return {"__tuple__": [_jsonable(x) for x in v]}
    if isinstance(v, list):
        return [_jsonable(x) for x in v]
    return v


def _unjson(v):
    if isinstance(v, dict) and "__tensor__" in v:
        return torch.tensor(v["__tensor__"], dtype=getattr(torch, v["dtype"]))
    if isinstance(v, dict) and "__tuple__" in v:
        return tuple(_unjson(x) for x in v["__tuple__"])
    if isinstance(v, list):
        return [_unjson(x) for x in v]
    return v


def save_fsdp_optimizer(fsdp_plugin, accelerator, optimizer, model, output_dir, optimizer_index=0):
    os.makedirs(output_dir, exist_ok=True)
    eng = _engine(model)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        sd = _optim_full_state(eng, optimizer)
        if _rank() == 0:
            name = f"{OPTIMIZER_NAME}.bin" if optimizer_index == 0 else f"{OPTIMIZER_NAME}_{optimizer_index}.bin"
            torch.save(sd, os.path.join(output_dir, name))
    else:
        # one safetensors file of this rank's 1-D state pieces ("{fqn}|{key}") + a JSON of their ranges, the scalar
        # states and the param groups: loads read only the overlapping byte ranges, like the model shards
        d = os.path.join(output_dir, f"{OPTIMIZER_NAME}_{optimizer_index}")
        os.makedirs(d, exist_ok=True)
        opt = getattr(optimizer, "optimizer", optimizer)
        tensors, meta, scalars = {}, {}, {}
        for unit in eng.units:
            for info in unit.infos:
                st = opt.state.get(info.shard_param) or {}
                keys = []
                for k, v in st.items():
                    if torch.is_tensor(v) and v.dim() > 0:  # stored in its own dtype (bf16 moments stay bf16)
                        tensors[f"{info.fqn}|{k}"] = v.detach().reshape(-1).contiguous()
                        keys.append(k)
                    else:
                        scalars.setdefault(info.fqn, {})[k] = _jsonable(v)
                meta[info.fqn] = {"param_lo": info.param_lo, "numel": info.local_hi - info.local_lo, "keys": keys}
        fqn_of = {id(info.shard_param): info.fqn for unit in eng.units for info in unit.infos}
        groups = [{**{k: _jsonable(v) for k, v in g.items() if k != "params"}, "params": [fqn_of.get(id(p)) for p in g["params"]]}
                  for g in opt.param_groups]
        if getattr(eng, "replicate_rank", 0) == 0:  # replicas hold identical optimizer shards
            t, tp = _tp_info(eng)
            stem = _shard_stem(eng)
            async_writer().save_file(tensors, os.path.join(d, f"{stem}.safetensors"))
            with open(os.path.join(d, stem.replace("shard_", "meta_") + ".json"), "w") as f:
                json.dump({"meta": meta, "scalars": scalars, "param_groups": groups, "tp_rank": t, "tp_size": tp}, f)
    _barrier()


@torch.no_grad()
def _load_sharded_optimizer(eng, opt, d):
    t, _ = _tp_info(eng)
    metas = _saved_metas(d, tp_rank=t)
    if metas:
        _check_tp_layout(metas, eng, f"The sharded optimizer in {d}")
    rd = _ShardReader()
    for unit in eng.units:
        for info in unit.infos:
            lo_need, hi_need = info.param_lo, info.param_lo + (info.local_hi - info.local_lo)
            new, keys = {}, set()
            for path, m in metas:
                pm = m["meta"].get(info.fqn)
                if pm is None:
                    continue
                keys.update(pm["keys"])
                for k, v in m["scalars"].get(info.fqn, {}).items():
                    new.setdefault(k, _unjson(v))
                a, b = max(lo_need, pm["param_lo"]), min(hi_need, pm["param_lo"] + pm["numel"])
                for k in pm["keys"]:
                    if b <= a:
                        continue
                    src = rd.read(path, f"{info.fqn}|{k}", a - pm["param_lo"], b - pm["param_lo"])
                    dst = new.setdefault(k, torch.zeros(hi_need - lo_need, dtype=src.dtype))
                    dst[a - lo_need : b - lo_need].copy_(src)
            for k in keys - set(new):  # an empty local piece: nothing to read
                new[k] = torch.zeros(hi_need - lo_need, dtype=torch.float32)
            if new:
                opt.state[info.shard_param] = {k: (v.to(eng.device) if torch.is_tensor(v) and v.dim() > 0 else v) for k, v in new.items()}
    if metas:
        _apply_groups(opt, [{k: _unjson(v) for k, v in g.items()} for g in metas[0][1]["param_groups"]])


def load_fsdp_optimizer(fsdp_plugin, accelerator, optimizer, model, input_dir, optimizer_index=0, adapter_only=False):
    _barrier()
    eng = _engine(model)
    opt = getattr(optimizer, "optimizer", optimizer)
    if fsdp_plugin.state_dict_type == "FULL_STATE_DICT":
        name = f"{OPTIMIZER_NAME}.bin" if optimizer_index == 0 else f"{OPTIMIZER_NAME}_{optimizer_index}.bin"
        path = os.path.join(input_dir, name)
        if _tp_info(eng)[1] > 1 or not (dist.is_available() and dist.is_initialized()):
            _optim_load_full(eng, optimizer, torch.load(path, map_location="cpu", weights_only=True, mmap=True))
        else:
            _optim_load_full_rank0(eng, optimizer, path)
    else:
        d = input_dir if os.path.basename(os.path.normpath(input_dir)).startswith(OPTIMIZER_NAME) else os.path.join(input_dir, f"{OPTIMIZER_NAME}_{optimizer_index}")
        if glob.glob(os.path.join(d, "meta_*.json")):
            _load_sharded_optimizer(eng, opt, d)
        else:
            _load_sharded_optimizer_v1(eng, opt, d)
    _barrier()


def _load_sharded_optimizer_v1(eng, opt, d):
    """Round-4 layout (`shard_{rank}.pt` holding every piece): read in full."""
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
        _apply_groups(opt, saved[0]["param_groups"])


def _unshard_tp_host(parts, dim, segments):
    """Full tensor from the tp ranks' local slices (rank order): each fused segment was split tp ways on its own
    (parallel/tensor_parallel.py `_shard_tensor`), so the pieces are re-interleaved segment by segment."""
    tp = len(parts)
    local = parts[0].shape[dim]
    segs = [s // tp for s in segments] if segments else [local]
    out, off = [], 0
    for s in segs:
        out += [p.narrow(dim, off, s) for p in parts]
        off += s
    return torch.cat(out, dim=dim)


def merge_fsdp_weights(checkpoint_dir: str, output_path: str, safe_serialization: bool = True, remove_checkpoint_dir: bool = False):
    """Merge a SHARDED_STATE_DICT model dir into a single weights file (reference fsdp_utils.py:366-418). FSDP pieces
    are placed by their flat offsets per tensor-parallel rank; with tp > 1 the TP-local tensors are then concatenated
    along each parameter's recorded shard dim (replicated parameters come from tp rank 0); expert-parallel stacks
    (engine extras) are concatenated in rank order."""
    from .async_checkpoint import wait_pending_saves

    wait_pending_saves()  # this process's own non-blocking save may still be writing into the directory
    pieces = _read_sharded_dir(checkpoint_dir)
    if not pieces:
        raise ValueError(f"No shards found in {checkpoint_dir}")
    tp_size = max(meta.get("tp_size", 1) for _, meta in pieces)
    by_tp = {}
    for tensors, meta in pieces:
        by_tp.setdefault(meta.get("tp_rank", 0) if tp_size > 1 else 0, []).append((tensors, meta))
    if sorted(by_tp) != list(range(tp_size)):
        raise ValueError(f"{checkpoint_dir}: shards of tp ranks {sorted(by_tp)} found, expected 0..{tp_size - 1}")
    local = {}
    for t, group in by_tp.items():
        full = OrderedDict()
        for tensors, meta in group:
            for fqn, pm in meta["params"].items():
                if fqn not in full:
                    shape = pm["shape"]
                    n = 1
                    for s_ in shape:
                        n *= s_
                    full[fqn] = (torch.zeros(n, dtype=tensors[fqn].dtype), shape, pm.get("tp"))
                buf = full[fqn][0]
                if pm["numel"] > 0:
                    buf[pm["param_lo"] : pm["param_lo"] + pm["numel"]].copy_(tensors[fqn])
        local[t] = full
    merged = OrderedDict()
    for fqn, (buf, shape, tpm) in local[0].items():
        if tp_size == 1 or tpm is None:
            merged[fqn] = buf.view(shape)
        else:
            merged[fqn] = _unshard_tp_host([local[t][fqn][0].view(local[t][fqn][1]) for t in range(tp_size)],
                                           tpm["dim"], tpm.get("segments"))
    # engine extras (ignored / expert-parallel parameters): replicated ones once, EP stacks in rank order
    ext_pieces = sorted(((meta.get("rank", 0), tensors, meta) for tensors, meta in by_tp[0]), key=lambda x: x[0])
    for _, tensors, meta in ext_pieces:
        for name, em in meta.get("extra", {}).items():
            if em.get("ep"):
                merged[name] = torch.cat([merged[name], tensors[name]]) if name in merged else tensors[name]
            elif name not in merged:
                merged[name] = tensors[name]
    sd = merged
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
