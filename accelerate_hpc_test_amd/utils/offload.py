"""Weight stores for offloaded big-model layers: a folder of raw tensor files on disk, and name-keyed views over
host state dicts / safetensors shards.

On-disk format (compatible with the reference's offload folders, `/root/reference/src/accelerate/utils/offload.py`):
one file `<name>.dat` per tensor holding its raw C-order bytes (numpy-memmap layout, no header; 0-d tensors stored as
one element), and `index.json` mapping each name to `{"dtype", "shape"}`. Types numpy lacks are stored as same-width
integers and named in the index: bfloat16 as int16 bits ("bfloat16"), fp8 as uint8 bits ("float8_e4m3fn" /
"float8_e5m2"). Index entries may instead point into a safetensors shard (`{"safetensors_file", "weight_name"}`),
which is read tensor by tensor (`safe_open`), never whole.

`TensorStore` is the folder; the module-level functions (`offload_weight`, `load_offloaded_weight`,
`save_offload_index`, `offload_state_dict`) and `OffloadedWeightsLoader` / `PrefixedDataset` are the reference's API
on top of it.
"""

from __future__ import annotations

import json
import os
from collections.abc import Mapping
from typing import Optional, Union

import numpy as np
import torch

# torch dtypes numpy cannot represent -> (index name, same-width integer used for the bits)
_BIT_TYPES = {
    torch.bfloat16: ("bfloat16", torch.int16),
    torch.float8_e4m3fn: ("float8_e4m3fn", torch.uint8),
    torch.float8_e5m2: ("float8_e5m2", torch.uint8),
}
_BY_NAME = {name: (dt, carrier) for dt, (name, carrier) in _BIT_TYPES.items()}


def _to_numpy(t: torch.Tensor) -> tuple[np.ndarray, str]:
    t = t.detach().cpu().contiguous()
    if t.dtype in _BIT_TYPES:
        name, carrier = _BIT_TYPES[t.dtype]
        return t.view(carrier).numpy(), name
    arr = t.numpy()
    return arr, str(arr.dtype)


class TensorStore:
    """A directory of raw tensor files plus `index.json` (see module docstring)."""

    INDEX = "index.json"

    def __init__(self, folder: Union[str, os.PathLike], index: Optional[dict] = None):
        self.folder = str(folder)
        if index is None:
            path = os.path.join(self.folder, self.INDEX)
            index = json.load(open(path, encoding="utf-8")) if os.path.isfile(path) else {}
        self.index = index

    def path(self, name: str) -> str:
        return os.path.join(self.folder, f"{name}.dat")

    def write(self, name: str, tensor: torch.Tensor) -> dict:
        arr, dtype_name = _to_numpy(tensor)
        entry = {"dtype": dtype_name, "shape": list(arr.shape)}
        os.makedirs(self.folder, exist_ok=True)
        np.ascontiguousarray(arr.reshape(-1) if arr.ndim else arr.reshape(1)).tofile(self.path(name))
        self.index[name] = entry
        return entry

    def read(self, name: str, entry: Optional[dict] = None, device=None) -> torch.Tensor:
        entry = entry if entry is not None else self.index[name]
        if entry.get("safetensors_file") is not None:
            from safetensors import safe_open

            with safe_open(entry["safetensors_file"], framework="pt", device=str(device or "cpu")) as f:
                t = f.get_tensor(entry.get("weight_name", name))
            return t.to(getattr(torch, entry["dtype"])) if "dtype" in entry else t
        return read_raw(self.path(name), entry)

    def flush_index(self):
        if not self.index:
            return
        path = os.path.join(self.folder, self.INDEX)
        merged = json.load(open(path, encoding="utf-8")) if os.path.isfile(path) else {}
        merged.update(self.index)
        os.makedirs(self.folder, exist_ok=True)
        with open(path, "w", encoding="utf-8") as f:
            json.dump(merged, f, indent=2)


def read_raw(path: str, entry: dict) -> torch.Tensor:
    """One `.dat` file back as a CPU tensor (memory-mapped read, one copy into a fresh tensor)."""
    shape = tuple(entry["shape"])
    name = entry["dtype"]
    dt, carrier = _BY_NAME.get(name, (None, None))
    np_dtype = np.dtype(str(carrier).replace("torch.", "")) if carrier is not None else np.dtype(name)
    mm = np.memmap(path, dtype=np_dtype, mode="r", shape=shape if shape else (1,))
    out = torch.from_numpy(np.array(mm))  # np.array copies out of the mapping: the result is writable
    if not shape:
        out = out.reshape(())
    return out.view(dt) if dt is not None else out


# ------------------------------------------------------------------------------------------ reference-named API
def offload_weight(weight: torch.Tensor, weight_name: str, offload_folder: str, index: Optional[dict] = None):
    entry = TensorStore(offload_folder, index={}).write(weight_name, weight)
    if index is not None:
        index[weight_name] = entry
    return index


def load_offloaded_weight(weight_file: str, weight_info: dict) -> torch.Tensor:
    return read_raw(weight_file, weight_info)


def save_offload_index(index: Optional[dict], offload_folder: str):
    if index:
        TensorStore(offload_folder, index=dict(index)).flush_index()


def offload_state_dict(save_dir: Union[str, os.PathLike], state_dict: dict):
    store = TensorStore(save_dir, index={})
    for name, t in state_dict.items():
        store.write(name, t)
    store.flush_index()


class PrefixedDataset(Mapping):
    """The entries of `dataset` under `prefix`, addressed without it."""

    def __init__(self, dataset: Mapping, prefix: str):
        self.dataset = dataset
        self.prefix = prefix

    def __getitem__(self, key):
        return self.dataset[self.prefix + key]

    def __iter__(self):
        return (k for k in self.dataset if k.startswith(self.prefix))

    def __len__(self):
        return len(self.dataset)


class OffloadedWeightsLoader(Mapping):
    """Name -> CPU tensor over (in priority order) a host state dict and a `TensorStore` folder / index; tensors
    are read from disk on access only."""

    def __init__(self, state_dict: Optional[dict] = None, save_folder=None, index: Optional[Mapping] = None, device=None):
        if state_dict is None and save_folder is None and index is None:
            raise ValueError("Need either a `state_dict`, a `save_folder` or an `index` containing offloaded weights.")
        self.state_dict = state_dict or {}
        self.save_folder = save_folder
        if index is None and save_folder is None:
            index = {}
        self.store = TensorStore(save_folder if save_folder is not None else "", index=dict(index) if index is not None else None)
        self.index = self.store.index
        self.device = device
        self.all_keys = list(self.state_dict) + [k for k in self.index if k not in self.state_dict]

    def __getitem__(self, key: str):
        if key in self.state_dict:
            return self.state_dict[key]
        return self.store.read(key, self.index[key], device=self.device)

    def __iter__(self):
        return iter(self.all_keys)

    def __len__(self):
        return len(self.all_keys)


def extract_submodules_state_dict(state_dict: dict, submodule_names: list) -> dict:
    """The entries of `state_dict` that belong to one of `submodule_names` (the name itself or below it)."""
    wanted = tuple(submodule_names)
    return {k: v for k, v in state_dict.items() if any(k == m or k.startswith(m + ".") for m in wanted)}
