"""Reading (sharded) checkpoints into models, one tensor at a time.

Reference behaviour: `/root/reference/src/accelerate/utils/modeling.py:1620-1712,1788-2046` (`load_state_dict`,
`load_checkpoint_in_model` incl. `broadcast_from_rank0` at `:1934-1953`). Design here:

* **Streaming.** A safetensors shard is opened with `safe_open` and read tensor by tensor (`SafetensorsShard`, a
  lazy mapping), so peak host memory is one tensor, not one shard — what makes 70B-class loading fit.
* **MI355X upload path.** Tensors bound for a GPU go through the native `H2DEngine` (csrc/runtime/h2d_engine.cpp):
  worker threads copy the (memory-mapped, pageable) bytes into a pinned ring and DMA them on the engine's own HIP
  stream, overlapping file reads, host copies and PCIe; one wait at the end orders the compute stream after them.
* **broadcast_from_rank0.** Only rank 0 touches the files. It broadcasts the key list once, then each tensor (over
  RCCL for GPU models, gloo for host models); every rank installs it — into its FSDP shard when the model is sharded
  by the native engine (`FullyShardedModule`), or as the full tensor otherwise.
"""

from __future__ import annotations

import gc
import json
import logging
import os
import shutil
import tempfile
from collections.abc import Mapping
from typing import Optional, Union

import torch
import torch.nn as nn

from .constants import SAFE_WEIGHTS_INDEX_NAME, SAFE_WEIGHTS_NAME, WEIGHTS_INDEX_NAME, WEIGHTS_NAME
from .device_map import find_tied_parameters
from .offload import TensorStore
from .placement import recursive_getattr, retie_parameters, set_module_tensor_to_device

logger = logging.getLogger(__name__)


# ------------------------------------------------------------------------------------------------ files
def checkpoint_files(checkpoint: Union[str, os.PathLike]) -> list:
    """The weight files of a checkpoint given as a file, an `*.index.json`, or a folder holding either."""
    checkpoint = str(checkpoint)
    if os.path.isfile(checkpoint):
        if not checkpoint.endswith(".json"):
            return [checkpoint]
        index = json.load(open(checkpoint, encoding="utf-8"))
        index = index.get("weight_map", index)
        folder = os.path.dirname(checkpoint)
        return sorted({os.path.join(folder, f) for f in index.values()})
    if os.path.isdir(checkpoint):
        for name in (SAFE_WEIGHTS_INDEX_NAME, WEIGHTS_INDEX_NAME):
            if os.path.isfile(os.path.join(checkpoint, name)):
                return checkpoint_files(os.path.join(checkpoint, name))
        for name in (SAFE_WEIGHTS_NAME, WEIGHTS_NAME):
            if os.path.isfile(os.path.join(checkpoint, name)):
                return [os.path.join(checkpoint, name)]
        indexes = [f for f in os.listdir(checkpoint) if f.endswith(".index.json")]
        if len(indexes) == 1:
            return checkpoint_files(os.path.join(checkpoint, indexes[0]))
        if len(indexes) > 1:
            raise ValueError(f"{checkpoint} containing more than one `.index.json` file, delete the irrelevant ones.")
        weights = [f for f in os.listdir(checkpoint) if f.endswith((".safetensors", ".bin"))]
        if len(weights) == 1:
            return [os.path.join(checkpoint, weights[0])]
        raise ValueError(f"{checkpoint} is not a folder containing a `.index.json` file or a {WEIGHTS_NAME} or a {SAFE_WEIGHTS_NAME} file")
    raise ValueError(
        "`checkpoint` should be the path to a file containing a whole state dict, or the index of a sharded checkpoint, "
        f"or a folder containing a sharded checkpoint or the whole state dict, but got {checkpoint}."
    )


_ST_DTYPES = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
              "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
              "BOOL": torch.bool, "F8_E4M3": torch.float8_e4m3fn, "F8_E5M2": torch.float8_e5m2}


class SafetensorsShard(Mapping):
    """Lazy name -> CPU tensor view of one safetensors file (one `get_tensor` per access)."""

    def __init__(self, path: str):
        from safetensors import safe_open

        self.path = path
        self._f = safe_open(path, framework="pt", device="cpu")
        self._keys = list(self._f.keys())
        meta = self._f.metadata() or {}
        if meta.get("format") not in (None, "pt", "flax", "np", "tf", "mlx"):
            raise OSError(f"The safetensors archive passed at {path} does not contain valid metadata.")

    def __getitem__(self, key):
        if key not in self._keys:
            raise KeyError(key)
        return self._f.get_tensor(key)

    def layout(self) -> dict:
        """name -> (torch dtype, shape, absolute byte offset, byte length) of every tensor, from the file's own header
        (8-byte little-endian header length, JSON header, data section): what lets the native engine pread a tensor's
        bytes straight into its pinned ring (`H2DEngine.copy_file`) without materialising a host tensor."""
        if getattr(self, "_layout", None) is None:
            with open(self.path, "rb") as fh:
                n = int.from_bytes(fh.read(8), "little")
                header = json.loads(fh.read(n))
            base = 8 + n
            out = {}
            for name, info in header.items():
                if name == "__metadata__":
                    continue
                dt = _ST_DTYPES.get(info["dtype"])
                lo, hi = info["data_offsets"]
                if dt is not None:
                    out[name] = (dt, tuple(info["shape"]), base + lo, hi - lo)
            self._layout = out
        return self._layout

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)


def load_state_dict(checkpoint_file: str, device_map: Optional[dict] = None):
    """One weight file as a name -> CPU tensor mapping: lazy (per-tensor reads) for safetensors, eager
    (`torch.load(weights_only=True)`) for pickled `.bin` files."""
    if str(checkpoint_file).endswith(".safetensors"):
        return SafetensorsShard(str(checkpoint_file))
    return torch.load(checkpoint_file, map_location="cpu", weights_only=True)


# ------------------------------------------------------------------------------------------------ loading
def _device_of(name: str, device_map: dict):
    probe = name
    while probe and probe not in device_map:
        probe = probe.rpartition(".")[0]
    if probe == "" and "" not in device_map:
        raise ValueError(f"{name} doesn't have any device set.")
    return device_map[probe]


_ENGINES = {}


def h2d_engine(device_index: int):
    """The shared native async H2D engine of a GPU (None without the extension)."""
    from ..ops import _ext

    if not _ext.available():
        return None
    if device_index not in _ENGINES:
        # 8 x 64 MB pinned slots, 8 worker threads: parallel pread / memcpy into the ring keeps PCIe Gen5 busy
        _ENGINES[device_index] = _ext.ext().H2DEngine(device_index, 8, 64 << 20, 8)
    return _ENGINES[device_index]


class _Installer:
    """Places checkpoint tensors one by one according to a device map (GPU through the H2D engine, host, or an
    offload folder) and finishes the deferred work at the end."""

    def __init__(self, model, device_map, dtype, keep_in_fp32_modules, offload_folder, offload_state_dict, offload_buffers, strict):
        self.model = model
        self.device_map = device_map
        self.dtype = getattr(torch, dtype.replace("torch.", "")) if isinstance(dtype, str) else dtype
        self.keep_fp32 = keep_in_fp32_modules
        self.strict = strict
        self.offload_buffers = offload_buffers
        self.disk = TensorStore(offload_folder, index={}) if offload_folder is not None else None
        self.host_spill = TensorStore(tempfile.mkdtemp(), index={}) if offload_state_dict else None
        self.buffer_names = {n for n, _ in model.named_buffers()}
        self.keys = set(model.state_dict().keys())
        self.unexpected = set()
        self.engines = set()
        # file-range uploads (safetensors -> pinned ring by pread -> HBM); ACCELERATE_LOAD_DIRECT=0 reads through
        # safetensors' own get_tensor instead
        self.direct = os.environ.get("ACCELERATE_LOAD_DIRECT", "1") != "0"

    def target_dtype(self, name, t):
        if self.dtype is None or not torch.is_floating_point(t):
            return None
        if self.keep_fp32 is not None and self.dtype == torch.float16 and any(
            (k in name and k + "." in name) or k == name for k in self.keep_fp32
        ):
            return torch.float32
        return self.dtype

    def put_from_file(self, name, path: str, dtype, shape, offset: int, nbytes: int) -> bool:
        """A GPU-bound tensor stored in the checkpoint with the dtype it keeps: the engine preads its bytes from the
        shard straight into the pinned ring and DMAs them (no host tensor). False when this path does not apply."""
        if name not in self.keys or not self.direct:
            return False
        dest = _device_of(name, self.device_map)
        if isinstance(dest, int):
            dev = torch.device("cuda", dest)
        elif isinstance(dest, (str, torch.device)) and str(dest).startswith("cuda"):
            dev = torch.device(dest)
        else:
            return False  # host / disk placements keep the tensor path
        old = recursive_getattr(self.model, name)
        # the installed tensor must come out of the DMA in its final dtype: a cast inside set_module_tensor_to_device
        # would read `dst` on the current stream before the engine's copy has landed
        want = self.target_dtype(name, torch.empty(0, dtype=dtype)) or old.dtype
        if want != dtype or tuple(old.shape) != tuple(shape) or nbytes != torch.Size(shape).numel() * dtype.itemsize:
            return False
        eng = h2d_engine(dev.index if dev.index is not None else torch.cuda.current_device())
        if eng is None or not hasattr(eng, "copy_file"):
            return False
        dst = torch.empty(shape, dtype=dtype, device=dev)
        if nbytes:
            eng.copy_file(path, offset, dst)
        self.engines.add(eng)
        set_module_tensor_to_device(self.model, name, dev, value=dst, dtype=want, clear_cache=False)
        return True

    def put(self, name, t):
        if name not in self.keys:
            self.unexpected.add(name)
            if not self.strict:
                return
        dest = _device_of(name, self.device_map)
        dt = self.target_dtype(name, t)
        if dest == "disk":
            # a buffer of a disk block stays unplaced unless buffers are offloaded too (upstream behaviour)
            if self.offload_buffers or name not in self.buffer_names:
                set_module_tensor_to_device(self.model, name, "meta", dtype=dt or t.dtype)
                self.disk.write(name, t)
            return
        if dest == "cpu" and self.host_spill is not None:
            set_module_tensor_to_device(self.model, name, "meta", dtype=dt or t.dtype)
            self.host_spill.write(name, t)
            return
        dev = torch.device("cuda", dest) if isinstance(dest, int) else torch.device(dest)
        if dev.type == "cuda" and t.is_contiguous():
            eng = h2d_engine(dev.index if dev.index is not None else torch.cuda.current_device())
            if eng is not None:
                old = recursive_getattr(self.model, name)
                # convert on the host so `dst` needs no cast after the (asynchronous) DMA: a cast here would read
                # it on the current stream before the engine's copy has landed
                final = dt if dt is not None else old.dtype
                src = t.to(final)
                dst = torch.empty(src.shape, dtype=final, device=dev)
                eng.copy(src.contiguous(), dst)
                self.engines.add(eng)
                set_module_tensor_to_device(self.model, name, dev, value=dst, dtype=final, clear_cache=False)
                return
        set_module_tensor_to_device(self.model, name, dest, value=t, dtype=dt, clear_cache=False)

    def release(self):
        """Close every shard file the engines opened and return the short-read count (reset in the engine); safe to
        call on an error path (the `finally` of `load_checkpoint_in_model`)."""
        errors = 0
        for eng in self.engines:
            if hasattr(eng, "close_files"):
                try:
                    eng.wait_on_current_stream()
                finally:
                    errors += int(eng.close_files() or 0)
        return errors

    def finish(self):
        for eng in self.engines:
            eng.wait_on_current_stream()
        errors = self.release()
        self.engines = set()
        if errors:
            raise OSError(f"checkpoint loading: {errors} short read(s) from the shard files")
        if self.disk is not None:
            self.disk.flush_index()
        if self.host_spill is not None:
            for name, entry in self.host_spill.index.items():
                set_module_tensor_to_device(self.model, name, "cpu", value=self.host_spill.read(name, entry))
            shutil.rmtree(self.host_spill.folder, ignore_errors=True)


def _broadcast_stream(model: nn.Module, files: list, strict: bool):
    """broadcast_from_rank0: rank 0 reads, every rank installs (full tensors, or FSDP shards)."""
    import torch.distributed as dist

    from ..parallel.fsdp import FullyShardedModule

    rank = dist.get_rank()
    fsdp = model if isinstance(model, FullyShardedModule) else None
    comm_dev = fsdp.engine.device if fsdp is not None else next((p.device for p in model.parameters()), torch.device("cpu"))
    if dist.get_backend() == "gloo":
        comm_dev = torch.device("cpu")
    unexpected, seen = set(), set()
    keys = set(model.state_dict().keys()) if fsdp is None else set()
    for path in files:
        shard = load_state_dict(path) if rank == 0 else None
        meta = [[(k, tuple(shard[k].shape), str(shard[k].dtype)) for k in shard] if rank == 0 else None]
        dist.broadcast_object_list(meta, src=0)
        for name, shape, dtype in meta[0]:
            dt = getattr(torch, dtype.replace("torch.", ""))
            buf = shard[name].to(comm_dev) if rank == 0 else torch.empty(shape, dtype=dt, device=comm_dev)
            dist.broadcast(buf, src=0)
            seen.add(name)
            if fsdp is not None:
                fsdp.engine.load_full_state_dict({name: buf}, strict=False)
                continue
            if name not in keys:
                unexpected.add(name)
                continue
            tgt = recursive_getattr(model, name)
            set_module_tensor_to_device(model, name, tgt.device if tgt.device.type != "meta" else comm_dev, value=buf)
        del shard
    if strict:
        expected = set(fsdp.engine.full_state_dict(rank0_only=False, cpu=True).keys()) if fsdp is not None else set(model.state_dict())
        missing = expected - seen
        if missing:
            raise KeyError(f"Missing keys in checkpoint: {sorted(missing)[:5]}")
    return unexpected


def load_checkpoint_in_model(
    model: nn.Module,
    checkpoint: Union[str, os.PathLike],
    device_map: Optional[dict] = None,
    offload_folder: Optional[Union[str, os.PathLike]] = None,
    dtype=None,
    offload_state_dict: bool = False,
    offload_buffers: bool = False,
    keep_in_fp32_modules: Optional[list] = None,
    offload_8bit_bnb: bool = False,
    strict: bool = False,
    full_state_dict: bool = True,
    broadcast_from_rank0: bool = False,
):
    """Load a (sharded) checkpoint into `model`, tensor by tensor, onto the devices `device_map` names (GPU, "cpu",
    "disk" with `offload_folder`); without a device map the tensors keep the model's placement. With
    `broadcast_from_rank0` (and an initialised process group) only rank 0 reads the files."""
    import torch.distributed as dist

    if offload_8bit_bnb:
        raise NotImplementedError("bitsandbytes is not supported on MI355X.")
    if device_map is not None and "disk" in device_map.values():
        if offload_folder is None:
            raise ValueError("At least one of the model submodule will be offloaded to disk, please pass along an `offload_folder`.")
        os.makedirs(offload_folder, exist_ok=True)
    tied = find_tied_parameters(model)
    if broadcast_from_rank0 and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if device_map is not None:
            raise ValueError("broadcast_from_rank0 loads full tensors into every rank; it cannot be combined with a device_map.")
        files = [checkpoint_files(checkpoint) if dist.get_rank() == 0 else None]  # only rank 0 sees the files
        dist.broadcast_object_list(files, src=0)
        unexpected = _broadcast_stream(model, files[0], strict)
    elif device_map is None:
        files = checkpoint_files(checkpoint)
        unexpected = set()
        keys = set(model.state_dict().keys())
        for path in files:
            shard = load_state_dict(path)
            sd = dict(shard.items()) if isinstance(shard, SafetensorsShard) else shard
            # a meta-initialised model takes the loaded tensors as its storage (assign), a materialised one copies
            on_meta = any(t.device.type == "meta" for t in model.state_dict().values())
            model.load_state_dict(sd, strict=strict, assign=on_meta)
            unexpected |= set(sd) - keys
            del shard, sd
            gc.collect()
    else:
        files = checkpoint_files(checkpoint)
        inst = _Installer(model, device_map, dtype, keep_in_fp32_modules, offload_folder, offload_state_dict, offload_buffers, strict)
        try:
            for path in files:
                shard = load_state_dict(path, device_map=device_map)
                layout = shard.layout() if isinstance(shard, SafetensorsShard) else {}
                for name in list(shard.keys()):
                    lay = layout.get(name)
                    if lay is not None and inst.put_from_file(name, path, *lay):
                        continue
                    inst.put(name, shard[name])  # one tensor resident at a time for safetensors shards
                del shard
                gc.collect()
            inst.finish()
        finally:
            inst.release()  # no-op after finish(); on an error path closes the shard files and clears the error count
        unexpected = inst.unexpected
    if unexpected:
        logger.warning(
            f"Some weights of the model checkpoint at {checkpoint} were not used when initializing "
            f"{model.__class__.__name__}: {sorted(unexpected)[:10]}"
        )
    retie_parameters(model, tied)
