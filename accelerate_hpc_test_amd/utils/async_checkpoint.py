"""Non-blocking sharded checkpoint writes (reference `checkpointing.py:62-177`, `utils/fsdp_utils.py:103-158`).

The reference writes FSDP shards through torch DCP synchronously. Here a save hands the shard tensors to the native
`D2HFileWriter` (csrc/runtime/d2h_writer.cpp) and returns:

1. snapshot: every shard tensor is cloned ON THE DEVICE (HBM -> HBM at TB/s; MI355X has 288 GB, the shards of one rank
   are a fraction of it), so the next optimizer step may overwrite the live state at once;
2. the writer's dispatcher streams the snapshot to the files in slot-sized pieces (pinned ring, own HIP stream,
   ordered after the snapshot by an event) and its worker threads `pwrite` them in the safetensors layout (8-byte
   header length, JSON header, raw little-endian bytes), so host memory stays at the ring size;
3. the next `save_state` / `load_state`, `end_training` and interpreter exit wait for the pending writes
   (`wait_pending_saves`), and a failed write raises there.

When the free HBM cannot hold the snapshot the same writer streams the live tensors and the save waits for it (still
bounded host memory). On CPU tensors (gloo tests) the files are written synchronously in the same format.
`ACCELERATE_ASYNC_SAVE=0` restores the synchronous safetensors path.
"""

from __future__ import annotations

import atexit
import json
import os
import struct
import threading
from typing import Optional

import torch

_DTYPES = {
    torch.float32: "F32", torch.float16: "F16", torch.bfloat16: "BF16", torch.float64: "F64", torch.int64: "I64",
    torch.int32: "I32", torch.int16: "I16", torch.int8: "I8", torch.uint8: "U8", torch.bool: "BOOL",
    torch.float8_e4m3fn: "F8_E4M3", torch.float8_e5m2: "F8_E5M2",
}
_ENABLED = os.environ.get("ACCELERATE_ASYNC_SAVE", "1") != "0"
_MARGIN = 4 << 30  # HBM left free after the snapshot


def safetensors_prefix(tensors: dict, metadata: Optional[dict] = None):
    """(header bytes incl. the 8-byte length, {name: byte offset of its data in the file}) of a safetensors file
    holding `tensors` in insertion order."""
    header, offsets, off = {}, {}, 0
    for name, t in tensors.items():
        nb = t.numel() * t.element_size()
        header[name] = {"dtype": _DTYPES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + nb]}
        offsets[name] = off
        off += nb
    if metadata:
        header["__metadata__"] = {str(k): str(v) for k, v in metadata.items()}
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    prefix = struct.pack("<Q", len(hb)) + hb
    return prefix, {k: len(prefix) + v for k, v in offsets.items()}


class AsyncCheckpointWriter:
    """One per process: the native writer (created on first use) and the saves not yet known to be on disk."""

    def __init__(self):
        self._writer = None
        self._pending = 0
        self._lock = threading.Lock()
        self.last_snapshot_bytes = 0
        self.last_async = False

    def _native(self, device: torch.device):
        if self._writer is None:
            from ..ops._ext import ext

            self._writer = ext().D2HFileWriter(device.index if device.index is not None else torch.cuda.current_device(),
                                               8, 64 << 20, 2)
        return self._writer

    def save_file(self, tensors: dict, path: str, metadata: Optional[dict] = None, wait: Optional[bool] = None) -> bool:
        """Write `tensors` (name -> tensor) as a safetensors file at `path`. HIP tensors go through the native writer:
        snapshotted on the device when the free HBM allows (the call returns before the bytes are on disk; True), else
        streamed from the live tensors and waited for. Returns True when the write is still pending."""
        tensors = {k: v.detach() for k, v in tensors.items()}
        cuda = [t for t in tensors.values() if t.is_cuda]
        prefix, offsets = safetensors_prefix(tensors, metadata)
        if not (_ENABLED and cuda):
            with open(path, "wb") as f:
                f.write(prefix)
                for t in tensors.values():
                    f.write(t.contiguous().cpu().reshape(-1).view(torch.uint8).numpy().tobytes())
            return False
        dev = cuda[0].device
        need = sum(t.numel() * t.element_size() for t in cuda)
        free, _ = torch.cuda.mem_get_info(dev)
        snapshot = need + _MARGIN <= free
        w = self._native(dev)
        with open(path, "wb"):
            pass  # create / truncate; the writer opens it for positional writes
        w.write_bytes(path, 0, prefix)
        for name, t in tensors.items():
            src = t.contiguous()
            if src.is_cuda and snapshot:
                src = src.clone()  # the live state may change after this call returns
            w.write(path, offsets[name], src.reshape(-1))
        with self._lock:
            self._pending += 1
        self.last_snapshot_bytes = need if snapshot else 0
        self.last_async = snapshot and wait is not True
        if not self.last_async:
            self.wait()
        return self.last_async

    def wait(self):
        """Block until every pending write is on disk; raise if any failed."""
        with self._lock:
            pending, self._pending = self._pending, 0
        if self._writer is None or pending == 0:
            return
        errors = self._writer.finish()
        if errors:
            raise OSError(f"async checkpoint writer: {errors} write(s) failed")

    @property
    def pending(self) -> int:
        return self._pending


_WRITER = AsyncCheckpointWriter()


def writer() -> AsyncCheckpointWriter:
    return _WRITER


def wait_pending_saves():
    """Wait for the checkpoint files of earlier non-blocking saves (called before every save / load and at exit)."""
    _WRITER.wait()


atexit.register(wait_pending_saves)
