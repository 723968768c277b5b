"""Failure detection, collective-order checking and fault injection.

Parity. The reference has no in-job failure handling of its own: relaunch is delegated to torchrun's elastic agent
(`/root/reference/src/accelerate/commands/launch.py:305-350`, `launchers.py:224-248`), hangs surface only as the
process-group timeout (`utils/dataclasses.py:272-299`), desynchronised collectives are caught only in debug mode by a
per-call shape all-gather (`utils/operations.py:355-415`), and its only fault injection lives in a test script
(`test_utils/scripts/test_notebook.py:34-51`). Here:

* `StepWatchdog` — a host thread fed a heartbeat by every `Accelerator.backward` and optimizer step. When no beat
  arrives for `timeout` seconds (a hung RCCL collective, a rank stuck in a data loader, a kernel that never retires)
  it prints which rank stalled and where, dumps every thread's Python stack (`faulthandler`) plus the collective log
  below, and ends the process with `os._exit(exit_code)` so torchrun's agent (`--max_restarts`) restarts the job
  from the latest `save_state` checkpoint instead of the job idling until the RCCL timeout. Enable with
  `RcclKwargs(watchdog_timeout=...)` or `ACCELERATE_WATCHDOG_TIMEOUT=<seconds>`.
* `CollectiveLog` — a rolling FNV-1a digest of (op, group size, dtype, numel) of every collective this rank issued
  through the framework (FSDP all-gather / reduce-scatter, DDP bucket all-reduce, `gather`/`reduce`/`broadcast`),
  kept by the native `_C.CollectiveSeq` when the extension is built. `check_collective_sequence()` all-gathers the
  (digest, count) pairs — one tiny collective every N steps in debug mode instead of one shape exchange per call —
  and raises `DistributedOperationException` naming the diverging ranks before RCCL deadlocks on them.
* `FaultInjector` — `ACCELERATE_FAULT_INJECT="rank:step:kind[,rank:step:kind...]"` (`rank` may be `*`), where `step`
  counts `Accelerator.backward` calls from 0 and `kind` is one of `raise` (RuntimeError), `oom` (an out-of-memory
  error, exercising `find_executable_batch_size`), `nan` (poisons that step's loss, exercising `check_trigger`-style
  early stops), `hang` (sleeps forever, exercising the watchdog) and `exit` (`os._exit(1)`, exercising elastic
  restarts). For tests and drills only.
"""

from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from dataclasses import dataclass
from typing import Optional

import torch

WATCHDOG_EXIT_CODE = 86


# ------------------------------------------------------------------------------------------------ collective log
class CollectiveLog:
    """Process-wide digest of the collectives this rank issued (see module docstring)."""

    _inst: Optional["CollectiveLog"] = None

    def __init__(self):
        self._native = None
        try:
            from ..ops._ext import _load

            mod = _load()
            if mod is not None and hasattr(mod, "CollectiveSeq"):
                self._native = mod.CollectiveSeq()
        except Exception:  # pragma: no cover - extension optional on CPU
            self._native = None
        self._h = 1469598103934665603
        self._n = 0
        self.last = None
        self.enabled = os.environ.get("ACCELERATE_CHECK_COLLECTIVES", "1") != "0"

    @classmethod
    def get(cls) -> "CollectiveLog":
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def record(self, op: str, group_size: int, dtype, numel: int):
        if not self.enabled:
            return
        dt = hash(str(dtype)) & 0xFFFF
        self.last = (op, int(group_size), str(dtype), int(numel))
        if self._native is not None:
            self._native.record(op, int(group_size), dt, int(numel))
            return
        for v in [*op.encode(), group_size, dt, numel]:
            for i in range(8):
                self._h ^= (int(v) >> (8 * i)) & 0xFF
                self._h = (self._h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        self._n += 1

    def digest(self) -> int:
        return int(self._native.digest()) if self._native is not None else self._h

    def count(self) -> int:
        return int(self._native.count()) if self._native is not None else self._n

    def reset(self):
        if self._native is not None:
            self._native.reset()
        self._h, self._n, self.last = 1469598103934665603, 0, None


def record_collective(op: str, tensor: Optional[torch.Tensor] = None, group=None, numel: Optional[int] = None):
    """Note one collective in the rank's log (cheap: a hash update on the host)."""
    log = CollectiveLog.get()
    if not log.enabled:
        return
    import torch.distributed as dist

    W = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    log.record(op, W, tensor.dtype if tensor is not None else "-", numel if numel is not None else (tensor.numel() if tensor is not None else 0))


def check_collective_sequence(group=None):
    """All-gather every rank's (digest, count) and raise if any rank issued a different collective sequence."""
    import torch.distributed as dist

    from .operations import DistributedOperationException

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    log = CollectiveLog.get()
    mine = (log.digest(), log.count(), log.last)
    everyone = [None] * dist.get_world_size(group)
    dist.all_gather_object(everyone, mine, group=group)
    if any(e[:2] != everyone[0][:2] for e in everyone):
        lines = "\n".join(f"  rank {r}: {e[1]} collectives, digest {e[0]:#018x}, last {e[2]}" for r, e in enumerate(everyone))
        raise DistributedOperationException(
            "Ranks issued different collective sequences (a desynchronised all-gather / reduce would deadlock RCCL):\n" + lines
        )


# ------------------------------------------------------------------------------------------------ watchdog
def abort_communicators() -> bool:
    """Abort every RCCL communicator of this process (torch `_abort_process_group`): kernels and host waits of
    collectives in flight end with an error here and, through RCCL's abort path, on the peers blocked in the same
    collective, instead of hanging until the process-group timeout. Returns whether an abort was issued."""
    try:
        import torch.distributed as dist
        from torch.distributed.distributed_c10d import _abort_process_group

        if not (dist.is_available() and dist.is_initialized()):
            return False
        _abort_process_group()
        return True
    except Exception as exc:  # noqa: BLE001 - best effort on the way out of a hung job
        sys.stderr.write(f"[accelerate watchdog] communicator abort failed: {exc!r}\n")
        return False



class StepWatchdog:
    """Host-side hang detector fed by training-step heartbeats (see module docstring)."""

    def __init__(self, timeout: float, rank: int = 0, exit_code: int = WATCHDOG_EXIT_CODE, action: str = "exit", poll: float = None):
        self.timeout = float(timeout)
        self.rank = rank
        self.exit_code = exit_code
        self.action = action  # "exit", "abort" (abort the RCCL communicators first, then exit) or "warn"
        self.poll = poll if poll is not None else max(0.05, min(5.0, self.timeout / 10))
        self._last = time.monotonic()
        self._tag = "start"
        self._beats = 0
        self._stop = threading.Event()
        self.fired = False
        self._thread = threading.Thread(target=self._run, name="accelerate-watchdog", daemon=True)
        self._thread.start()

    @classmethod
    def from_env(cls, timeout: Optional[float] = None, rank: int = 0) -> Optional["StepWatchdog"]:
        if timeout is None:
            env = os.environ.get("ACCELERATE_WATCHDOG_TIMEOUT")
            timeout = float(env) if env else None
        if not timeout or timeout <= 0:
            return None
        return cls(timeout, rank=rank, action=os.environ.get("ACCELERATE_WATCHDOG_ACTION", "exit"))

    def beat(self, tag: str = "step"):
        self._last = time.monotonic()
        self._tag = tag
        self._beats += 1

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(self.poll):
            idle = time.monotonic() - self._last
            if idle < self.timeout:
                continue
            log = CollectiveLog.get()
            sys.stderr.write(
                f"[accelerate watchdog] rank {self.rank}: no training progress for {idle:.1f}s (timeout {self.timeout:.1f}s); "
                f"last heartbeat '{self._tag}' after {self._beats} beats; collectives issued {log.count()}, last {log.last}\n"
            )
            sys.stderr.flush()
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            sys.stderr.flush()
            self.fired = True
            if self.action == "abort":
                abort_communicators()
            if self.action in ("exit", "abort"):
                os._exit(self.exit_code)
            self._last = time.monotonic()  # warn mode: report again after another full timeout


# ------------------------------------------------------------------------------------------------ fault injection
@dataclass
class _Fault:
    rank: Optional[int]
    step: int
    kind: str


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    KINDS = ("raise", "oom", "nan", "hang", "exit")

    def __init__(self, spec: str, rank: int = 0):
        self.rank = rank
        self.faults: list[_Fault] = []
        for item in filter(None, (s.strip() for s in spec.split(","))):
            parts = item.split(":")
            if len(parts) != 3 or parts[2] not in self.KINDS:
                raise ValueError(f"ACCELERATE_FAULT_INJECT entry {item!r}: expected rank:step:kind with kind in {self.KINDS}")
            r = None if parts[0] in ("*", "") else int(parts[0])
            self.faults.append(_Fault(r, int(parts[1]), parts[2]))

    @classmethod
    def from_env(cls, rank: int = 0) -> Optional["FaultInjector"]:
        spec = os.environ.get("ACCELERATE_FAULT_INJECT", "")
        return cls(spec, rank) if spec.strip() else None

    def before_backward(self, step: int, loss: torch.Tensor) -> torch.Tensor:
        for f in self.faults:
            if f.step != step or (f.rank is not None and f.rank != self.rank):
                continue
            if f.kind == "raise":
                raise InjectedFault(f"injected fault on rank {self.rank} at step {step}")
            if f.kind == "oom":
                raise torch.cuda.OutOfMemoryError(f"HIP out of memory. (injected on rank {self.rank} at step {step})")
            if f.kind == "nan":
                loss = loss * float("nan")
            elif f.kind == "hang":
                while True:  # the watchdog (or the RCCL timeout) must end this process
                    time.sleep(3600)
            elif f.kind == "exit":
                sys.stderr.write(f"[accelerate fault] rank {self.rank} exiting at step {step} (injected)\n")
                sys.stderr.flush()
                os._exit(1)
        return loss
