"""Environment-variable helpers and device/runtime introspection for MI355X nodes.

Parity: `/root/reference/src/accelerate/utils/environment.py:34-471` (str_to_bool, get_int_from_env,
parse_flag_from_env, patch_environment, clear_environment, purge_accelerate_environment,
get_cpu_distributed_information). The nvidia-smi / pynvml / compute-capability probes of the reference
are replaced by ROCm equivalents: `gcnArchName` (gfx950 detection), `rocm-smi`, and the HIP device
properties exposed by torch.
"""

from __future__ import annotations

import contextlib
import functools
import os
import platform
import shutil
import subprocess
from dataclasses import dataclass, field
from typing import Any


def str_to_bool(value, to_bool: bool = False) -> int | bool:
    """Convert a truthy/falsy string to 1/0 (or True/False when `to_bool`)."""
    value = str(value).lower()
    if value in ("y", "yes", "t", "true", "on", "1"):
        return True if to_bool else 1
    if value in ("n", "no", "f", "false", "off", "0"):
        return False if to_bool else 0
    raise ValueError(f"invalid truth value {value}")


def get_int_from_env(env_keys, default):
    """Return the first non-negative integer found among `env_keys`, else `default`."""
    for e in env_keys:
        val = int(os.environ.get(e, "-1"))
        if val >= 0:
            return val
    return default


def parse_flag_from_env(key, default=False):
    value = os.environ.get(key, str(default))
    return str_to_bool(value) == 1


def parse_choice_from_env(key, default="no"):
    return os.environ.get(key, str(default))


def are_libraries_initialized(*library_names: str) -> list[str]:
    """Libraries in `library_names` already imported (used by notebook_launcher's fork pre-flight)."""
    import sys

    return [lib for lib in library_names if lib in sys.modules.keys()]


def _device_count_no_init() -> int:
    """Count HIP devices without creating a HIP context (fork safe)."""
    import torch

    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


def get_current_device_type() -> tuple[str, str]:
    """Return ("cuda", "cuda") when an MI355X (any ROCm GPU) is visible, else ("cpu", "cpu")."""
    if _device_count_no_init() > 0:
        return "cuda", "cuda"
    return "cpu", "cpu"


@functools.lru_cache
def get_gpu_arch(device_index: int = 0) -> str | None:
    """gfx architecture name of a device (e.g. 'gfx950:sramecc+:xnack-'), or None without a GPU."""
    import torch

    if not torch.cuda.is_available():
        return None
    props = torch.cuda.get_device_properties(device_index)
    return getattr(props, "gcnArchName", None)


def is_gfx950(device_index: int = 0) -> bool:
    arch = get_gpu_arch(device_index)
    return bool(arch) and arch.startswith("gfx950")


def check_fp8_capability() -> bool:
    """fp8 (OCP e4m3fn/e5m2) MFMA is native on gfx950. Replaces `check_cuda_fp8_capability`
    (reference `utils/environment.py:226-245`)."""
    return is_gfx950()


def get_gpu_info() -> tuple[list[str], int]:
    """Names and count of the visible GPUs."""
    import torch

    n = _device_count_no_init()
    names = []
    for i in range(n):
        try:
            names.append(torch.cuda.get_device_name(i))
        except Exception:
            names.append("unknown")
    return names, n


def rocm_smi_available() -> bool:
    return shutil.which("rocm-smi") is not None


def get_xgmi_topology() -> str | None:
    """Raw `rocm-smi --showtopotype` output, or None if unavailable (used by `accelerate env`)."""
    if not rocm_smi_available():
        return None
    try:
        return subprocess.run(
            ["rocm-smi", "--showtopotype"], capture_output=True, text=True, timeout=20
        ).stdout
    except Exception:
        return None


def get_cpu_distributed_information():
    """Rank/world information for multi-CPU launches (MPI, PMI, torchrun)."""

    @dataclass
    class CPUInformation:
        rank: int = field(default=0)
        world_size: int = field(default=1)
        local_rank: int = field(default=0)
        local_world_size: int = field(default=1)

    information = {}
    information["rank"] = get_int_from_env(["RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", "MV2_COMM_WORLD_RANK"], 0)
    information["world_size"] = get_int_from_env(
        ["WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE"], 1
    )
    information["local_rank"] = get_int_from_env(
        ["LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK"], 0
    )
    information["local_world_size"] = get_int_from_env(
        ["LOCAL_WORLD_SIZE", "MPI_LOCALNRANKS", "OMPI_COMM_WORLD_LOCAL_SIZE", "MV2_COMM_WORLD_LOCAL_SIZE"], 1
    )
    return CPUInformation(**information)


def override_numa_affinity(local_process_index: int, verbose: bool | None = None) -> None:
    """Pin this process to the CPUs closest to its GPU.

    MI355X nodes expose the NUMA node of each GPU in sysfs (`/sys/class/drm/card*/device/numa_node`);
    we read it directly instead of going through pynvml as the reference does
    (`utils/environment.py:283-338`).
    """
    if platform.system() != "Linux":
        return
    import glob

    cards = sorted(glob.glob("/sys/class/drm/card*/device/numa_node"))
    if not cards:
        return
    try:
        node = int(open(cards[local_process_index % len(cards)]).read().strip())
    except Exception:
        return
    if node < 0:
        return
    cpulist_path = f"/sys/devices/system/node/node{node}/cpulist"
    if not os.path.exists(cpulist_path):
        return
    cpus = set()
    for part in open(cpulist_path).read().strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    if cpus:
        os.sched_setaffinity(0, cpus)
        if verbose:
            print(f"Assigned process {local_process_index} to NUMA node {node} CPUs {sorted(cpus)[:4]}...")


def set_numa_affinity(local_process_index: int, verbose: bool | None = None) -> None:
    override_numa_affinity(local_process_index, verbose=verbose)


@contextlib.contextmanager
def clear_environment():
    """Temporarily empty `os.environ` (restored on exit, even on error)."""
    saved = os.environ.copy()
    os.environ.clear()
    try:
        yield
    finally:
        os.environ.clear()
        os.environ.update(saved)


@contextlib.contextmanager
def patch_environment(**kwargs):
    """Set upper-cased env vars for the duration of the block; previous values are restored."""
    existing = {}
    for key, value in kwargs.items():
        key = key.upper()
        if key in os.environ:
            existing[key] = os.environ[key]
        os.environ[key] = str(value)
    try:
        yield
    finally:
        for key in kwargs:
            key = key.upper()
            if key in existing:
                os.environ[key] = existing[key]
            else:
                os.environ.pop(key, None)


def purge_accelerate_environment(func_or_cls):
    """Decorator: restore any `ACCELERATE_*` env var changed by the wrapped function / test class."""

    def _snapshot():
        return {k: v for k, v in os.environ.items() if k.startswith("ACCELERATE_")}

    def _restore(before):
        for k in list(os.environ.keys()):
            if k.startswith("ACCELERATE_") and k not in before:
                del os.environ[k]
        os.environ.update(before)

    if isinstance(func_or_cls, type):
        for name in dir(func_or_cls):
            if name.startswith("test") or name in ("setUp", "tearDown"):
                attr = getattr(func_or_cls, name)
                if callable(attr):
                    setattr(func_or_cls, name, purge_accelerate_environment(attr))
        return func_or_cls

    @functools.wraps(func_or_cls)
    def wrapper(*args, **kwargs):
        before = _snapshot()
        try:
            return func_or_cls(*args, **kwargs)
        finally:
            _restore(before)

    return wrapper


def convert_dict_to_env_variables(current_env: dict) -> list[str]:
    """Render a dict as `KEY=value\\n` lines, dropping malformed entries."""
    forbidden = [";", "\n", "<", ">", " "]
    valid = []
    for key, value in current_env.items():
        if all(c not in (key + str(value)) for c in forbidden) and len(key) >= 1 and len(str(value)) >= 1:
            valid.append(f"{key}={value}\n")
    return valid


def get_ccl_version() -> str:
    """RCCL version reported by torch (ROCm build)."""
    import torch

    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return "unavailable"


def env_summary() -> dict[str, Any]:
    """Facts reported by `accelerate env` on an MI355X node."""
    import torch

    names, n = get_gpu_info()
    info = {
        "torch": torch.__version__,
        "hip": getattr(torch.version, "hip", None),
        "rccl": get_ccl_version() if n else "n/a",
        "gpus": n,
        "gpu_names": names,
        "arch": get_gpu_arch() if n else None,
        "hbm_per_device_gb": (
            round(torch.cuda.get_device_properties(0).total_memory / 2**30, 1) if n and torch.cuda.is_available() else None
        ),
        "platform": platform.platform(),
        "python": platform.python_version(),
    }
    return info
