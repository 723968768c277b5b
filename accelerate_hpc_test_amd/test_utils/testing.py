"""Test harness helpers: backend discovery, launch commands, skip decorators, base test cases, subprocess runners.

Public names follow the reference's `accelerate.test_utils.testing` (`/root/reference/src/accelerate/test_utils/
testing.py:83-880`) so test suites written against it run here. The design is this framework's:

  * ONE decorator factory (`requires`) builds every `require_*` from a predicate evaluated lazily at decoration time;
    accelerators this build does not target (XPU / NPU / MLU / HPU / MPS / TPU / SDAA / MUSA) are permanent skips,
    `require_cuda` means "a HIP GPU" (ROCm exposes HIP devices through `torch.cuda`), `require_fp8` means gfx950;
  * `get_launch_command` builds this framework's launcher (`accelerate-amd launch`, or `python -m` of the CLI module
    when the console script is not installed);
  * `execute_subprocess_async` streams both pipes through reader threads (no asyncio event loop), tees them, and
    enforces the timeout by killing the child.
"""

from __future__ import annotations

import importlib.util
import inspect
import io
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import unittest
from contextlib import contextmanager
from pathlib import Path
from typing import Callable, Optional, Union
from unittest import mock

import torch

from ..state import AcceleratorState, PartialState
from ..utils.environment import str_to_bool
from ..utils.imports import is_cuda_available, is_fp8_available, is_native_extension_available


# ------------------------------------------------------------------------------------------------ backend
def get_backend():
    """(device type, device count, memory-allocated callable) of this machine: "cuda" (HIP) or "cpu"."""
    if is_cuda_available():
        return "cuda", torch.cuda.device_count(), torch.cuda.memory_allocated
    return "cpu", 1, lambda *_a, **_k: 0


torch_device, device_count, memory_allocated_func = get_backend()


def _launcher_prefix() -> list:
    exe = shutil.which("accelerate-amd")
    if exe is not None:
        return [exe]
    return [sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli"]


def get_launch_command(**kwargs) -> list:
    """`[<launcher>, "launch", "--k=v", ...]`; True booleans become bare flags, None values are dropped.

    >>> get_launch_command(num_processes=2, debug=True)[-2:]
    ['--num_processes=2', '--debug']
    """
    cmd = _launcher_prefix() + ["launch"]
    for k, v in kwargs.items():
        if v is True:
            cmd.append(f"--{k}")
        elif v is not None and v is not False:
            cmd.append(f"--{k}={v}")
    return cmd


DEFAULT_LAUNCH_COMMAND = get_launch_command(num_processes=device_count, monitor_interval=0.1)


def parse_flag_from_env(key: str, default: bool = False) -> bool:
    if key not in os.environ:
        return default
    try:
        return bool(str_to_bool(os.environ[key]))
    except ValueError as exc:
        raise ValueError(f"If set, {key} must be yes or no.") from exc


_run_slow_tests = parse_flag_from_env("RUN_SLOW", default=False)


# ------------------------------------------------------------------------------------------------ decorators
def requires(predicate: Callable[[], bool], reason: str):
    """Decorator factory: skip the test (function or class) unless `predicate()` holds."""

    def deco(test_case):
        return unittest.skipUnless(predicate(), reason)(test_case)

    return deco


def _module(name: str) -> Callable[[], bool]:
    return lambda: importlib.util.find_spec(name) is not None


def _never() -> bool:
    return False


def skip(test_case):
    return unittest.skip("Test was skipped")(test_case)


def slow(test_case):
    """Runs only with RUN_SLOW=yes."""
    return unittest.skipUnless(_run_slow_tests, "test is slow")(test_case)


require_cpu = requires(lambda: torch_device == "cpu", "test requires only a CPU")
require_non_cpu = requires(lambda: torch_device != "cpu", "test requires a GPU")
require_cuda = requires(is_cuda_available, "test requires a HIP GPU")
require_cuda_or_hpu = require_cuda
require_cuda_or_xpu = require_cuda
require_multi_gpu_or_xpu = requires(lambda: torch_device == "cuda" and device_count > 1, "test requires multiple GPUs")
require_fp16 = requires(is_cuda_available, "test requires fp16 support (a GPU)")
require_fp8 = requires(is_fp8_available, "test requires fp8 support (gfx950)")
require_fsdp2 = requires(lambda: True, "FSDP2 is always available")
require_single_device = requires(lambda: torch_device != "cpu" and device_count == 1, "test requires one GPU")
require_single_gpu = requires(lambda: torch_device == "cuda" and device_count == 1, "test requires one GPU")
require_multi_device = requires(lambda: torch_device != "cpu" and device_count > 1, "test requires multiple GPUs")
require_multi_gpu = requires(lambda: torch_device == "cuda" and device_count > 1, "test requires multiple GPUs")
require_native_extension = requires(is_native_extension_available, "test requires the compiled HIP extension")
require_tp = requires(lambda: True, "tensor parallelism is always available")
require_non_torch_xla = requires(lambda: True, "torch_xla is not used by this build")
require_non_xpu = requires(lambda: True, "XPU is not used by this build")
require_non_hpu = requires(lambda: True, "HPU is not used by this build")
# accelerators this build does not target
require_xpu = requires(_never, "XPU is not supported on MI355X builds")
require_single_xpu = require_multi_xpu = require_xpu
require_mlu = requires(_never, "MLU is not supported on MI355X builds")
require_sdaa = requires(_never, "SDAA is not supported on MI355X builds")
require_musa = requires(_never, "MUSA is not supported on MI355X builds")
require_npu = requires(_never, "NPU is not supported on MI355X builds")
require_mps = requires(_never, "MPS is not supported on MI355X builds")
require_tpu = requires(_never, "TPU is not supported on MI355X builds")
require_bnb = requires(_never, "bitsandbytes is not part of this build")
require_deepspeed = requires(_module("deepspeed"), "test requires DeepSpeed")
require_transformer_engine = requires(lambda: True, "fp8 TE recipes run on the native kernels")
require_transformer_engine_mxfp8 = requires(is_fp8_available, "MXFP8 needs gfx950")
require_torchao = requires(lambda: True, "fp8 AO recipes run on the native kernels")
# optional third-party packages
require_huggingface_suite = requires(lambda: _module("transformers")() and _module("datasets")(), "test requires transformers and datasets")
require_transformers = requires(_module("transformers"), "test requires transformers")
require_timm = requires(_module("timm"), "test requires timm")
require_torchvision = requires(_module("torchvision"), "test requires torchvision")
require_triton = requires(_never, "Triton is not used by this build")
require_schedulefree = requires(_module("schedulefree"), "test requires schedulefree")
require_tensorboard = requires(lambda: _module("tensorboard")() or _module("tensorboardX")(), "test requires tensorboard")
require_wandb = requires(_module("wandb"), "test requires wandb")
require_trackio = requires(_module("trackio"), "test requires trackio")
require_comet_ml = requires(_module("comet_ml"), "test requires comet_ml")
require_aim = requires(_module("aim"), "test requires aim")
require_clearml = requires(_module("clearml"), "test requires clearml")
require_dvclive = requires(_module("dvclive"), "test requires dvclive")
require_swanlab = requires(_module("swanlab"), "test requires swanlab")
require_mlflow = requires(_module("mlflow"), "test requires mlflow")
require_pandas = requires(_module("pandas"), "test requires pandas")
require_matplotlib = requires(_module("matplotlib"), "test requires matplotlib")
require_pippy = requires(lambda: True, "pipeline inference is native")
require_import_timer = requires(_module("import_timer"), "test requires import_timer")
require_torchdata_stateful_dataloader = requires(_module("torchdata"), "test requires torchdata")
require_trackers = requires(
    lambda: any(_module(m)() for m in ("wandb", "comet_ml", "tensorboard", "tensorboardX", "mlflow", "aim", "clearml",
                                       "dvclive", "swanlab", "trackio")),
    "test requires at least one tracker package",
)


def require_torch_min_version(test_case=None, version: Optional[str] = None):
    """Skip unless torch >= `version` (usable bare or with arguments)."""
    if test_case is None:
        return lambda tc: require_torch_min_version(tc, version=version)
    from packaging.version import Version

    ok = version is None or Version(torch.__version__.split("+")[0]) >= Version(version)
    return unittest.skipUnless(ok, f"test requires torch >= {version}")(test_case)


def run_first(test_case):
    """Order the test first when pytest-order is installed (a no-op otherwise)."""
    try:
        import pytest

        return pytest.mark.order(1)(test_case)
    except ImportError:
        return test_case


# ------------------------------------------------------------------------------------------------ test cases
class TempDirTestCase(unittest.TestCase):
    """One temporary directory per test class (`self.tmpdir`), emptied before every test when `clear_on_setup`."""

    clear_on_setup = True

    @classmethod
    def setUpClass(cls):
        cls.tmpdir = Path(tempfile.mkdtemp())

    @classmethod
    def tearDownClass(cls):
        shutil.rmtree(cls.tmpdir, ignore_errors=True)

    def setUp(self):
        if self.clear_on_setup:
            for child in list(self.tmpdir.iterdir()):
                shutil.rmtree(child) if child.is_dir() else child.unlink()


class AccelerateTestCase(unittest.TestCase):
    """Resets the AcceleratorState / PartialState singletons after every test."""

    def tearDown(self):
        super().tearDown()
        AcceleratorState._reset_state(True)


class MockingTestCase(unittest.TestCase):
    """`add_mocks(m)` (called at the end of `setUp`) starts mocks that are stopped after each test."""

    def add_mocks(self, mocks: Union[mock.Mock, list]):
        self.mocks = list(mocks) if isinstance(mocks, (list, tuple)) else [mocks]
        for m in self.mocks:
            m.start()
            self.addCleanup(m.stop)


def are_the_same_tensors(tensor: torch.Tensor) -> bool:
    """Whether every process holds the same `tensor` (gathers it across processes)."""
    from ..utils.operations import gather

    state = PartialState()
    local = tensor[None].clone().to(state.device)
    allt = gather(local).cpu()
    mine = local[0].cpu()
    return all(torch.equal(allt[i], mine) for i in range(allt.shape[0]))


# ------------------------------------------------------------------------------------------------ subprocesses
class _RunOutput:
    def __init__(self, returncode: int, stdout: list, stderr: list):
        self.returncode, self.stdout, self.stderr = returncode, stdout, stderr


def _pump(pipe, sink: list, echo_to, label: str, quiet: bool):
    for raw in iter(pipe.readline, b""):
        line = raw.decode("utf-8", errors="replace").rstrip()
        sink.append(line)
        if not quiet:
            print(label, line, file=echo_to)
    pipe.close()


def execute_subprocess_async(cmd: list, env=None, stdin=None, timeout: float = 180, quiet: bool = False,
                             echo: bool = True) -> _RunOutput:
    """Run `cmd`, streaming (and collecting) stdout / stderr line by line; kill it after `timeout` seconds. Raises
    RuntimeError with the collected stderr on a non-zero exit."""
    cmd = [str(c) for c in cmd]
    if echo:
        print("\nRunning: ", " ".join(cmd))
    p = subprocess.Popen(cmd, stdin=stdin, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
    out, err = [], []
    readers = [threading.Thread(target=_pump, args=(p.stdout, out, sys.stdout, "stdout:", quiet), daemon=True),
               threading.Thread(target=_pump, args=(p.stderr, err, sys.stderr, "stderr:", quiet), daemon=True)]
    for t in readers:
        t.start()
    try:
        rc = p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        rc = p.wait()
        err.append(f"killed after {timeout} s timeout")
    for t in readers:
        t.join(timeout=5)
    if rc != 0:
        raise RuntimeError(f"'{' '.join(cmd)}' failed with returncode {rc}\n\nThe combined stderr from workers follows:\n"
                           + "\n".join(err))
    return _RunOutput(rc, out, err)


def pytest_xdist_worker_id() -> int:
    """Numeric id of this pytest-xdist worker ("gw3" -> 3), 0 outside xdist."""
    w = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    return int(w[2:]) if w.startswith("gw") and w[2:].isdigit() else 0


def get_torch_dist_unique_port() -> int:
    """A master port distinct per xdist worker (29500 + worker id)."""
    return 29500 + pytest_xdist_worker_id()


class SubprocessCallException(Exception):
    pass


def run_command(command: list, return_stdout: bool = False, env=None):
    """`subprocess.check_output` with stderr folded in; raises SubprocessCallException carrying the output."""
    command = [str(c) for c in command]
    try:
        res = subprocess.check_output(command, stderr=subprocess.STDOUT, env=env if env is not None else os.environ.copy())
    except subprocess.CalledProcessError as exc:
        raise SubprocessCallException(
            f"Command `{' '.join(command)}` failed with the following error:\n\n{exc.output.decode()}") from exc
    if return_stdout:
        return res.decode("utf-8") if hasattr(res, "decode") else res
    return None


def path_in_accelerate_package(*components: str) -> Path:
    """A path inside this package's directory."""
    import accelerate_hpc_test_amd

    return Path(inspect.getfile(accelerate_hpc_test_amd)).parent.joinpath(*components)


@contextmanager
def assert_exception(exception_class, msg: Optional[str] = None):
    """Assert that the block raises `exception_class` (with `msg` in its text, when given)."""
    try:
        yield
    except Exception as exc:  # noqa: BLE001 - checked below
        assert isinstance(exc, exception_class), f"Expected exception of type {exception_class} but got {type(exc)}"
        if msg is not None:
            assert msg in str(exc), f"Expected message '{msg}' to be in exception but got '{exc}'"
        return
    raise AssertionError(f"Expected exception of type {exception_class} but ran without issue.")


def capture_call_output(func, *args, **kwargs) -> str:
    """stdout produced by `func(*args, **kwargs)`."""
    buf = io.StringIO()
    old = sys.stdout
    sys.stdout = buf
    try:
        func(*args, **kwargs)
    finally:
        sys.stdout = old
    return buf.getvalue()
