"""The test-harness module (`test_utils/testing.py`): launch command, env flags, skip decorators, base test cases and
subprocess runners — including an end-to-end 2-process CPU launch through `get_launch_command`."""

import os
import sys
import tempfile
import textwrap
import unittest
from unittest import mock

import pytest
import torch

from accelerate_hpc_test_amd.state import AcceleratorState, PartialState
from accelerate_hpc_test_amd.test_utils import testing as T
from accelerate_hpc_test_amd.utils.other import get_free_port


def test_backend_and_launch_command():
    dev, n, mem = T.get_backend()
    assert dev in ("cuda", "cpu") and n >= 1 and mem() >= 0
    cmd = T.get_launch_command(num_processes=2, cpu=True, debug=False, mixed_precision=None, main_process_port=123)
    assert cmd[-4:] == ["launch", "--num_processes=2", "--cpu", "--main_process_port=123"]
    assert "--monitor_interval=0.1" in T.DEFAULT_LAUNCH_COMMAND


def test_parse_flag_from_env():
    with mock.patch.dict(os.environ, {"X_FLAG": "yes", "Y_FLAG": "0", "Z_FLAG": "maybe"}):
        assert T.parse_flag_from_env("X_FLAG") is True
        assert T.parse_flag_from_env("Y_FLAG", default=True) is False
        assert T.parse_flag_from_env("MISSING_FLAG", default=True) is True
        with pytest.raises(ValueError):
            T.parse_flag_from_env("Z_FLAG")


def _run_case(case_cls):
    res = unittest.TestResult()
    unittest.defaultTestLoader.loadTestsFromTestCase(case_cls).run(res)
    return res


def test_require_decorators_skip_and_run():
    class Case(unittest.TestCase):
        @T.require_xpu
        def test_xpu(self):
            raise AssertionError("must be skipped")

        @T.require_fsdp2
        def test_fsdp2(self):
            pass

        @T.requires(lambda: False, "custom reason")
        def test_custom(self):
            raise AssertionError("must be skipped")

        @T.require_torch_min_version(version="1.0")
        def test_min_version(self):
            pass

        @T.require_torch_min_version(version="99.0")
        def test_future_version(self):
            raise AssertionError("must be skipped")

    res = _run_case(Case)
    skipped = {t.id().split(".")[-1]: why for t, why in res.skipped}
    assert set(skipped) == {"test_xpu", "test_custom", "test_future_version"}, skipped
    assert skipped["test_custom"] == "custom reason"
    assert res.wasSuccessful() and res.testsRun == 5
    gpu = T.require_cuda(lambda: None)
    assert getattr(gpu, "__unittest_skip__", False) == (not torch.cuda.is_available())


def test_tempdir_and_accelerate_test_cases():
    seen = []

    class Tmp(T.TempDirTestCase):
        def test_a(self):
            (self.tmpdir / "f.txt").write_text("x")
            (self.tmpdir / "d").mkdir()
            seen.append(self.tmpdir)

        def test_b(self):
            assert list(self.tmpdir.iterdir()) == []  # emptied before each test
            seen.append(self.tmpdir)

    assert _run_case(Tmp).wasSuccessful()
    assert seen[0] == seen[1] and not seen[0].exists()  # one dir per class, removed at the end

    class Acc(T.AccelerateTestCase):
        def test_state(self):
            AcceleratorState(cpu=True)
            assert AcceleratorState._shared_state != {}

    assert _run_case(Acc).wasSuccessful()
    assert AcceleratorState._shared_state == {} and PartialState._shared_state == {}


def test_mocking_test_case():
    class M(T.MockingTestCase):
        def setUp(self):
            super().setUp()
            self.add_mocks(mock.patch.dict(os.environ, {"MOCKED_VAR": "1"}))

        def test_env(self):
            assert os.environ["MOCKED_VAR"] == "1"

    assert _run_case(M).wasSuccessful()
    assert "MOCKED_VAR" not in os.environ


def test_subprocess_helpers():
    out = T.execute_subprocess_async([sys.executable, "-c", "import sys; print('hi'); print('err', file=sys.stderr)"], quiet=True, echo=False)
    assert out.returncode == 0 and out.stdout == ["hi"] and out.stderr == ["err"]
    with pytest.raises(RuntimeError, match="returncode 3"):
        T.execute_subprocess_async([sys.executable, "-c", "raise SystemExit(3)"], quiet=True, echo=False)
    with pytest.raises(RuntimeError, match="timeout"):
        T.execute_subprocess_async([sys.executable, "-c", "import time; time.sleep(30)"], timeout=1, quiet=True, echo=False)
    assert T.run_command([sys.executable, "-c", "print(42)"], return_stdout=True).strip() == "42"
    with pytest.raises(T.SubprocessCallException, match="boom"):
        T.run_command([sys.executable, "-c", "raise RuntimeError('boom')"])
    with mock.patch.dict(os.environ, {"PYTEST_XDIST_WORKER": "gw3"}):
        assert T.pytest_xdist_worker_id() == 3 and T.get_torch_dist_unique_port() == 29503


def test_exception_and_output_helpers():
    with T.assert_exception(ValueError, "bad"):
        raise ValueError("a bad value")
    with pytest.raises(AssertionError):
        with T.assert_exception(ValueError):
            pass
    with pytest.raises(AssertionError):
        with T.assert_exception(KeyError):
            raise ValueError("wrong type")
    assert T.capture_call_output(print, "hello") == "hello\n"
    assert T.path_in_accelerate_package("test_utils", "testing.py").exists()


def test_launch_command_end_to_end_two_cpu_processes():
    """`get_launch_command(...) + [script]` really launches a 2-process gloo job; `are_the_same_tensors` runs in it."""
    script = textwrap.dedent("""
        import os, sys, torch
        from accelerate_hpc_test_amd import Accelerator
        from accelerate_hpc_test_amd.test_utils.testing import are_the_same_tensors
        acc = Accelerator(cpu=True)
        assert acc.num_processes == 2
        assert are_the_same_tensors(torch.arange(4.0))
        assert not are_the_same_tensors(torch.tensor([float(acc.process_index)]))
        open(os.path.join(sys.argv[1], f"rank{acc.process_index}"), "w").write("ok")
    """)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "job.py")
        open(path, "w").write(script)
        cmd = T.get_launch_command(num_processes=2, cpu=True, main_process_ip="127.0.0.1", main_process_port=get_free_port())
        env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.getcwd(), os.environ.get("PYTHONPATH", "")]))
        T.execute_subprocess_async(cmd + [path, d], env=env, timeout=180, quiet=True, echo=False)
        assert sorted(f for f in os.listdir(d) if f.startswith("rank")) == ["rank0", "rank1"]
