"""bench.py's communicator pre-flight (utils/preflight.py): known-value checks and bandwidth per process group, and
the two failure forms — a wrong result raises / exits naming the group and operation, a stuck collective ends the
process with exit code 3 and a JSON line instead of hanging."""

import json
import os
import subprocess
import sys

import pytest

from accelerate_hpc_test_amd import debug_launcher

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ok_two_ranks():
    import torch
    import torch.distributed as dist

    from accelerate_hpc_test_amd.state import PartialState
    from accelerate_hpc_test_amd.utils.preflight import communicator_preflight

    PartialState(cpu=True)
    sub = dist.new_group([0, 1])
    rep = communicator_preflight({"world": None, "dup": sub}, torch.device("cpu"), big_bytes=1 << 16, iters=1)
    assert rep["world"]["ok"] and rep["dup"]["ok"] and rep["world"]["world"] == 2
    assert rep["world"]["all_gather_busbw_gbs"] > 0 and rep["world"]["reduce_scatter_busbw_gbs"] > 0


def test_preflight_two_ranks_passes():
    debug_launcher(_ok_two_ranks, num_processes=2)


def _wrong_result():
    import torch
    import torch.distributed as dist

    from accelerate_hpc_test_amd.state import PartialState
    from accelerate_hpc_test_amd.utils import preflight

    PartialState(cpu=True)
    real = dist.all_gather_into_tensor

    def broken(out, inp, group=None, **kw):  # a communicator that delivers garbage
        r = real(out, inp, group=group, **kw)
        out.add_(1.0)
        return r

    dist.all_gather_into_tensor = broken
    try:
        with pytest.raises(preflight.PreflightError, match="world/all_gather"):
            preflight.communicator_preflight({"world": None}, torch.device("cpu"), big_bytes=1 << 16, iters=1,
                                             hard_exit=False)
    finally:
        dist.all_gather_into_tensor = real


def test_preflight_wrong_result_names_the_operation():
    debug_launcher(_wrong_result, num_processes=1)


_HANG = """
import time, torch, torch.distributed as dist
from accelerate_hpc_test_amd.utils import preflight
dist.init_process_group("gloo", rank=0, world_size=1)
dist.reduce_scatter_tensor = lambda *a, **k: time.sleep(60)   # a collective that never completes
preflight.communicator_preflight({"world": None}, torch.device("cpu"), big_bytes=1 << 16, timeout_s=2.0)
print("UNREACHABLE")
"""


def test_preflight_stuck_collective_exits_with_json(tmp_path):
    from accelerate_hpc_test_amd.utils.other import get_free_port

    script = tmp_path / "hang.py"
    script.write_text(_HANG)
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(get_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0", HF_HOME=str(tmp_path))
    r = subprocess.run([sys.executable, str(script)], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["preflight_error"]["group"] == "world" and rec["preflight_error"]["op"] == "reduce_scatter"
    assert "UNREACHABLE" not in r.stdout
