"""notebook_launcher on CPU workers: elastic restarts after an injected failure, and the monitor ending a job whose
peer failed while another rank hangs. Parity: the reference's test_utils/scripts/test_notebook.py
(`test_fault_tolerant`, `test_monitoring`), which needs >= 2 processes; here the workers are forked CPU processes."""

import os
import time

import pytest

from accelerate_hpc_test_amd import notebook_launcher


def _fail_on_first_attempt(out_dir):
    # torch elastic exports the attempt number to every worker
    attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    rank = os.environ["LOCAL_RANK"]
    if attempt == 0:
        raise RuntimeError(f"injected failure on rank {rank}, attempt 0")
    with open(os.path.join(out_dir, f"done_{rank}"), "w") as f:
        f.write(str(attempt))


def _even_raises_odd_sleeps(sleep_s):
    if int(os.environ["LOCAL_RANK"]) % 2 == 0:
        raise RuntimeError("even rank failed")
    time.sleep(sleep_s)


def test_notebook_launcher_restarts_after_failure(tmp_path):
    notebook_launcher(_fail_on_first_attempt, (str(tmp_path),), num_processes=2, max_restarts=2, monitor_interval=0.1)
    for r in range(2):
        assert (tmp_path / f"done_{r}").read_text() == "1"


def test_notebook_launcher_monitor_stops_hung_peer():
    from torch.distributed.elastic.multiprocessing.errors import ChildFailedError

    t0 = time.time()
    with pytest.raises(ChildFailedError, match="even rank failed"):
        notebook_launcher(_even_raises_odd_sleeps, (120,), num_processes=2, monitor_interval=0.05)
    assert time.time() - t0 < 60, "the elastic monitor did not stop the sleeping rank"
