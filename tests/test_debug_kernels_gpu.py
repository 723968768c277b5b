"""Debug build of the HIP kernels (device-side bounds checks compiled in with ACC_DEBUG_BOUNDS): one
kernel per family runs clean on valid inputs and matches the release build; deliberate violations are caught (check
id + kernel source line reported by `debug_status()`) without the faulting access taking place."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_debug_kernels_catch_violations_and_match_release():
    script = os.path.join(REPO, "accelerate_hpc_test_amd", "test_utils", "scripts", "debug_kernels_check.py")
    env = dict(os.environ, ACCELERATE_DEBUG_KERNELS="1", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, script], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(res)
    for name, f in res["families"].items():
        assert f["status"] == 0, (name, f)  # no check fires on valid inputs
        assert f["max_diff"] <= (1e-5 if name == "adamw" else 0.0), (name, f)  # same results as the release build
    assert res["selftest_status"] >> 32 == 99 and res["selftest_guard_untouched"], res
    assert res["bad_label_status"] >> 32 == 5, res  # kChkXentLabel, with the kernel's source line
    assert res["after_clear"] == 0, res
