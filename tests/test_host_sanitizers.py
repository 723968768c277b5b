"""Host-side sanitizers for the native runtime's CPU code: tests/native/host_sanitize.cpp is built with
g++ -fsanitize=address,undefined against csrc/runtime/host_kernels.h (the OpenMP host AdamW used by FSDP CPU offload,
bf16 rounding, the collective-sequence digest) and run; any sanitizer report or numerics mismatch fails the test.
GPU-side AddressSanitizer is not available on this pool, so the HIP kernels rely on their numerics tests."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_runtime_under_address_and_ub_sanitizers(tmp_path):
    exe = tmp_path / "host_sanitize"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fopenmp", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "accelerate_hpc_test_amd", "csrc", "runtime"),
           os.path.join(ROOT, "tests", "native", "host_sanitize.cpp"), "-o", str(exe)]
    build = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if build.returncode != 0 and "asan" in build.stderr.lower():
        pytest.skip("sanitizer runtime not installed: " + build.stderr[-300:])
    assert build.returncode == 0, build.stderr[-2000:]
    # verify_asan_link_order=0: an environment that preloads a library of its own is left as it is
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="4")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0, (run.stdout[-2000:], run.stderr[-4000:])
    assert "0 failure(s)" in run.stdout and "ERROR: AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr
