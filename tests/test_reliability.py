"""Failure detection / fault injection / collective-order checks / gradient-sync oracle / throughput tracking
(SURVEY §5.1-§5.3, §4.3 `test_sync`). CPU only."""

import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

from accelerate_hpc_test_amd import Accelerator, debug_launcher
from accelerate_hpc_test_amd.test_utils.scripts import test_distributed as td
from accelerate_hpc_test_amd.utils import find_executable_batch_size
from accelerate_hpc_test_amd.utils.fault_tolerance import CollectiveLog, FaultInjector, InjectedFault, StepWatchdog
from accelerate_hpc_test_amd.utils.tracing import ThroughputTracker, model_flops_per_token, trace_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _loss():
    w = torch.nn.Parameter(torch.ones(3))
    return (w * 2).sum()


def test_fault_injection_raise_and_nan(monkeypatch):
    monkeypatch.setenv("ACCELERATE_FAULT_INJECT", "0:1:raise,*:0:nan")
    acc = Accelerator(cpu=True)
    loss = _loss()
    acc.backward(loss)  # step 0: loss poisoned (backward of NaN-scaled loss still runs)
    with pytest.raises(InjectedFault):
        acc.backward(_loss())  # step 1 on rank 0
    acc.backward(_loss())  # step 2: nothing
    inj = FaultInjector("*:0:nan", rank=3)
    assert torch.isnan(inj.before_backward(0, torch.tensor(1.0)))
    with pytest.raises(ValueError):
        FaultInjector("0:1:explode")


def test_fault_injection_oom_drives_find_executable_batch_size():
    inj = FaultInjector("0:0:oom,0:1:oom", rank=0)
    step = {"n": 0}
    tried = []

    @find_executable_batch_size(starting_batch_size=64)
    def train(batch_size):
        tried.append(batch_size)
        s = step["n"]
        step["n"] += 1
        inj.before_backward(s, torch.tensor(1.0))
        return batch_size

    assert train() == 51 and tried == [64, 57, 51]


def test_watchdog_warn_fires_without_heartbeat(capfd):
    wd = StepWatchdog(0.3, rank=5, action="warn", poll=0.05)
    try:
        t0 = time.time()
        while not wd.fired and time.time() - t0 < 5:
            time.sleep(0.05)
        assert wd.fired
    finally:
        wd.stop()
    err = capfd.readouterr().err
    assert "[accelerate watchdog] rank 5" in err


def test_watchdog_beats_keep_it_quiet():
    wd = StepWatchdog(0.5, action="warn", poll=0.05)
    try:
        for _ in range(15):
            wd.beat("step")
            time.sleep(0.05)
        assert not wd.fired
    finally:
        wd.stop()


def test_watchdog_kills_injected_hang_in_subprocess():
    script = textwrap.dedent(
        f"""
        import sys, torch
        sys.path.insert(0, {ROOT!r})
        from accelerate_hpc_test_amd import Accelerator
        acc = Accelerator(cpu=True)
        for i in range(3):
            w = torch.nn.Parameter(torch.ones(2))
            acc.backward((w * 3).sum())
        print("unreachable", flush=True)
        """
    )
    env = dict(os.environ, ACCELERATE_FAULT_INJECT="0:1:hang", ACCELERATE_WATCHDOG_TIMEOUT="2")
    t0 = time.time()
    res = subprocess.run([sys.executable, "-c", script], env=env, capture_output=True, text=True, timeout=120)
    assert res.returncode == 86, (res.returncode, res.stderr[-2000:])
    assert "[accelerate watchdog] rank 0" in res.stderr and "before_backward" in res.stderr
    assert "unreachable" not in res.stdout
    assert time.time() - t0 < 100


def test_watchdog_abort_releases_peer_blocked_in_collective():
    """Two gloo ranks: rank 1 hangs before its all-reduce; its watchdog (action "abort") aborts the communicators and
    exits 86, and rank 0 — blocked in the same all-reduce — gets an error instead of hanging until the PG timeout."""
    script = textwrap.dedent(
        f"""
        import os, sys, time, torch, torch.distributed as dist
        sys.path.insert(0, {ROOT!r})
        from accelerate_hpc_test_amd.utils.fault_tolerance import StepWatchdog
        rank = int(sys.argv[1])
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=rank, world_size=2)
        dist.barrier()
        if rank == 1:
            StepWatchdog(2.0, rank=1, action="abort", poll=0.1)
            time.sleep(120)  # hung before the collective
        try:
            dist.all_reduce(torch.ones(4))
            print("completed", flush=True)
        except Exception as exc:
            print("collective failed:", type(exc).__name__, flush=True)
            os._exit(3)  # skip interpreter teardown: destroying the broken gloo context there can abort (SIGABRT)
        """
    )
    from accelerate_hpc_test_amd.utils.other import get_free_port

    port = str(get_free_port())
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, "-c", script, str(r), port], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for r in range(2)]
    try:
        outs = [p.communicate(timeout=90) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert procs[1].returncode == 86, outs[1][1][-2000:]
    assert "[accelerate watchdog] rank 1" in outs[1][1]
    assert procs[0].returncode == 3 and "collective failed" in outs[0][0], (procs[0].returncode, outs[0])
    assert time.time() - t0 < 80


def test_collective_log_digest_is_order_sensitive():
    log = CollectiveLog()
    log.record("all_reduce", 2, torch.float32, 10)
    log.record("all_gather", 2, torch.bfloat16, 4)
    a = log.digest()
    log.reset()
    log.record("all_gather", 2, torch.bfloat16, 4)
    log.record("all_reduce", 2, torch.float32, 10)
    assert log.digest() != a and log.count() == 2


@pytest.mark.parametrize("mismatch", [False, True])
def test_collective_sequence_check(mismatch):
    debug_launcher(td.check_collective_sequence, args=(mismatch,), num_processes=2)


@pytest.mark.parametrize("mode,each", [("no_sync", False), ("accumulate", False), ("accumulate", True), ("trigger", False)])
def test_grad_sync_oracle(mode, each):
    debug_launcher(td.check_grad_sync, args=(mode, each), num_processes=2)


def test_throughput_tracker_contract():
    tr = ThroughputTracker(warmup_steps=2, num_processes=4)
    assert tr.step(100) == {}
    assert tr.step(100) == {"warmup_completed": True}
    time.sleep(0.01)
    m = tr.step(100, model_flops_per_token=1e9)
    assert m["total_tokens"] == 100 and m["tokens_per_second_whole_job"] == pytest.approx(4 * m["tokens_per_second"])
    assert m["tflops_per_device"] > 0
    assert "tokens/s" in ThroughputTracker.get_print_message(m)


def test_model_flops_per_token_matches_llama_config():
    from transformers import LlamaConfig as HFLlamaConfig

    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS

    ours = LLAMA_PRESETS["llama3-8b"]
    hf = HFLlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                       num_attention_heads=32, num_key_value_heads=8)
    a, b = model_flops_per_token(ours, 8192), model_flops_per_token(hf, 8192)
    assert abs(a - b) / a < 1e-3, (a, b)
    assert 5.0e10 < a < 6.0e10  # ≈ 5.5e10 FLOP/token


def test_trace_range_shows_in_profiler():
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        with trace_range("acc.test_region"):
            torch.ones(4).sum()
    assert any(e.name == "acc.test_region" for e in prof.events())
