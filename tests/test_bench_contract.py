"""The driver's bench.py contract at N > 1, on CPU ranks: `torch.distributed.run` with 2 gloo ranks and a small model
(`--cpu --model llama-tiny`) runs the same loop as the GPU bench (FSDP2 engine, warm-up, barrier-bracketed timed
steps, MAX of the elapsed time over ranks) and rank 0 alone prints ONE JSON line with the required fields."""

import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_prints_one_json_line(tmp_path):
    from accelerate_hpc_test_amd.utils.other import get_free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(get_free_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--model", "llama-tiny", "--seq", "256", "--cpu"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, PYTHONPATH=REPO, HF_HOME=str(tmp_path)))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1 and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 2 and rec["config"]["seq_len"] == 256 and rec["config"]["model"] == "llama-tiny"
    assert rec["config"]["parallelism"] == "fsdp-w2" and rec["vs_baseline"] is None  # not the headline model
    pf = rec["preflight"]  # every communicator checked before training (utils/preflight.py)
    assert pf["world"]["ok"] and pf["fsdp_all_gather"]["ok"] and pf["fsdp_reduce_scatter"]["ok"], pf
    # value is the whole-job rate: all ranks' tokens over the slowest rank's timed window
    tokens = 2 * 1 * 256 * 2
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] * 2 / 1000)) / rec["value"] < 0.01, rec


def test_bench_spawns_its_own_ranks(tmp_path):
    """`python bench.py --gpus 2` with no launcher (the driver's SCALE form): bench.py starts torch.distributed.run as a
    child, every rank trains, and exactly one JSON line reports n_gpus=2 on the sharded path."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "llama-tiny", "--seq",
           "256", "--cpu"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600,
                       env=dict(env, PYTHONPATH=REPO, HF_HOME=str(tmp_path)))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "fsdp-w2" and rec["config"]["global_batch"] == 2


def test_rccl_bench_tool_gloo_plumbing():
    """tools/bench_rccl.py (the xGMI collective bandwidth sweep) on 2 gloo ranks: one JSON line per (op, size) from rank 0,
    bus bandwidth following the rccl-tests factors."""
    from accelerate_hpc_test_amd.utils.other import get_free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(get_free_port()), "tools/bench_rccl.py", "--cpu", "--max-mb", "2", "--iters", "2"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=dict(os.environ, PYTHONPATH=REPO))
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert {(x["op"], x["bytes"]) for x in recs} == {(op, b) for op in ("all_gather", "all_reduce") for b in (1 << 20, 2 << 20)}
    for x in recs:
        f = 0.5 if x["op"] == "all_gather" else 1.0
        assert abs(x["busbw_GBs"] - x["algbw_GBs"] * f) <= 0.011 + 0.01 * x["algbw_GBs"], x


def test_bench_rejects_world_size_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", PYTHONPATH=REPO, HF_HOME=str(tmp_path))
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--cpu", "--model", "llama-tiny"], cwd=REPO,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "must match" in r.stderr
