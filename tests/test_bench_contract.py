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
    assert rec["config"]["parallelism"] == "fsdp2" and rec["vs_baseline"] is None  # not the headline model
    # value is the whole-job rate: all ranks' tokens over the slowest rank's timed window
    tokens = 2 * 1 * 256 * 2
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] * 2 / 1000)) / rec["value"] < 0.01, rec
