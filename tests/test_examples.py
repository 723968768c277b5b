"""BASELINE config #1: examples/nlp_example.py (BERT MRPC-shaped, CPU) through the Accelerator API — single process
and a 2-rank gloo launch via `accelerate-amd launch` (parity: reference tests/test_examples.py)."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "examples"))

transformers = pytest.importorskip("transformers")


def test_nlp_example_cpu_learns():
    import nlp_example

    metric = nlp_example.main(["--cpu", "--tiny", "--num_epochs", "3", "--n_train", "512", "--n_eval", "128"])
    assert metric["accuracy"] > 0.9, metric


def test_nlp_example_two_ranks_via_launch(tmp_path):
    cfg = tmp_path / "cpu2.yaml"
    cfg.write_text("compute_environment: LOCAL_MACHINE\ndistributed_type: MULTI_CPU\nnum_processes: 2\nuse_cpu: true\nmixed_precision: 'no'\n")
    env = dict(os.environ, HF_HOME=str(tmp_path), PYTHONPATH=REPO)
    r = subprocess.run(
        [sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch", "--config_file", str(cfg),
         os.path.join(REPO, "examples", "nlp_example.py"), "--cpu", "--tiny", "--num_epochs", "2", "--n_train", "256", "--n_eval", "64"],
        cwd=REPO, env=env, capture_output=True, text=True, timeout=600,
    )
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "epoch 1:" in r.stdout
