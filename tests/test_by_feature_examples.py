"""Every examples/by_feature script runs end to end on CPU with the tiny BERT (parity: the reference's
`FeatureExamplesTests`, tests/test_examples.py:158-320, which launch each by_feature example on mocked data), plus a
checkpoint → resume round trip and two-rank launches of the gradient-sync examples."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FEAT = os.path.join(REPO, "examples", "by_feature")
sys.path.insert(0, FEAT)

pytest.importorskip("transformers")

TINY = ["--cpu", "--tiny", "--num_epochs", "1", "--n_train", "96", "--n_eval", "40"]


def _port() -> str:
    """A free rendezvous port per launch: parallel test workers must not share the default 29500."""
    from accelerate_hpc_test_amd.utils.other import get_free_port

    return str(get_free_port())


@pytest.mark.parametrize(
    "name",
    ["gradient_accumulation", "early_stopping", "local_sgd", "tracking", "memory", "multi_process_metrics",
     "ddp_comm_hook", "fsdp_with_peak_mem_tracking", "automatic_gradient_accumulation"],
)
def test_feature_example_runs(name):
    import importlib

    mod = importlib.import_module(name)
    out = mod.main(TINY)
    assert out is not None


def test_cross_validation_example():
    import cross_validation

    m = cross_validation.main(TINY + ["--num_folds", "2"])
    assert 0.0 <= m["accuracy"] <= 1.0


def test_profiler_example_writes_trace(tmp_path):
    import profiler

    profiler.main(TINY + ["--output_trace_dir", str(tmp_path), "--steps", "5"])
    assert (tmp_path / "profile_0.json").exists()


def test_autoregressive_gradient_accumulation_example():
    import gradient_accumulation_for_autoregressive_models as ex

    losses = ex.main(["--cpu", "--steps", "3", "--gradient_accumulation_steps", "2", "--seq_len", "64"])
    assert len(losses) == 3 and losses[-1] < losses[0] + 1.0


def test_checkpointing_example_resume(tmp_path):
    import checkpointing

    checkpointing.main(TINY + ["--num_epochs", "2", "--checkpointing_steps", "4", "--output_dir", str(tmp_path)])
    saved = sorted((p for p in os.listdir(tmp_path) if p.startswith("step_")), key=lambda p: int(p[5:]))
    assert saved, os.listdir(tmp_path)
    ckpt = tmp_path / saved[0]
    assert (ckpt / "model.safetensors").exists() and (ckpt / "optimizer.bin").exists()
    m = checkpointing.main(TINY + ["--num_epochs", "2", "--resume_from_checkpoint", str(ckpt), "--output_dir", str(tmp_path / "r")])
    assert m is not None


@pytest.mark.parametrize("name", ["gradient_accumulation", "ddp_comm_hook", "multi_process_metrics"])
def test_feature_example_two_ranks(name, tmp_path):
    cfg = tmp_path / "cpu2.yaml"
    cfg.write_text("compute_environment: LOCAL_MACHINE\ndistributed_type: MULTI_CPU\nnum_processes: 2\nuse_cpu: true\nmixed_precision: 'no'\n")
    env = dict(os.environ, HF_HOME=str(tmp_path), PYTHONPATH=REPO)
    r = subprocess.run(
        [sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch",
         "--main_process_port", _port(), "--config_file", str(cfg),
         os.path.join(FEAT, f"{name}.py"), *TINY],
        cwd=REPO, env=env, capture_output=True, text=True, timeout=600,
    )
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "epoch 0:" in r.stdout
