"""BASELINE config #1: examples/nlp_example.py (BERT MRPC-shaped, CPU) through the Accelerator API — single process
and a 2-rank gloo launch via `accelerate-amd launch` (parity: reference tests/test_examples.py)."""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "examples"))

transformers = pytest.importorskip("transformers")


def _port() -> str:
    """A free rendezvous port per launch: parallel test workers must not share the default 29500."""
    from accelerate_hpc_test_amd.utils.other import get_free_port

    return str(get_free_port())


def test_nlp_example_cpu_learns():
    import nlp_example

    metric = nlp_example.main(["--cpu", "--tiny", "--num_epochs", "3", "--n_train", "512", "--n_eval", "128"])
    assert metric["accuracy"] > 0.9, metric


def test_nlp_example_two_ranks_via_launch(tmp_path):
    cfg = tmp_path / "cpu2.yaml"
    cfg.write_text("compute_environment: LOCAL_MACHINE\ndistributed_type: MULTI_CPU\nnum_processes: 2\nuse_cpu: true\nmixed_precision: 'no'\n")
    env = dict(os.environ, HF_HOME=str(tmp_path), PYTHONPATH=REPO)
    r = subprocess.run(
        [sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch",
         "--main_process_port", _port(), "--config_file", str(cfg),
         os.path.join(REPO, "examples", "nlp_example.py"), "--cpu", "--tiny", "--num_epochs", "2", "--n_train", "256", "--n_eval", "64"],
        cwd=REPO, env=env, capture_output=True, text=True, timeout=600,
    )
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "epoch 1:" in r.stdout


def test_complete_nlp_example_checkpoint_and_resume(tmp_path):
    """examples/complete_nlp_example.py: step and epoch checkpoints, a mid-epoch resume (skip_first_batches on the
    restored loader position), and a run that still learns after resuming."""
    import complete_nlp_example

    out = str(tmp_path / "run")
    common = ["--cpu", "--tiny", "--num_epochs", "3", "--n_train", "512", "--n_eval", "128", "--output_dir", out]
    first = complete_nlp_example.main(common + ["--checkpointing_steps", "40"])
    assert first["accuracy"] > 0.9, first
    saved = sorted(os.listdir(out))
    assert "step_40" in saved and "step_80" in saved, saved
    resumed = complete_nlp_example.main(common + ["--resume_from_checkpoint", os.path.join(out, "step_40")])
    assert resumed["accuracy"] > 0.9, resumed


def test_cv_example_cpu_learns():
    import cv_example

    metric = cv_example.main(["--cpu", "--image_size", "32", "--n_train", "512", "--n_eval", "128", "--num_epochs", "4",
                              "--batch_size", "32"])
    assert metric["accuracy"] > 0.9, metric


def test_config_templates_load_and_launch(tmp_path):
    """examples/config_yaml_templates: every file parses with the launcher's schema; run_me.py launches with the
    single-accelerator template (on CPU) and with a 2-rank CPU variant of the DDP template."""
    import glob

    import yaml

    from accelerate_hpc_test_amd.commands.config.config_args import load_config_from_file

    files = sorted(glob.glob(os.path.join(REPO, "examples", "config_yaml_templates", "*.yaml")))
    assert len(files) == 5
    for f in files:
        cfg = load_config_from_file(f)
        assert cfg.num_processes >= 1, f
    env = dict(os.environ, HF_HOME=str(tmp_path), PYTHONPATH=REPO)
    script = os.path.join(REPO, "examples", "config_yaml_templates", "run_me.py")
    ddp = yaml.safe_load(open(os.path.join(REPO, "examples", "config_yaml_templates", "multi_gpu.yaml")))
    ddp.update(distributed_type="MULTI_CPU", num_processes=2, use_cpu=True, mixed_precision="no")
    cpu2 = tmp_path / "cpu2.yaml"
    cpu2.write_text(yaml.safe_dump(ddp))
    for cfg, extra, expect in ((os.path.join(REPO, "examples", "config_yaml_templates", "single_accelerator.yaml"),
                                ["--cpu"], "num_processes=1"), (str(cpu2), [], "num_processes=2")):
        r = subprocess.run([sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch",
         "--main_process_port", _port(),
                            "--config_file", cfg, *extra, script], cwd=REPO, env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        assert expect in r.stdout and "final loss" in r.stdout, r.stdout


@pytest.mark.parametrize("script,expect", [
    ("examples/inference/pippy/llama.py", "max |staged - unsplit| = 0.00e+00"),
    ("examples/inference/pippy/bert.py", "BertForMaskedLM: stages=2"),
    ("examples/inference/pippy/gpt2.py", "GPT2ForSequenceClassification: stages=2"),
    ("examples/inference/pippy/t5.py", "T5ForConditionalGeneration: stages=2"),
    ("examples/inference/distributed/llama_generation.py", "generated 10 completions on 2 process(es)"),
    ("examples/alst_ulysses_sequence_parallelism/sp_ulysses.py", "local tokens 32 of 64"),
])
def test_inference_and_sequence_parallel_examples_two_ranks(tmp_path, script, expect):
    """Pipeline inference (prepare_pippy), split_between_processes generation and Ulysses SP training, each launched
    on 2 CPU ranks through `accelerate-amd launch` (reference examples/inference/*, examples/alst_ulysses_*)."""
    env = dict(os.environ, HF_HOME=str(tmp_path), PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch",
         "--main_process_port", _port(), "--cpu",
                        "--num_processes", "2", os.path.join(REPO, script), "--cpu"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert expect in r.stdout, r.stdout[-2000:]


def test_complete_cv_example_epoch_checkpoint_and_resume(tmp_path):
    """examples/complete_cv_example.py: epoch and step checkpoints, resume from both, still learns."""
    import complete_cv_example

    out = str(tmp_path / "cv")
    common = ["--cpu", "--image_size", "32", "--n_train", "256", "--n_eval", "128", "--batch_size", "32",
              "--num_epochs", "3", "--output_dir", out]
    first = complete_cv_example.main(common + ["--checkpointing_steps", "epoch"])
    assert sorted(os.listdir(out)) == ["epoch_0", "epoch_1", "epoch_2"]
    resumed = complete_cv_example.main(common + ["--resume_from_checkpoint", os.path.join(out, "epoch_1")])
    assert resumed["accuracy"] > 0.5 and first["accuracy"] > 0.5, (first, resumed)
    step_out = str(tmp_path / "cv_steps")
    steps = ["--output_dir", step_out, "--checkpointing_steps", "5"]
    complete_cv_example.main(common[:-2] + steps)
    res = complete_cv_example.main(common[:-2] + steps[:2] + ["--resume_from_checkpoint", os.path.join(step_out, "step_10")])
    assert res["accuracy"] > 0.5, res
