"""CLI / config-file tests (parity: reference tests/test_cli.py, tests/test_configs/*).

Config fixtures are written inline: they carry the same key sets as the reference's historical config files
(0.11 / 0.12 era, MPI, fp8, FSDP1, invalid keys) so that compatibility with files produced by the reference's
`accelerate config` is pinned.
"""

import os
import subprocess
import sys
import textwrap

import pytest
import yaml

from accelerate_hpc_test_amd.commands.accelerate_cli import build_parser
from accelerate_hpc_test_amd.commands.config import ClusterConfig, load_config_from_file, write_basic_config
from accelerate_hpc_test_amd.commands.config.cluster import get_cluster_input
from accelerate_hpc_test_amd.commands.estimate import estimate_command_parser, gather_data
from accelerate_hpc_test_amd.commands.launch import _validate_launch_command, launch_command_parser
from accelerate_hpc_test_amd.commands.to_fsdp2 import convert_config_to_fsdp2
from accelerate_hpc_test_amd.utils.dataclasses import DistributedType
from accelerate_hpc_test_amd.utils.launch import (
    _convert_nargs_to_dict,
    build_torchrun_cmd,
    prepare_multi_gpu_env,
    prepare_simple_launcher_cmd_env,
)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    "legacy_0_11.yaml": """
        compute_environment: LOCAL_MACHINE
        deepspeed_config: {}
        distributed_type: 'NO'
        fsdp_config: {}
        machine_rank: 0
        main_process_ip: null
        main_process_port: null
        main_training_function: main
        mixed_precision: 'no'
        num_machines: 1
        num_processes: 1
        use_cpu: false
    """,
    "legacy_fp16.yaml": """
        compute_environment: LOCAL_MACHINE
        distributed_type: 'NO'
        fp16: true
        dynamo_backend: INDUCTOR
        num_processes: 1
    """,
    "mpi.yaml": """
        compute_environment: LOCAL_MACHINE
        debug: false
        distributed_type: MULTI_CPU
        downcast_bf16: 'no'
        machine_rank: 0
        main_process_ip: 127.0.0.1
        main_process_port: 29500
        main_training_function: main
        mixed_precision: 'no'
        mpirun_config:
          mpirun_hostfile: /tmp/hostfile
        num_machines: 4
        num_processes: 16
        rdzv_backend: static
        same_network: true
        tpu_env: []
        tpu_use_cluster: false
        tpu_use_sudo: false
        use_cpu: true
    """,
    "fp8.yaml": """
        compute_environment: LOCAL_MACHINE
        debug: false
        distributed_type: MULTI_GPU
        enable_cpu_affinity: false
        fp8_config:
          amax_compute_algo: max
          amax_history_len: 1024
          backend: TE
          fp8_format: E4M3
          interval: 1
          margin: 0
          use_autocast_during_eval: false
        gpu_ids: all
        machine_rank: 0
        main_training_function: main
        mixed_precision: fp8
        num_machines: 1
        num_processes: 2
        rdzv_backend: static
        same_network: true
        use_cpu: false
    """,
    "fsdp1.yaml": """
        compute_environment: LOCAL_MACHINE
        debug: false
        distributed_type: FSDP
        enable_cpu_affinity: false
        fsdp_config:
          fsdp_activation_checkpointing: false
          fsdp_auto_wrap_policy: TRANSFORMER_BASED_WRAP
          fsdp_backward_prefetch: BACKWARD_PRE
          fsdp_cpu_ram_efficient_loading: true
          fsdp_forward_prefetch: false
          fsdp_offload_params: false
          fsdp_sharding_strategy: SHARD_GRAD_OP
          fsdp_state_dict_type: SHARDED_STATE_DICT
          fsdp_sync_module_states: true
          fsdp_transformer_layer_cls_to_wrap: LlamaDecoderLayer
          fsdp_use_orig_params: true
        machine_rank: 0
        main_training_function: main
        mixed_precision: bf16
        num_machines: 1
        num_processes: 8
        rdzv_backend: static
        same_network: true
        use_cpu: false
    """,
    "invalid.yaml": """
        compute_environment: LOCAL_MACHINE
        distributed_type: 'NO'
        mixed_precision: 'no'
        num_processes: 1
        use_cpu: false
        invalid_key: "invalid_value"
        another_invalid_key: "another_invalid_value"
    """,
    "multi_cpu2.yaml": """
        compute_environment: LOCAL_MACHINE
        distributed_type: MULTI_CPU
        mixed_precision: 'no'
        num_machines: 1
        num_processes: 2
        use_cpu: true
        main_process_ip: 127.0.0.1
    """,
}


@pytest.fixture
def cfgdir(tmp_path):
    for name, body in CONFIGS.items():
        (tmp_path / name).write_text(textwrap.dedent(body))
    return tmp_path


@pytest.mark.parametrize("name", ["legacy_0_11.yaml", "mpi.yaml", "fp8.yaml", "fsdp1.yaml"])
def test_config_files_load(cfgdir, name):
    cfg = load_config_from_file(str(cfgdir / name))
    assert isinstance(cfg, ClusterConfig)
    # round trip through YAML and JSON
    for ext in ("yaml", "json"):
        out = cfgdir / f"rt.{ext}"
        cfg.save(out)
        again = load_config_from_file(str(out))
        assert again.to_dict() == cfg.to_dict()


def test_legacy_key_migration(cfgdir):
    cfg = load_config_from_file(str(cfgdir / "legacy_fp16.yaml"))
    assert cfg.mixed_precision == "fp16"
    assert cfg.dynamo_config == {"dynamo_backend": "INDUCTOR"}
    assert cfg.debug is False and cfg.use_cpu is False


def test_invalid_keys_rejected(cfgdir):
    with pytest.raises(ValueError, match="another_invalid_key"):
        load_config_from_file(str(cfgdir / "invalid.yaml"))


def test_missing_config_file():
    with pytest.raises(FileNotFoundError):
        load_config_from_file("/nonexistent/cfg.yaml")


def test_write_basic_config(tmp_path):
    path = tmp_path / "sub" / "default_config.yaml"
    out = write_basic_config("bf16", str(path))
    assert out and path.exists()
    cfg = load_config_from_file(str(path))
    assert cfg.mixed_precision == "bf16"
    assert write_basic_config("bf16", str(path)) is False
    with pytest.raises(ValueError):
        write_basic_config("int3", str(tmp_path / "x.yaml"))


def test_questionnaire_fsdp(tmp_path):
    # env, nodes, paradigm=FSDP2, debug, compile?, reshard, offload, wrap, cls, sd type, ram-eff, ckpt, nproc, gpu ids, affinity, precision
    answers = ["0", "1", "3", "no", "no", "yes", "no", "0", "LlamaDecoderLayer", "2", "yes", "no", "8", "all", "yes", "1"]
    cfg = get_cluster_input(answers)
    assert cfg.distributed_type == DistributedType.FSDP
    assert cfg.mixed_precision == "bf16"
    assert cfg.num_processes == 8
    assert cfg.fsdp_config["fsdp_transformer_layer_cls_to_wrap"] == "LlamaDecoderLayer"
    assert cfg.fsdp_config["fsdp_state_dict_type"] == "SHARDED_STATE_DICT"
    assert cfg.fsdp_config["fsdp_version"] == 2
    p = tmp_path / "q.yaml"
    cfg.save(p)
    assert load_config_from_file(str(p)).to_dict() == cfg.to_dict()


def test_launch_config_merge_fsdp(cfgdir):
    args = launch_command_parser().parse_args(["--config_file", str(cfgdir / "fsdp1.yaml"), "train.py", "--lr", "1"])
    args = _validate_launch_command(args)
    assert args.use_fsdp and not args.multi_gpu
    assert args.num_processes == 8
    assert args.mixed_precision == "bf16"
    assert args.fsdp_transformer_layer_cls_to_wrap == "LlamaDecoderLayer"
    assert args.fsdp_sharding_strategy == "SHARD_GRAD_OP"
    assert args.training_script_args == ["--lr", "1"]
    env = prepare_multi_gpu_env(args)
    assert env["ACCELERATE_USE_FSDP"] == "true"
    assert env["FSDP_TRANSFORMER_CLS_TO_WRAP"] == "LlamaDecoderLayer"
    assert env["FSDP_SHARDING_STRATEGY"] == "SHARD_GRAD_OP"
    assert env["FSDP_STATE_DICT_TYPE"] == "SHARDED_STATE_DICT"
    assert env["ACCELERATE_MIXED_PRECISION"] == "bf16"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert args.nproc_per_node == "8" and args.master_addr == "127.0.0.1"
    cmd = build_torchrun_cmd(args)
    assert "--nproc-per-node=8" in cmd and cmd[-3:] == ["train.py", "--lr", "1"]


def test_launch_cli_overrides_config(cfgdir):
    args = launch_command_parser().parse_args(
        ["--config_file", str(cfgdir / "fsdp1.yaml"), "--mixed-precision", "fp8", "--num-processes", "4", "train.py"]
    )
    args = _validate_launch_command(args)
    assert args.mixed_precision == "fp8" and args.num_processes == 4


def test_launch_fp8_env(cfgdir):
    args = launch_command_parser().parse_args(["--config_file", str(cfgdir / "fp8.yaml"), "train.py"])
    args = _validate_launch_command(args)
    assert args.multi_gpu
    env = prepare_multi_gpu_env(args)
    assert env["ACCELERATE_MIXED_PRECISION"] == "fp8"
    assert env["ACCELERATE_FP8_FORMAT"] == "E4M3"
    assert env["ACCELERATE_FP8_AMAX_COMPUTE_ALGO"] == "max"
    assert env["ACCELERATE_FP8_BACKEND"] == "TE"


def test_launch_parallelism_and_deepspeed_translation():
    args = launch_command_parser().parse_args(
        ["--use_fsdp", "--fsdp_version", "2", "--use_parallelism_config", "--parallelism_config_tp_size", "2",
         "--parallelism_config_dp_shard_size", "4", "--num_processes", "8", "x.py"]
    )
    args = _validate_launch_command(args)
    env = prepare_multi_gpu_env(args)
    assert env["ACCELERATE_USE_PARALLELISM_CONFIG"] == "true"
    assert env["PARALLELISM_CONFIG_TP_SIZE"] == "2" and env["PARALLELISM_CONFIG_DP_SHARD_SIZE"] == "4"

    args = launch_command_parser().parse_args(["--use_deepspeed", "--zero_stage", "3", "--num_processes", "2", "x.py"])
    args = _validate_launch_command(args)
    env = prepare_multi_gpu_env(args)
    assert env["ACCELERATE_USE_FSDP"] == "true" and env["FSDP_RESHARD_AFTER_FORWARD"] == "true"
    args = launch_command_parser().parse_args(["--use_deepspeed", "--zero_stage", "2", "--num_processes", "2", "x.py"])
    env = prepare_multi_gpu_env(_validate_launch_command(args))
    assert env["FSDP_SHARDING_STRATEGY"] == "SHARD_GRAD_OP"


def test_launch_validation_errors():
    with pytest.raises(ValueError):
        _validate_launch_command(launch_command_parser().parse_args(["--cpu", "--multi_gpu", "x.py"]))
    with pytest.raises(ValueError):
        _validate_launch_command(launch_command_parser().parse_args(["--multi_gpu", "--num_processes", "1", "x.py"]))


def test_simple_launcher_env():
    args = launch_command_parser().parse_args(["--mixed_precision", "bf16", "--gpu_ids", "3", "-m", "pkg.mod", "--a", "b"])
    args = _validate_launch_command(args)
    cmd, env = prepare_simple_launcher_cmd_env(args)
    assert cmd[1:] == ["-m", "pkg.mod", "--a", "b"]
    assert env["HIP_VISIBLE_DEVICES"] == "3" and env["ACCELERATE_MIXED_PRECISION"] == "bf16"


def test_nargs_to_dict():
    assert _convert_nargs_to_dict(["--lr", "3e-4", "--flag", "--name", "x", "--n=3"]) == {"lr": 3e-4, "flag": True, "name": "x", "n": 3}


def test_to_fsdp2_conversion():
    cfg = yaml.safe_load(textwrap.dedent(CONFIGS["fsdp1.yaml"]))
    new = convert_config_to_fsdp2(cfg)["fsdp_config"]
    assert new["fsdp_version"] == 2
    assert new["fsdp_reshard_after_forward"] is False  # SHARD_GRAD_OP
    for removed in ("fsdp_backward_prefetch", "fsdp_sync_module_states", "fsdp_use_orig_params", "fsdp_forward_prefetch"):
        assert removed not in new
    assert new["fsdp_transformer_layer_cls_to_wrap"] == "LlamaDecoderLayer"


def test_estimate_memory_preset():
    args = estimate_command_parser().parse_args(["llama3-8b", "--dtypes", "float32", "bfloat16", "--num_gpus", "8"])
    rows, fsdp = gather_data(args)
    total32 = rows[0][2]
    assert 7.9e9 * 4 < total32 < 8.2e9 * 4
    assert rows[1][2] == total32 / 2
    assert 15e9 < fsdp < 30e9  # ~18 B/param / 8 + unsharded layer


def test_root_parser_has_all_commands():
    parser = build_parser()
    sub = [a for a in parser._actions if a.__class__.__name__ == "_SubParsersAction"][0]
    assert set(sub.choices) >= {"config", "env", "estimate-memory", "launch", "merge-weights", "test", "to-fsdp2"}


def _run(cmd, env=None, timeout=240):
    e = os.environ.copy()
    e["PYTHONPATH"] = REPO + os.pathsep + e.get("PYTHONPATH", "")
    e.update(env or {})
    return subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=timeout)


def test_launch_end_to_end_multi_cpu(cfgdir, tmp_path):
    """`accelerate-amd launch` with a 2-process MULTI_CPU config runs the bundled sanity script over gloo."""
    script = os.path.join(REPO, "accelerate_hpc_test_amd", "test_utils", "scripts", "test_script.py")
    r = _run([sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch", "--config_file", str(cfgdir / "multi_cpu2.yaml"), script],
             env={"HF_HOME": str(tmp_path)})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Training parity vs single process" in r.stdout


def test_env_command(cfgdir):
    r = _run([sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "env", "--config_file", str(cfgdir / "fp8.yaml")])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "PyTorch version" in r.stdout and "mixed_precision: fp8" in r.stdout


def test_opt_in_upstream_command_aliases(tmp_path):
    """`accelerate-amd aliases install --dir D` writes the reference's command names (accelerate, accelerate-launch,
    ...) as launchers of this CLI; they run, refuse to overwrite foreign files, and `remove` deletes only ours."""
    import subprocess
    import sys

    from accelerate_hpc_test_amd.commands import aliases
    from accelerate_hpc_test_amd.commands.accelerate_cli import main

    d = tmp_path / "bin"
    main(["aliases", "install", "--dir", str(d)])
    assert sorted(p.name for p in d.iterdir()) == sorted(aliases.ALIASES)
    out = subprocess.run([str(d / "accelerate"), "env"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "accelerate_hpc_test_amd" in out.stdout + out.stderr
    out = subprocess.run([str(d / "accelerate-launch"), "--help"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "num_processes" in out.stdout
    assert aliases.listed(str(d))["accelerate-config"] == "installed"
    foreign = tmp_path / "other"
    foreign.mkdir()
    (foreign / "accelerate-merge-weights").write_text("#!/bin/sh\necho upstream\n")  # the LAST alias written
    with pytest.raises(FileExistsError):
        aliases.install(str(foreign))
    assert [p.name for p in foreign.iterdir()] == ["accelerate-merge-weights"]  # refused before writing anything
    (foreign / "accelerate-merge-weights").rename(foreign / "accelerate")
    assert aliases.remove(str(foreign)) == [] and (foreign / "accelerate").exists()
    main(["aliases", "remove", "--dir", str(d)])
    assert list(d.iterdir()) == []


# ---- MPI multi-CPU launches and --debug (reference tests/test_cli.py:117-146, commands/launch.py:870-892) ----------
def _mpi_cmd(cfgdir, version: bytes):
    from unittest.mock import patch

    args = launch_command_parser().parse_args(["--config_file", str(cfgdir / "mpi.yaml"), "train.py", "--cpu"])
    args = _validate_launch_command(args)
    with patch("accelerate_hpc_test_amd.utils.launch.which", return_value=True), \
            patch("accelerate_hpc_test_amd.utils.launch.subprocess.check_output", return_value=version):
        return prepare_simple_launcher_cmd_env(args)


def test_mpi_multicpu_config_cmd_intel(cfgdir):
    cmd, env = _mpi_cmd(cfgdir, b"Intel(R) MPI Library")
    expected = ["mpirun", "-f", "/tmp/hostfile", "-ppn", "4", "-n", "16"]
    assert cmd[: len(expected)] == expected
    assert cmd[len(expected):] == [sys.executable, "train.py", "--cpu"]
    assert "WORLD_SIZE" not in env and env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500"


def test_mpi_multicpu_config_cmd_openmpi(cfgdir):
    cmd, _ = _mpi_cmd(cfgdir, b"mpirun (Open MPI) 4.1.2")
    assert cmd[:9] == ["mpirun", "--hostfile", "/tmp/hostfile", "--npernode", "4", "-n", "16", "--bind-to", "socket"]


def test_mpi_launcher_missing_raises(cfgdir):
    from unittest.mock import patch

    args = _validate_launch_command(launch_command_parser().parse_args(["--config_file", str(cfgdir / "mpi.yaml"), "t.py"]))
    with patch("accelerate_hpc_test_amd.utils.launch.which", return_value=None), pytest.raises(OSError, match="mpirun"):
        prepare_simple_launcher_cmd_env(args)


def test_launch_debug_flag_sets_debug_mode():
    args = _validate_launch_command(launch_command_parser().parse_args(["--debug", "--cpu", "x.py"]))
    assert args.debug
    _, env = prepare_simple_launcher_cmd_env(args)
    assert env["ACCELERATE_DEBUG_MODE"] == "true"


_MISMATCH_SCRIPT = """
import sys
import torch
from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.utils import DistributedOperationException
acc = Accelerator(cpu=True)
t = torch.ones(acc.process_index + 2)  # a different shape on every rank
try:
    acc.gather(t)
except DistributedOperationException as e:
    # one write per line: the two ranks share the launcher's stdout
    sys.stdout.write(f"MISMATCH CAUGHT {acc.process_index} {'Process 1: [3]' in str(e)}\\n")
    sys.stdout.flush()
else:
    print("NO CHECK", acc.process_index)
"""


def test_launch_debug_trips_verify_operation(tmp_path):
    """`launch --debug`: a collective with mismatched shapes raises DistributedOperationException on every rank
    instead of hanging or corrupting (SURVEY §5.2 debug-mode operation checker)."""
    import socket

    script = tmp_path / "mismatch.py"
    script.write_text(_MISMATCH_SCRIPT)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = _run([sys.executable, "-m", "accelerate_hpc_test_amd.commands.accelerate_cli", "launch", "--cpu", "--debug",
              "--num_processes", "2", "--main_process_port", str(port), str(script)], env={"HF_HOME": str(tmp_path)})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("MISMATCH CAUGHT") == 2 and "MISMATCH CAUGHT 0 True\n" in r.stdout, r.stdout[-2000:]
