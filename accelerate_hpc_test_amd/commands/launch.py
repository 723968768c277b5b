"""`accelerate-amd launch`: start a training script on one MI355X node (or several) with the config contract.

Parity target: `/root/reference/src/accelerate/commands/launch.py:141-1409` — the same flag names are accepted
(so `accelerate launch ...` command lines and config files carry over), config-file values fill every flag that
was not given on the command line, and the launcher is chosen from the resulting distributed type.

MI355X-first design: there are exactly two launchers.
  * `simple_launcher` — one process (`python script.py ...` as a child process).
  * `multi_gpu_launcher` — `torch.distributed.run` (in-process elastic agent), one rank per GPU over RCCL.
DeepSpeed requests are translated to the native FSDP2/DDP engines (see utils/launch.py); Megatron-LM, TPU and
SageMaker requests are rejected with a pointer to the native equivalent.
"""

from __future__ import annotations

import argparse
import logging
import os
import sys

from ..utils.dataclasses import ComputeEnvironment, DistributedType
from ..utils.launch import (
    build_torchrun_cmd,
    prepare_multi_gpu_env,
    prepare_simple_launcher_cmd_env,
    run_child,
    torchrun_namespace,
)
from .config.config_args import default_config_file, load_config_from_file
from .utils import add_bool

logger = logging.getLogger(__name__)

description = "Launch a python script in a distributed scenario. Arguments can be passed in with either hyphens (`--num-processes=2`) or underscores (`--num_processes=2`)"

_MEGATRON_FLAGS = [
    "tp_degree", "pp_degree", "num_micro_batches", "sequence_parallelism", "recompute_activations",
    "use_distributed_optimizer", "gradient_clipping", "context_parallel_size", "expert_model_parallel_size",
    "expert_tensor_parallel_size", "decoder_last_pipeline_num_layers", "recompute_granularity",
    "recompute_method", "recompute_num_layers", "attention_backend", "calculate_per_token_loss",
    "use_rotary_position_embeddings", "use_custom_fsdp", "hidden_dropout", "attention_dropout",
    "attention_softmax_in_fp32", "eod_mask_loss", "no_load_optim", "no_save_optim", "optimizer_cpu_offload",
    "overlap_cpu_optimizer_d2h_h2d", "use_precision_aware_optimizer",
]


class _DualDashParser(argparse.ArgumentParser):
    """Accepts `--num-processes` as well as `--num_processes` for every long option."""

    def parse_known_args(self, args=None, namespace=None):
        args = list(sys.argv[1:] if args is None else args)
        fixed, i = [], 0
        while i < len(args):
            a = args[i]
            if not a.startswith("-"):
                fixed.extend(args[i:])  # the training script: everything from here on belongs to it
                break
            if a.startswith("--"):
                name, eq, val = a[2:].partition("=")
                a = "--" + name.replace("-", "_") + eq + val
                if "--" + name.replace("-", "_") not in self._option_string_actions:
                    a = args[i]
                opt = a.split("=", 1)[0]
            else:
                opt, eq = a, ""
            fixed.append(a)
            i += 1
            act = self._option_string_actions.get(opt)
            if act is None or eq or act.nargs == 0:
                continue
            if act.nargs == "?":  # optional boolean value
                if i < len(args) and args[i].lower() in ("true", "false", "yes", "no", "1", "0", "t", "f", "y", "n"):
                    fixed.append(args[i])
                    i += 1
                continue
            if i < len(args):
                fixed.append(args[i])
                i += 1
        return super().parse_known_args(fixed, namespace)


def launch_command_parser(subparsers=None):
    common = dict(description=description, add_help=False, allow_abbrev=False)
    if subparsers is not None:
        parser = subparsers.add_parser("launch", **common)
        parser.__class__ = _DualDashParser
    else:
        parser = _DualDashParser("accelerate-amd launch", **common)
    parser.add_argument("-h", "--help", action="help", help="Show this help message and exit.")
    parser.add_argument("--config_file", default=None, help="Config file to use for default values in the launching script.")
    parser.add_argument("--quiet", "-q", action="store_true", help="Silence subprocess errors from the launch stack trace.")

    hw = parser.add_argument_group("Hardware Selection Arguments")
    hw.add_argument("--cpu", default=False, action="store_true", help="Force training on the CPU.")
    hw.add_argument("--multi_gpu", default=False, action="store_true", help="Launch distributed GPU training (one rank per GPU, RCCL).")
    hw.add_argument("--tpu", default=False, action="store_true", help="Not supported on MI355X.")

    rs = parser.add_argument_group("Resource Selection Arguments")
    rs.add_argument("--dynamo_backend", type=str, choices=["no", "eager", "aot_eager", "inductor", "aot_ts_nvfuser", "nvprims_nvfuser", "cudagraphs", "ofi", "fx2trt", "onnxrt", "tensorrt", "aot_torchxla_trace_once", "torhchxla_trace_once", "ipex", "tvm", "hpu_backend"], help="Dynamo backend (torch.compile).")
    rs.add_argument("--dynamo_mode", type=str, default="default", choices=["default", "reduce-overhead", "max-autotune"])
    add_bool(rs, "--dynamo_use_fullgraph", "Use full-graph mode for torch.compile.", default=False)
    add_bool(rs, "--dynamo_use_dynamic", "Enable dynamic shape tracing.", default=False)
    add_bool(rs, "--dynamo_use_regional_compilation", "Compile repeated blocks once.", default=False)
    rs.add_argument("--mixed_precision", type=str, choices=["no", "fp16", "bf16", "fp8"], help="Mixed precision mode.")
    rs.add_argument("--num_processes", type=int, default=None, help="Total number of processes (GPUs) to launch.")
    rs.add_argument("--num_machines", type=int, default=None, help="Total number of machines.")
    rs.add_argument("--num_cpu_threads_per_process", type=int, default=None, help="OMP threads per rank.")
    add_bool(rs, "--enable_cpu_affinity", "Pin each rank to its GPU's NUMA node.", default=False)

    para = parser.add_argument_group("Training Paradigm Arguments")
    para.add_argument("--use_deepspeed", default=False, action="store_true", help="DeepSpeed ZeRO semantics (run by the native FSDP2/DDP engines).")
    para.add_argument("--use_fsdp", default=False, action="store_true", help="Native FSDP2 engine.")
    para.add_argument("--use_parallelism_config", default=False, action="store_true", help="N-d parallelism (dp_replicate x dp_shard x tp x cp x sp).")
    para.add_argument("--use_megatron_lm", default=False, action="store_true", help="Not available; use --use_parallelism_config.")

    dist = parser.add_argument_group("Distributed GPUs")
    dist.add_argument("--gpu_ids", default=None, help="Comma-separated GPU ids (HIP_VISIBLE_DEVICES) or 'all'.")
    dist.add_argument("--same_network", default=False, action="store_true")
    dist.add_argument("--machine_rank", type=int, default=None, help="Rank of this machine.")
    dist.add_argument("--main_process_ip", type=str, default=None, help="Address of the rank-0 machine.")
    dist.add_argument("--main_process_port", type=int, default=None, help="Port of the rank-0 machine.")
    dist.add_argument("-t", "--tee", default="0", type=str, help="Tee std streams into a log file and the console.")
    dist.add_argument("--log_dir", type=str, default=None, help="torchrun log directory.")
    dist.add_argument("--role", type=str, default="default", help="User-defined role for the workers.")
    dist.add_argument("--rdzv_backend", type=str, default=None, help="Rendezvous backend ('static' or 'c10d').")
    dist.add_argument("--rdzv_conf", type=str, default="", help="Additional rendezvous configuration (<key1>=<value1>,...).")
    dist.add_argument("--max_restarts", type=int, default=0, help="Maximum worker group restarts before failing.")
    dist.add_argument("--monitor_interval", type=float, default=0.1, help="Seconds between worker-state polls.")

    parser.add_argument("-m", "--module", action="store_true", help="Run the training script as a python module.")
    parser.add_argument("--no_python", action="store_true", help="Run the training script directly (not via python).")

    tpu = parser.add_argument_group("TPU (accepted for compatibility; rejected at launch)")
    tpu.add_argument("--tpu_cluster", action="store_true", dest="tpu_use_cluster")
    tpu.add_argument("--no_tpu_cluster", action="store_false", dest="tpu_use_cluster")
    tpu.add_argument("--tpu_use_sudo", action="store_true")
    tpu.add_argument("--vm", type=str, action="append")
    tpu.add_argument("--env", type=str, action="append")
    tpu.add_argument("--main_training_function", type=str, default=None)
    tpu.add_argument("--downcast_bf16", action="store_true", help="Downcast fp32 to bf16 (XLA compatibility flag).")

    ds = parser.add_argument_group("DeepSpeed Arguments (translated to native FSDP2/DDP)")
    ds.add_argument("--deepspeed_config_file", default=None, type=str)
    ds.add_argument("--zero_stage", default=None, type=int)
    ds.add_argument("--offload_optimizer_device", default=None, type=str)
    ds.add_argument("--offload_param_device", default=None, type=str)
    ds.add_argument("--offload_optimizer_nvme_path", default=None, type=str)
    ds.add_argument("--offload_param_nvme_path", default=None, type=str)
    ds.add_argument("--gradient_accumulation_steps", default=None, type=int)
    ds.add_argument("--gradient_clipping", default=None, type=float)
    ds.add_argument("--zero3_init_flag", default=None, type=str)
    ds.add_argument("--zero3_save_16bit_model", default=None, type=str)
    ds.add_argument("--deepspeed_hostfile", default=None, type=str)
    ds.add_argument("--deepspeed_exclusion_filter", default=None, type=str)
    ds.add_argument("--deepspeed_inclusion_filter", default=None, type=str)
    ds.add_argument("--deepspeed_multinode_launcher", default=None, type=str)
    ds.add_argument("--deepspeed_moe_layer_cls_names", default=None, type=str)

    fsdp = parser.add_argument_group("FSDP Arguments")
    fsdp.add_argument("--fsdp_version", type=str, default="1", choices=["1", "2"], help="FSDP version (1 maps onto the FSDP2 engine).")
    add_bool(fsdp, "--fsdp_offload_params", "Offload parameters and gradients to CPU.", default=False)
    fsdp.add_argument("--fsdp_min_num_params", type=int, default=int(1e8))
    fsdp.add_argument("--fsdp_sharding_strategy", type=str, default="FULL_SHARD")
    fsdp.add_argument("--fsdp_reshard_after_forward", type=str, default="true")
    fsdp.add_argument("--fsdp_auto_wrap_policy", type=str, default=None)
    fsdp.add_argument("--fsdp_transformer_layer_cls_to_wrap", default=None, type=str)
    fsdp.add_argument("--fsdp_backward_prefetch", default=None, type=str)
    fsdp.add_argument("--fsdp_state_dict_type", default=None, type=str)
    add_bool(fsdp, "--fsdp_forward_prefetch", "Explicitly prefetch the next all-gather in forward.", default=False)
    add_bool(fsdp, "--fsdp_use_orig_params", "Keep original parameters visible (always true here).", default=True)
    add_bool(fsdp, "--fsdp_cpu_ram_efficient_loading", "Load weights on rank 0 only and broadcast.", default=True)
    add_bool(fsdp, "--fsdp_sync_module_states", "Broadcast module states from rank 0.", default=True)
    add_bool(fsdp, "--fsdp_activation_checkpointing", "Recompute wrapped blocks in backward.", default=False)

    pc = parser.add_argument_group("Parallelism Config Arguments")
    pc.add_argument("--parallelism_config_dp_replicate_size", type=int, default=1)
    pc.add_argument("--parallelism_config_dp_shard_size", type=int, default=1)
    pc.add_argument("--parallelism_config_tp_size", type=int, default=1)
    pc.add_argument("--parallelism_config_cp_size", type=int, default=1)
    pc.add_argument("--parallelism_config_cp_backend", type=str, choices=["torch"], default="torch")
    pc.add_argument("--parallelism_config_cp_comm_strategy", type=str, choices=["allgather", "alltoall"], default="allgather")
    pc.add_argument("--parallelism_config_sp_size", type=int, default=1)
    pc.add_argument("--parallelism_config_sp_backend", type=str, choices=["deepspeed"], default="deepspeed")
    pc.add_argument("--parallelism_config_sp_seq_length", type=str, default=None)
    pc.add_argument("--parallelism_config_sp_seq_length_is_variable", type=bool, default=True)
    pc.add_argument("--parallelism_config_sp_attn_implementation", type=str, default="sdpa")

    mg = parser.add_argument_group("Megatron-LM Arguments (accepted; rejected at launch)")
    for name in _MEGATRON_FLAGS:
        mg.add_argument(f"--megatron_lm_{name}", default=None, type=str)

    fp8 = parser.add_argument_group("FP8 Arguments")
    fp8.add_argument("--fp8_backend", type=str, default="te", choices=["te", "msamp", "ao", "native"], help="fp8 backend; all run the native MX-MFMA fp8 path on MI355X.")
    fp8.add_argument("--fp8_use_autocast_during_eval", default=False, action="store_true")
    fp8.add_argument("--fp8_margin", type=int, default=0)
    fp8.add_argument("--fp8_interval", type=int, default=1)
    fp8.add_argument("--fp8_format", type=str, default="HYBRID", choices=["HYBRID", "E4M3", "E5M2"])
    fp8.add_argument("--fp8_amax_history_len", type=int, default=1024)
    fp8.add_argument("--fp8_amax_compute_algo", type=str, default="most_recent", choices=["max", "most_recent"])
    fp8.add_argument("--fp8_override_linear_precision", type=lambda x: tuple(map(lambda s: s.strip().lower() == "true", x.split(","))), default=(False, False, False))
    fp8.add_argument("--fp8_opt_level", type=str, default="O2", choices=["O1", "O2"])
    add_bool(fp8, "--fp8_enable_fsdp_float8_all_gather", "All-gather fp8 weights under FSDP.", default=True)
    add_bool(fp8, "--fp8_pad_inner_dim", "Pad inner dims to multiples of 16.", default=True)

    rc = parser.add_argument_group("RCCL / MI355X Arguments")
    rc.add_argument("--rccl_ddp_bucket_mb", type=int, default=None, help="DDP all-reduce bucket size (MB).")
    rc.add_argument("--rccl_fsdp_prefetch", type=int, default=None, help="FSDP all-gather prefetch depth.")
    rc.add_argument("--rccl_stream_priority", type=int, default=None, help="HIP priority of the comm streams.")
    rc.add_argument("--dry_run", action="store_true", help="Print the resolved command and env delta instead of running.")
    parser.add_argument("--debug", action="store_true",
                        help="Debug mode: every collective verifies that all ranks pass matching shapes "
                             "(ACCELERATE_DEBUG_MODE, utils/operations.verify_operation) and failures print the "
                             "torch.distributed stack trace.")
    mpi = parser.add_argument_group("MPI Arguments", "Multi-CPU launches through mpirun / mpiexec")
    mpi.add_argument("--mpirun_hostfile", type=str, default=None,
                     help="Hostfile for a multi-CPU launch with mpirun (passed as --hostfile / -f).")
    mpi.add_argument("--bind_to", type=str, default=None, help="Open MPI --bind-to value (default: socket).")

    parser.add_argument("training_script", type=str, help="The script (or module with -m) to launch.")
    parser.add_argument("training_script_args", nargs=argparse.REMAINDER, help="Arguments of the training script.")

    if subparsers is not None:
        parser.set_defaults(func=launch_command)
    return parser


# ------------------------------------------------------------------------------------------------------------
# config-file merge + validation
# ------------------------------------------------------------------------------------------------------------

_MULTI_TYPES = (DistributedType.MULTI_GPU, DistributedType.FSDP, DistributedType.DEEPSPEED)
_SECTION_PREFIX = {"fsdp_config": "", "fp8_config": "fp8_", "dynamo_config": "", "rccl_config": "rccl_"}


def _merge_config_defaults(args, parser_defaults: dict):
    """Fill every argument still at its parser default from the config file (CLI wins)."""
    use_file = args.config_file is not None or (os.path.isfile(default_config_file) and not args.cpu)
    if not use_file:
        return None
    cfg = load_config_from_file(args.config_file)
    if cfg.compute_environment != ComputeEnvironment.LOCAL_MACHINE:
        raise NotImplementedError("Only LOCAL_MACHINE configs can be launched from an MI355X node.")
    explicit_paradigm = any(getattr(args, k) for k in ("multi_gpu", "tpu", "use_deepspeed", "use_fsdp", "use_megatron_lm", "cpu"))
    dt = cfg.distributed_type
    if not explicit_paradigm:
        args.multi_gpu = dt in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU)
        args.use_fsdp = dt == DistributedType.FSDP
        args.use_deepspeed = dt == DistributedType.DEEPSPEED
        args.use_megatron_lm = dt == DistributedType.MEGATRON_LM
        args.tpu = dt == DistributedType.XLA
        args.use_parallelism_config = bool(cfg.parallelism_config)
    if args.gpu_ids is None:
        args.gpu_ids = cfg.gpu_ids if cfg.gpu_ids is not None else "all"

    def fill(name, value):
        if not hasattr(args, name):
            return
        if getattr(args, name) is None or getattr(args, name) == parser_defaults.get(name):
            setattr(args, name, value)

    for key, value in vars(cfg).items():
        if isinstance(value, dict):
            prefix = _SECTION_PREFIX.get(key, "")
            for sub, subval in value.items():
                name = sub if sub.startswith(prefix) else prefix + sub
                fill(name, subval)
        elif key not in ("compute_environment", "distributed_type", "gpu_ids"):
            fill(key, value)
    if cfg.mixed_precision and args.mixed_precision is None:
        args.mixed_precision = cfg.mixed_precision
    if cfg.use_cpu:
        args.cpu = True
    return cfg


def _validate_launch_command(args):
    if sum(bool(x) for x in (args.multi_gpu, args.cpu, args.tpu, args.use_deepspeed, args.use_fsdp)) > 1:
        raise ValueError("You can only use one of `--cpu`, `--multi_gpu`, `--tpu`, `--use_deepspeed`, `--use_fsdp` at a time.")
    if args.multi_gpu and args.num_processes is not None and args.num_processes < 2:
        raise ValueError("You need to use at least 2 processes to use `--multi_gpu`.")
    parser_defaults = vars(launch_command_parser().parse_args(["x"]))
    cfg = _merge_config_defaults(args, parser_defaults)
    if args.use_parallelism_config and (not args.use_fsdp or str(args.fsdp_version) == "1") and cfg is None:
        raise ValueError("You cannot use `--use_parallelism_config` without `--use_fsdp` and `--fsdp_version=2`.")
    if args.tpu or getattr(args, "tpu_use_cluster", False):
        raise NotImplementedError("TPU launches are not supported by the MI355X framework.")
    if args.gpu_ids is None:
        args.gpu_ids = "all"
    if args.num_machines is None:
        args.num_machines = 1
    if args.machine_rank is None:
        args.machine_rank = 0
    if args.num_processes is None:
        import torch

        n = torch.cuda.device_count() if not args.cpu else 1
        if args.gpu_ids != "all":
            n = len(args.gpu_ids.split(","))
        args.num_processes = max(n, 1) * args.num_machines if (args.multi_gpu or args.use_fsdp or args.use_deepspeed) else 1
        if (args.multi_gpu or args.use_fsdp or args.use_deepspeed) and args.num_processes < 2:
            args.num_processes = max(args.num_processes, 1)
    if args.mixed_precision is None:
        args.mixed_precision = "no"
    if args.dynamo_backend is None:
        args.dynamo_backend = "no"
    if args.num_cpu_threads_per_process is None:
        args.num_cpu_threads_per_process = 1
        if args.num_processes > 1:
            total = os.cpu_count() or 1
            local = max(args.num_processes // max(args.num_machines, 1), 1)
            args.num_cpu_threads_per_process = max(total // local, 1)
    return args


def simple_launcher(args) -> int:
    cmd, env = prepare_simple_launcher_cmd_env(args)
    if args.dry_run:
        _print_dry_run(cmd, env)
        return 0
    rc = run_child(cmd, env)
    if rc != 0 and not args.quiet:
        raise SystemExit(rc)
    return rc


def multi_gpu_launcher(args) -> int:
    env = prepare_multi_gpu_env(args)
    if args.dry_run:
        _print_dry_run(build_torchrun_cmd(args), env)
        return 0
    from torch.distributed import run as distrib_run
    from torch.distributed.elastic.multiprocessing.errors import ChildFailedError

    ns = torchrun_namespace(args)
    saved = os.environ.copy()
    os.environ.clear()
    os.environ.update(env)
    try:
        distrib_run.run(ns)
    except ChildFailedError:
        if args.quiet:
            raise SystemExit(1)
        raise
    finally:
        os.environ.clear()
        os.environ.update(saved)
    return 0


def _print_dry_run(cmd, env):
    delta = {k: v for k, v in env.items() if os.environ.get(k) != v}
    print(" ".join(cmd))
    for k in sorted(delta):
        print(f"{k}={delta[k]}")


def launch_command(args) -> int:
    args = _validate_launch_command(args)
    if args.use_megatron_lm:
        raise NotImplementedError("Megatron-LM is not available on this stack; use `--use_parallelism_config`.")
    distributed = args.multi_gpu or args.use_fsdp or args.use_deepspeed or args.num_processes > 1 or args.num_machines > 1
    if args.cpu and args.num_processes <= 1:
        distributed = False
    if args.mpirun_hostfile is not None:  # multi-CPU over MPI: mpirun starts the ranks (reference launch.py)
        if not args.cpu:
            raise ValueError("--mpirun_hostfile launches multi-CPU jobs: add --cpu (GPU jobs launch one rank per "
                             "MI355X through torch.distributed.run)")
        return simple_launcher(args)
    if distributed:
        return multi_gpu_launcher(args)
    return simple_launcher(args)


def main():
    parser = launch_command_parser()
    args = parser.parse_args()
    launch_command(args)


if __name__ == "__main__":
    main()
