"""Interactive questionnaire for `accelerate-amd config` on an MI355X node.

Parity target: `/root/reference/src/accelerate/commands/config/cluster.py:60-924` (`get_cluster_input`). The
reference walks every vendor back-end; here the questions are the ones that matter on ROCm: number of machines /
GPUs, DDP vs FSDP2 vs N-d parallelism, FSDP wrap/sharding/state-dict options, mixed precision (incl. native fp8
MX-MFMA), torch.compile, CPU affinity and the RCCL bucket/prefetch knobs. The answers produce the same
`ClusterConfig` fields the reference writes.

Questions are plain line prompts (`_Prompter`) so they also work over non-tty ssh sessions and in tests, where
answers are fed from a list.
"""

from __future__ import annotations

from typing import Callable, Optional

from ...utils.dataclasses import ComputeEnvironment, DistributedType
from ...utils.constants import FSDP_AUTO_WRAP_POLICY, FSDP_SHARDING_STRATEGY, FSDP_STATE_DICT_TYPE
from .config_args import ClusterConfig


class _Prompter:
    """Asks typed questions; `answers` (for tests / scripting) replaces stdin."""

    def __init__(self, answers: Optional[list] = None):
        self._answers = list(answers) if answers is not None else None

    def _raw(self, prompt: str) -> str:
        if self._answers is not None:
            return str(self._answers.pop(0)) if self._answers else ""
        return input(prompt)

    def ask(self, prompt: str, convert: Callable = str, default=None, error: str = "Please enter a valid value."):
        while True:
            text = self._raw(f"{prompt} ").strip()
            if not text and default is not None:
                return default
            try:
                return convert(text)
            except (ValueError, TypeError):
                print(error)
                if self._answers is not None and not self._answers:
                    raise

    def yes_no(self, prompt: str, default: bool = False) -> bool:
        def conv(t):
            t = t.lower()
            if t in ("y", "yes", "true", "1"):
                return True
            if t in ("n", "no", "false", "0"):
                return False
            raise ValueError(t)

        return self.ask(f"{prompt} [yes/NO]:" if not default else f"{prompt} [YES/no]:", conv, default)

    def choose(self, prompt: str, options: list, default: int = 0):
        print(prompt)
        for i, opt in enumerate(options):
            print(f"  [{i}] {opt}")

        def conv(t):
            if t in options:
                return t
            i = int(t)
            if not 0 <= i < len(options):
                raise ValueError(t)
            return options[i]

        return self.ask(f"Choice (default {options[default]}):", conv, options[default])


def get_cluster_input(answers: Optional[list] = None) -> ClusterConfig:
    p = _Prompter(answers)
    machine = p.choose("In which compute environment are you running?", ["This machine"])
    assert machine == "This machine"
    num_machines = p.ask("How many machines (nodes) will you use?", int, 1)
    machine_rank, main_ip, main_port, rdzv, same_network = 0, None, None, "static", True
    if num_machines > 1:
        machine_rank = p.ask("What is the rank of this machine?", int, 0)
        main_ip = p.ask("What is the IP address of the machine that will host the main process?", str)
        main_port = p.ask("What is the port you will use to communicate with the main process?", int, 29500)
        same_network = p.yes_no("Are all the machines on the same local network?", True)
        if not same_network:
            rdzv = p.ask("What rendezvous backend will you use? ('static', 'c10d', ...):", str, "static")
    paradigm = p.choose(
        "Which type of training will you use?",
        ["No distributed training", "multi-CPU", "multi-GPU DDP (RCCL)", "FSDP2 (RCCL)", "N-d parallelism (FSDP2 + TP/CP/SP)"],
        default=3,
    )
    use_cpu = paradigm == "multi-CPU"
    distributed_type = {
        "No distributed training": DistributedType.NO,
        "multi-CPU": DistributedType.MULTI_CPU,
        "multi-GPU DDP (RCCL)": DistributedType.MULTI_GPU,
        "FSDP2 (RCCL)": DistributedType.FSDP,
        "N-d parallelism (FSDP2 + TP/CP/SP)": DistributedType.FSDP,
    }[paradigm]
    debug = False
    if distributed_type != DistributedType.NO:
        debug = p.yes_no("Should distributed operations be checked while running for errors (debug mode)?", False)

    dynamo_config = {}
    if p.yes_no("Do you wish to optimize your script with torch.compile?", False):
        dynamo_config["dynamo_backend"] = p.choose("Which backend?", ["INDUCTOR", "EAGER", "AOT_EAGER", "CUDAGRAPHS"]).upper()
        dynamo_config["dynamo_mode"] = p.choose("Which mode?", ["default", "reduce-overhead", "max-autotune"])
        dynamo_config["dynamo_use_fullgraph"] = p.yes_no("Use full-graph mode?", False)
        dynamo_config["dynamo_use_dynamic"] = p.yes_no("Enable dynamic shapes?", False)
        dynamo_config["dynamo_use_regional_compilation"] = p.yes_no("Compile repeated blocks once (regional compilation)?", False)

    fsdp_config, parallelism_config = {}, {}
    if distributed_type == DistributedType.FSDP:
        fsdp_config["fsdp_version"] = 2
        fsdp_config["fsdp_reshard_after_forward"] = p.yes_no("Reshard parameters after forward (ZeRO-3; NO = ZeRO-2)?", True)
        fsdp_config["fsdp_offload_params"] = p.yes_no("Offload parameters and gradients to CPU?", False)
        fsdp_config["fsdp_auto_wrap_policy"] = p.choose("What should be your auto wrap policy?", list(FSDP_AUTO_WRAP_POLICY))
        if fsdp_config["fsdp_auto_wrap_policy"] == "TRANSFORMER_BASED_WRAP":
            names = p.ask("Transformer layer class names to wrap (comma separated, empty = model._no_split_modules):", str, "")
            if names:
                fsdp_config["fsdp_transformer_layer_cls_to_wrap"] = names
        elif fsdp_config["fsdp_auto_wrap_policy"] == "SIZE_BASED_WRAP":
            fsdp_config["fsdp_min_num_params"] = p.ask("Minimum number of parameters per unit:", int, 100000000)
        fsdp_config["fsdp_state_dict_type"] = p.choose("What should be your FSDP's state dict type?", list(FSDP_STATE_DICT_TYPE), default=2)
        fsdp_config["fsdp_cpu_ram_efficient_loading"] = p.yes_no("Materialise weights on rank 0 only and broadcast?", True)
        fsdp_config["fsdp_activation_checkpointing"] = p.yes_no("Use activation checkpointing?", False)
        if paradigm.startswith("N-d"):
            for dim in ("dp_replicate_size", "dp_shard_size", "tp_size", "cp_size", "sp_size"):
                parallelism_config[f"parallelism_config_{dim}"] = p.ask(f"{dim}:", int, 1)

    num_processes = 1
    if distributed_type in (DistributedType.MULTI_GPU, DistributedType.FSDP, DistributedType.MULTI_CPU):
        unit = "CPU processes" if use_cpu else "GPUs"
        num_processes = p.ask(f"How many {unit} should be used for distributed training (total over all machines)?", int, 8 * num_machines)
    gpu_ids = None
    if distributed_type in (DistributedType.MULTI_GPU, DistributedType.FSDP, DistributedType.NO) and not use_cpu:
        gpu_ids = p.ask("Which GPU ids (by id) should be used on this machine, as a comma-separated list?", str, "all")
    enable_cpu_affinity = False
    if not use_cpu:
        enable_cpu_affinity = p.yes_no("Pin each rank to the NUMA node of its GPU?", True)

    rccl_config = {}
    if distributed_type == DistributedType.MULTI_GPU:
        mb = p.ask("DDP all-reduce bucket size in MB (xGMI ring sweet spot ~128):", int, 128)
        if mb != 128:
            rccl_config["rccl_ddp_bucket_mb"] = mb

    mixed_precision = p.choose("Do you wish to use mixed precision?", ["no", "bf16", "fp16", "fp8"], default=1)
    fp8_config = {}
    if mixed_precision == "fp8":
        fp8_config["backend"] = "NATIVE"
        fp8_config["fp8_format"] = p.choose("Which fp8 format?", ["HYBRID", "E4M3", "E5M2"])
        fp8_config["amax_history_len"] = p.ask("amax history length:", int, 16)
        fp8_config["amax_compute_algo"] = p.choose("amax compute algorithm?", ["max", "most_recent"])

    return ClusterConfig(
        compute_environment=ComputeEnvironment.LOCAL_MACHINE,
        distributed_type=distributed_type,
        mixed_precision=mixed_precision,
        use_cpu=use_cpu,
        debug=debug,
        num_processes=num_processes,
        machine_rank=machine_rank,
        num_machines=num_machines,
        gpu_ids=gpu_ids,
        main_process_ip=main_ip,
        main_process_port=main_port,
        rdzv_backend=rdzv,
        same_network=same_network,
        enable_cpu_affinity=enable_cpu_affinity,
        fsdp_config=fsdp_config,
        parallelism_config=parallelism_config,
        fp8_config=fp8_config,
        dynamo_config=dynamo_config,
        rccl_config=rccl_config,
    )
