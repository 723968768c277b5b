"""Configuration dataclasses, enums and kwargs handlers.

Parity: `/root/reference/src/accelerate/utils/dataclasses.py:68-3196`. Field names, defaults, env-var
names and the "constructor > env > default" resolution order are kept so YAML configs, `accelerate launch`
flags and user code written for the reference keep working. What the fields *drive* is different:
the FSDP plugin configures our own flat-shard engine (`parallel/fsdp.py`) instead of
`torch.distributed.fsdp`, the fp8 recipes route to our HIP kernels (`ops/fp8.py`), and DeepSpeed /
Megatron plugins are accepted for API compatibility but map onto native capabilities or raise.
"""

from __future__ import annotations

import copy
import enum
import functools
import os
import warnings
from dataclasses import dataclass, field, fields
from datetime import timedelta
from typing import Any, Callable, Iterable, Literal, Optional, Union

import torch

from .constants import (
    DEFAULT_DDP_BUCKET_MB,
    FSDP2_STATE_DICT_TYPE,
    FSDP_AUTO_WRAP_POLICY,
    FSDP_BACKWARD_PREFETCH,
    FSDP_SHARDING_STRATEGY,
    FSDP_STATE_DICT_TYPE,
)
from .environment import parse_flag_from_env, str_to_bool


# ---------------------------------------------------------------------------------------------------
# Kwargs handlers
# ---------------------------------------------------------------------------------------------------
class KwargsHandler:
    """Base for dataclasses whose non-default fields are forwarded as keyword arguments."""

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_kwargs(self):
        """Only the fields that differ from the defaults (reference `dataclasses.py:76-86`)."""
        default_dict = self.__class__().to_dict()
        this_dict = self.to_dict()
        return {k: v for k, v in this_dict.items() if default_dict[k] != v}


class EnumWithContains(enum.EnumMeta):
    def __contains__(cls, item):
        try:
            cls(item)
        except ValueError:
            return False
        return True


class BaseEnum(enum.Enum, metaclass=EnumWithContains):
    def __str__(self):
        return self.value

    @classmethod
    def list(cls):
        return [str(x) for x in list(cls)]


@dataclass
class AutocastKwargs(KwargsHandler):
    enabled: bool = True
    cache_enabled: bool = None


class DDPCommunicationHookType(BaseEnum):
    """Gradient compression applied inside our bucket pack kernel (see parallel/ddp.py)."""

    NO = "no"
    FP16 = "fp16"
    BF16 = "bf16"
    POWER_SGD = "power_sgd"
    BATCHED_POWER_SGD = "batched_power_sgd"


@dataclass
class DistributedDataParallelKwargs(KwargsHandler):
    """Options of our RCCL DDP reducer. Same names as torch DDP; `bucket_cap_mb` defaults to a larger
    value sized for 8-way xGMI (8 MB+ per peer per collective) instead of torch's 25 MB."""

    dim: int = 0
    broadcast_buffers: bool = True
    bucket_cap_mb: int = 25
    find_unused_parameters: bool = False
    check_reduction: bool = False
    gradient_as_bucket_view: bool = False
    static_graph: bool = False

    comm_hook: DDPCommunicationHookType = DDPCommunicationHookType.NO
    comm_wrapper: Literal[DDPCommunicationHookType.NO, DDPCommunicationHookType.FP16, DDPCommunicationHookType.BF16] = (
        DDPCommunicationHookType.NO
    )
    comm_state_option: dict = field(default_factory=dict)

    def to_dict(self, ignore_keys=("comm_hook", "comm_wrapper", "comm_state_option")):
        return {k: v for k, v in super().to_dict().items() if k not in ignore_keys}

    def effective_bucket_bytes(self) -> int:
        # A user-specified value wins; the torch default (25) is replaced by the xGMI-sized default.
        mb = self.bucket_cap_mb if self.bucket_cap_mb != 25 else DEFAULT_DDP_BUCKET_MB
        return int(mb * (1 << 20))

    def register_comm_hook(self, model):
        """Kept for API parity: our reducer reads `comm_hook`/`comm_wrapper` directly."""
        if hasattr(model, "set_comm_hook"):
            model.set_comm_hook(self.comm_hook, self.comm_wrapper, self.comm_state_option)


@dataclass
class GradScalerKwargs(KwargsHandler):
    init_scale: float = 65536.0
    growth_factor: float = 2.0
    backoff_factor: float = 0.5
    growth_interval: int = 2000
    enabled: bool = True


@dataclass
class InitProcessGroupKwargs(KwargsHandler):
    backend: Optional[str] = "nccl"
    init_method: Optional[str] = None
    timeout: Optional[timedelta] = None

    def __post_init__(self):
        if self.timeout is None:
            seconds = 1800 if self.backend != "nccl" else 600
            self.timeout = timedelta(seconds=seconds)


Backend = Literal["MSAMP", "TE", "AO", "NATIVE"]
OptLevel = Literal["O1", "O2"]
FP8Format = Literal["HYBRID", "E4M3", "E5M2"]
AmaxComputeAlgorithm = Literal["max", "most_recent"]


@dataclass
class Float8LinearConfig:
    """Minimal stand-in for torchao's config (torchao is not installed on the MI355X image).
    Only the knobs our fp8 path implements are kept."""

    enable_fsdp_float8_all_gather: bool = False
    pad_inner_dim: bool = True
    emulate: bool = False
    round_scales_to_power_of_2: bool = False


@dataclass
class AORecipeKwargs(KwargsHandler):
    """torchao-style dynamic per-tensor fp8 recipe, executed by our HIP kernels (ops/fp8.py).
    Parity: reference `dataclasses.py:310-355`."""

    config: Optional[Any] = None
    module_filter_func: Optional[Callable] = None
    pad_inner_dim: Optional[bool] = None
    enable_fsdp_float8_all_gather: Optional[bool] = None

    def __post_init__(self):
        env_prefix = "ACCELERATE_FP8_"
        if self.config is None:
            self.config = Float8LinearConfig()
        if self.pad_inner_dim is None:
            self.pad_inner_dim = parse_flag_from_env(env_prefix + "PAD_INNER_DIM", True)
        if self.enable_fsdp_float8_all_gather is None:
            self.enable_fsdp_float8_all_gather = parse_flag_from_env(env_prefix + "ENABLE_FSDP_FLOAT8_ALL_GATHER", True)
        if hasattr(self.config, "pad_inner_dim"):
            try:
                self.config.pad_inner_dim = self.pad_inner_dim
                self.config.enable_fsdp_float8_all_gather = self.enable_fsdp_float8_all_gather
            except Exception:
                pass


@dataclass
class TERecipeKwargs(KwargsHandler):
    """TransformerEngine-style delayed-scaling recipe, executed by our HIP kernels with an amax
    history ring buffer in HBM. Parity: reference `dataclasses.py:358-434`."""

    use_autocast_during_eval: bool = None
    margin: int = None
    interval: int = None
    fp8_format: FP8Format = None
    amax_history_len: int = None
    amax_compute_algo: AmaxComputeAlgorithm = None
    override_linear_precision: tuple[bool, bool, bool] = None
    use_mxfp8_block_scaling: bool = None

    def __post_init__(self):
        env_prefix = "ACCELERATE_FP8_"
        if self.use_autocast_during_eval is None:
            self.use_autocast_during_eval = parse_flag_from_env(env_prefix + "USE_AUTOCAST_DURING_EVAL")
        if self.margin is None:
            self.margin = int(os.environ.get(env_prefix + "MARGIN", 0))
        if self.interval is None:
            self.interval = int(os.environ.get(env_prefix + "INTERVAL", 1))
        if self.fp8_format is None:
            self.fp8_format = os.environ.get(env_prefix + "FORMAT", "HYBRID")
        self.fp8_format = self.fp8_format.upper()
        if self.fp8_format not in ("HYBRID", "E4M3", "E5M2"):
            raise ValueError(f"`fp8_format` must be one of HYBRID, E4M3, E5M2, got {self.fp8_format}")
        if self.amax_compute_algo is None:
            self.amax_compute_algo = os.environ.get(env_prefix + "AMAX_COMPUTE_ALGO", "most_recent")
        if self.amax_history_len is None:
            self.amax_history_len = int(os.environ.get(env_prefix + "AMAX_HISTORY_LEN", 1024))
        if self.override_linear_precision is None:
            fprop = parse_flag_from_env(env_prefix + "OVERRIDE_FPROP")
            dgrad = parse_flag_from_env(env_prefix + "OVERRIDE_DGRAD")
            wgrad = parse_flag_from_env(env_prefix + "OVERRIDE_WGRAD")
            self.override_linear_precision = (fprop, dgrad, wgrad)
        if self.use_mxfp8_block_scaling is None:
            self.use_mxfp8_block_scaling = parse_flag_from_env(env_prefix + "USE_MXFP8_BLOCK_SCALING")


@dataclass
class MSAMPRecipeKwargs(KwargsHandler):
    """Accepted for API compatibility; MS-AMP is deprecated upstream and not supported here."""

    opt_level: OptLevel = None

    def __post_init__(self):
        raise NotImplementedError("MS-AMP is not supported on MI355X; use AORecipeKwargs or TERecipeKwargs.")


@dataclass
class FP8RecipeKwargs(TERecipeKwargs):
    """Deprecated alias of `TERecipeKwargs` (reference `dataclasses.py:454-476`)."""

    backend: Backend = None
    opt_level: OptLevel = None

    def __post_init__(self):
        warnings.warn("FP8RecipeKwargs is deprecated; use TERecipeKwargs or AORecipeKwargs.", FutureWarning)
        if self.backend is None:
            self.backend = os.environ.get("ACCELERATE_FP8_BACKEND", "TE")
        self.backend = self.backend.upper()
        super().__post_init__()


ProfilerActivity = Literal["cpu", "xpu", "mtia", "cuda", "hpu"]


@dataclass
class ProfileKwargs(KwargsHandler):
    """torch.profiler configuration. `cuda` activity is served by roctracer via kineto on ROCm.
    Parity: reference `dataclasses.py:483-597`."""

    activities: Optional[list[ProfilerActivity]] = None
    schedule_option: Optional[dict[str, int]] = None
    on_trace_ready: Optional[Callable] = None
    record_shapes: bool = False
    profile_memory: bool = False
    with_stack: bool = False
    with_flops: bool = False
    with_modules: bool = False
    output_trace_dir: Optional[str] = None

    def _get_profiler_activity(self, activity: ProfilerActivity):
        mapping = {"cpu": torch.profiler.ProfilerActivity.CPU, "cuda": torch.profiler.ProfilerActivity.CUDA}
        if activity not in mapping:
            raise ValueError(f"Invalid profiler activity: {activity}. Must be one of {list(mapping)}.")
        return mapping[activity]

    def build(self):
        activities = None
        if self.activities is not None:
            activities = [self._get_profiler_activity(a) for a in self.activities]
        schedule = None
        if self.schedule_option is not None:
            schedule = torch.profiler.schedule(**self.schedule_option)
        return torch.profiler.profile(
            activities=activities,
            schedule=schedule,
            on_trace_ready=self.on_trace_ready,
            record_shapes=self.record_shapes,
            profile_memory=self.profile_memory,
            with_stack=self.with_stack,
            with_flops=self.with_flops,
            with_modules=self.with_modules,
        )


@dataclass
class RcclKwargs(KwargsHandler):
    """MI355X-specific communication knobs (new; no reference equivalent).

    - `ddp_bucket_mb`: DDP gradient bucket size (default 128 MB → 16 MB per peer at 8 GPUs).
    - `fsdp_prefetch_depth`: how many FSDP units are all-gathered ahead of compute.
    - `comm_stream_priority`: HIP stream priority of the collective streams (-1 = high).
    - `watchdog_timeout`: seconds without a training-step heartbeat after which the rank dumps its stacks and exits
      (utils/fault_tolerance.py); `ACCELERATE_WATCHDOG_TIMEOUT`; None = off.
    - `collective_check_interval`: in debug mode, compare every rank's collective-sequence digest each N backward
      passes (`ACCELERATE_COLLECTIVE_CHECK_INTERVAL`, default 50).
    - `fsdp_optimizer_overlap`: run the optimizer update of each FSDP unit on a side HIP stream as soon as that unit's
      gradient shard is final, overlapped with the rest of the backward; `optimizer.step()` then only updates what is
      left and waits for the side stream (`ACCELERATE_FSDP_OPTIMIZER_OVERLAP`). Incompatible with gradient clipping
      (the norm needs every gradient before any update: `clip_grad_norm_` raises) and with fp16 loss scaling (not
      enabled then).
    - `fsdp_force_sharded`: at world size 1, run the FSDP engine's multi-GPU code anyway (separate full buffers, RCCL
      all-gather / reduce-scatter with nranks=1, bf16 flat gradient buffers) instead of the degenerate no-collective
      path; needs an initialised process group (`ACCELERATE_FSDP_FORCE_SHARDED`). Used to measure and test the sharded
      path on one GPU.
    - `ddp_force`: at world size 1 with an initialised process group, wrap the model in this framework's DDP reducer
      anyway (flat buckets, post-accumulate hooks, RCCL all-reduce with nranks=1 on the reducer's own communicator and
      side stream) instead of leaving it unwrapped (`ACCELERATE_DDP_FORCE`). Used to measure and test the DDP path on
      one GPU.
    """

    ddp_bucket_mb: int = None
    fsdp_prefetch_depth: int = None
    comm_stream_priority: int = None
    watchdog_timeout: float = None
    collective_check_interval: int = None
    fsdp_optimizer_overlap: bool = None
    fsdp_force_sharded: bool = None
    ddp_force: bool = None

    def __post_init__(self):
        if self.ddp_bucket_mb is None:
            self.ddp_bucket_mb = int(os.environ.get("ACCELERATE_RCCL_DDP_BUCKET_MB", DEFAULT_DDP_BUCKET_MB))
        if self.fsdp_prefetch_depth is None:
            self.fsdp_prefetch_depth = int(os.environ.get("ACCELERATE_RCCL_FSDP_PREFETCH", 1))
        if self.comm_stream_priority is None:
            self.comm_stream_priority = int(os.environ.get("ACCELERATE_RCCL_STREAM_PRIORITY", -1))
        if self.watchdog_timeout is None and os.environ.get("ACCELERATE_WATCHDOG_TIMEOUT"):
            self.watchdog_timeout = float(os.environ["ACCELERATE_WATCHDOG_TIMEOUT"])
        if self.collective_check_interval is None:
            self.collective_check_interval = int(os.environ.get("ACCELERATE_COLLECTIVE_CHECK_INTERVAL", 50))
        if self.fsdp_optimizer_overlap is None:
            self.fsdp_optimizer_overlap = parse_flag_from_env("ACCELERATE_FSDP_OPTIMIZER_OVERLAP", False)
        if self.fsdp_force_sharded is None:
            self.fsdp_force_sharded = parse_flag_from_env("ACCELERATE_FSDP_FORCE_SHARDED", False)
        if self.ddp_force is None:
            self.ddp_force = parse_flag_from_env("ACCELERATE_DDP_FORCE", False)


# ---------------------------------------------------------------------------------------------------
# Enums
# ---------------------------------------------------------------------------------------------------
class DistributedType(str, enum.Enum):
    """Only CPU and ROCm-GPU variants are executable here; the rest exist so configs parse."""

    NO = "NO"
    MULTI_CPU = "MULTI_CPU"
    MULTI_GPU = "MULTI_GPU"
    FSDP = "FSDP"
    DEEPSPEED = "DEEPSPEED"
    MEGATRON_LM = "MEGATRON_LM"
    MULTI_NPU = "MULTI_NPU"
    MULTI_MLU = "MULTI_MLU"
    MULTI_SDAA = "MULTI_SDAA"
    MULTI_MUSA = "MULTI_MUSA"
    MULTI_XPU = "MULTI_XPU"
    MULTI_HPU = "MULTI_HPU"
    XLA = "XLA"


class SageMakerDistributedType(str, enum.Enum):
    NO = "NO"
    DATA_PARALLEL = "DATA_PARALLEL"
    MODEL_PARALLEL = "MODEL_PARALLEL"


class FP8BackendType(str, enum.Enum):
    NO = "NO"
    TE = "TE"
    MSAMP = "MSAMP"
    AO = "AO"
    NATIVE = "NATIVE"


class ComputeEnvironment(str, enum.Enum):
    LOCAL_MACHINE = "LOCAL_MACHINE"
    AMAZON_SAGEMAKER = "AMAZON_SAGEMAKER"


class DynamoBackend(str, BaseEnum):
    NO = "NO"
    EAGER = "EAGER"
    AOT_EAGER = "AOT_EAGER"
    INDUCTOR = "INDUCTOR"
    AOT_TS_NVFUSER = "AOT_TS_NVFUSER"
    NVPRIMS_NVFUSER = "NVPRIMS_NVFUSER"
    CUDAGRAPHS = "CUDAGRAPHS"
    OFI = "OFI"
    FX2TRT = "FX2TRT"
    ONNXRT = "ONNXRT"
    TENSORRT = "TENSORRT"
    AOT_TORCHXLA_TRACE_ONCE = "AOT_TORCHXLA_TRACE_ONCE"
    TORCHXLA_TRACE_ONCE = "TORCHXLA_TRACE_ONCE"
    IPEX = "IPEX"
    TVM = "TVM"
    HPU_BACKEND = "HPU_BACKEND"


class LoggerType(BaseEnum):
    ALL = "all"
    AIM = "aim"
    TENSORBOARD = "tensorboard"
    WANDB = "wandb"
    TRACKIO = "trackio"
    COMETML = "comet_ml"
    MLFLOW = "mlflow"
    CLEARML = "clearml"
    DVCLIVE = "dvclive"
    SWANLAB = "swanlab"
    JSONL = "jsonl"


class PrecisionType(str, BaseEnum):
    NO = "no"
    FP8 = "fp8"
    FP16 = "fp16"
    BF16 = "bf16"


class RNGType(BaseEnum):
    TORCH = "torch"
    CUDA = "cuda"
    NPU = "npu"
    XLA = "xla"
    XPU = "xpu"
    HPU = "hpu"
    GENERATOR = "generator"


class CustomDtype(enum.Enum):
    FP8 = "fp8"
    INT4 = "int4"
    INT2 = "int2"


class TensorInformation:
    def __init__(self, shape: torch.Size, dtype: torch.dtype):
        self.shape = shape
        self.dtype = dtype

    def __repr__(self):
        return f"TensorInformation(shape={self.shape}, dtype={self.dtype})"


@dataclass
class DataLoaderConfiguration:
    """Parity: reference `dataclasses.py:813-905`. `prefetch_to_device` is an MI355X addition: depth of the
    pinned-ring / copy-stream prefetcher used by `DataLoaderShard` on GPU (0 disables it)."""

    split_batches: bool = False
    dispatch_batches: bool = None
    even_batches: bool = True
    use_seedable_sampler: bool = False
    data_seed: int = None
    non_blocking: bool = False
    use_stateful_dataloader: bool = False
    prefetch_to_device: int = 2


@dataclass
class ProjectConfiguration:
    """Parity: reference `dataclasses.py:908-968`."""

    project_dir: str = None
    logging_dir: str = None
    automatic_checkpoint_naming: bool = False
    total_limit: int = None
    iteration: int = 0
    save_on_each_node: bool = False

    def set_directories(self, project_dir: str = None):
        self.project_dir = project_dir
        if self.logging_dir is None:
            self.logging_dir = project_dir

    def __post_init__(self):
        self.set_directories(self.project_dir)


@dataclass
class GradientAccumulationPlugin(KwargsHandler):
    num_steps: int = None
    adjust_scheduler: bool = True
    sync_with_dataloader: bool = True
    sync_each_batch: bool = False


@dataclass
class TorchDynamoPlugin(KwargsHandler):
    """Kept for API parity; `torch.compile` is only invoked when the user asks for it and is never on the
    benchmarked path (our fusions are hand-written HIP kernels)."""

    backend: DynamoBackend = None
    mode: str = None
    fullgraph: bool = None
    dynamic: bool = None
    options: Any = None
    disable: bool = False
    use_regional_compilation: bool = None

    def __post_init__(self):
        prefix = "ACCELERATE_DYNAMO_"
        if self.backend is None:
            self.backend = os.environ.get(prefix + "BACKEND", "no")
        self.backend = DynamoBackend(str(self.backend).upper())
        if self.mode is None:
            self.mode = os.environ.get(prefix + "MODE", "default")
        if self.fullgraph is None:
            self.fullgraph = str_to_bool(os.environ.get(prefix + "USE_FULLGRAPH", "False")) == 1
        if self.use_regional_compilation is None:
            self.use_regional_compilation = str_to_bool(os.environ.get(prefix + "USE_REGIONAL_COMPILATION", "False")) == 1
        if self.dynamic is None and prefix + "USE_DYNAMIC" in os.environ:
            self.dynamic = str_to_bool(os.environ[prefix + "USE_DYNAMIC"]) == 1

    def to_dict(self):
        d = copy.deepcopy(self.__dict__)
        d["backend"] = d["backend"].value.lower()
        return d

    def to_kwargs(self):
        kwargs = super().to_kwargs()
        kwargs.pop("use_regional_compilation", None)
        return kwargs


@dataclass
class DeepSpeedPlugin:
    """API-compatible placeholder. ZeRO-3 maps onto our FSDP engine (full shard) and ZeRO-1/2 onto
    `reshard_after_forward=False`; the DeepSpeed runtime itself is not a dependency here.
    `to_fsdp_plugin()` performs that mapping."""

    hf_ds_config: Any = None
    gradient_accumulation_steps: int = None
    gradient_clipping: float = None
    zero_stage: int = None
    is_train_batch_min: bool = True
    offload_optimizer_device: str = None
    offload_param_device: str = None
    offload_optimizer_nvme_path: str = None
    offload_param_nvme_path: str = None
    zero3_init_flag: bool = None
    zero3_save_16bit_model: bool = None
    transformer_moe_cls_names: str = None
    enable_msamp: bool = None
    msamp_opt_level: Optional[Literal["O1", "O2"]] = None

    def __post_init__(self):
        prefix = "ACCELERATE_DEEPSPEED_"
        if self.zero_stage is None:
            self.zero_stage = int(os.environ.get(prefix + "ZERO_STAGE", 2))
        if self.gradient_accumulation_steps is None:
            ga = os.environ.get("ACCELERATE_GRADIENT_ACCUMULATION_STEPS", "1")
            self.gradient_accumulation_steps = int(ga) if ga != "auto" else 1
        if self.gradient_clipping is None:
            gc = os.environ.get("ACCELERATE_GRADIENT_CLIPPING", "none")
            self.gradient_clipping = float(gc) if gc not in ("none", "auto") else None
        self.deepspeed_config = {"zero_optimization": {"stage": self.zero_stage}}

    def to_fsdp_plugin(self) -> "FullyShardedDataParallelPlugin":
        return FullyShardedDataParallelPlugin(
            fsdp_version=2,
            reshard_after_forward=self.zero_stage >= 3,
            cpu_offload=self.offload_param_device == "cpu",
        )

    def set_mixed_precision(self, mixed_precision):
        self.deepspeed_config["bf16" if mixed_precision == "bf16" else "fp16"] = {"enabled": mixed_precision != "no"}

    def select(self, _from_accelerator_state: bool = False):
        self._selected = True


@dataclass
class MixedPrecisionPolicy:
    """Our FSDP engine's dtype policy (same field names as torch's FSDP2 `MixedPrecisionPolicy`).
    `param_dtype` is the all-gather/compute dtype, `reduce_dtype` the reduce-scatter dtype, master
    weights and optimizer state are always fp32 when `param_dtype` is lower precision."""

    param_dtype: Optional[torch.dtype] = None
    reduce_dtype: Optional[torch.dtype] = None
    output_dtype: Optional[torch.dtype] = None
    cast_forward_inputs: bool = True


@dataclass
class CPUOffloadPolicy:
    """Keep fp32 master shards + optimizer state in pinned host memory (moved in/out on a copy stream)."""

    pin_memory: bool = True


def _parse_ignored_modules(value):
    if value is None:
        return None
    return value


@dataclass
class FullyShardedDataParallelPlugin:
    """FSDP configuration for our native flat-shard engine (`parallel/fsdp.py`).

    Parity: reference `dataclasses.py:1565-2167`. FSDP1 flags are mapped onto the FSDP2 semantics (as the
    reference's `accelerate to-fsdp2` does, `commands/to_fsdp2.py:31-66`): FULL_SHARD → reshard_after_forward
    True, SHARD_GRAD_OP → False, NO_SHARD → DDP, HYBRID_SHARD → HSDP (replicate × shard mesh).
    """

    fsdp_version: int = None
    sharding_strategy: Union[str, int] = None
    reshard_after_forward: Union[str, bool] = None
    backward_prefetch: Optional[str] = None
    mixed_precision_policy: Optional[Union[dict, MixedPrecisionPolicy, str, torch.dtype]] = None
    auto_wrap_policy: Optional[Union[Callable, Literal["transformer_based_wrap", "size_based_wrap", "no_wrap"]]] = None
    cpu_offload: Union[bool, CPUOffloadPolicy] = None
    ignored_modules: Optional[Union[Iterable[torch.nn.Module], str]] = None
    state_dict_type: str = None
    state_dict_config: Optional[dict] = None
    optim_state_dict_config: Optional[dict] = None
    limit_all_gathers: bool = True
    use_orig_params: Optional[bool] = None
    param_init_fn: Optional[Callable[[torch.nn.Module], None]] = None
    sync_module_states: Optional[bool] = None
    forward_prefetch: bool = None
    activation_checkpointing: bool = None
    cpu_ram_efficient_loading: bool = None
    transformer_cls_names_to_wrap: Optional[list[str]] = None
    min_num_params: Optional[int] = None

    def __post_init__(self):
        env_prefix = "FSDP_"
        if self.fsdp_version is None:
            self.fsdp_version = int(os.environ.get(env_prefix + "VERSION", "1"))
        if self.fsdp_version not in (1, 2):
            raise ValueError(f"fsdp_version must be 1 or 2, got {self.fsdp_version}")

        # --- sharding strategy / reshard_after_forward (FSDP1 strings map to FSDP2 booleans) ---
        if self.sharding_strategy is None and self.fsdp_version == 1 and self.reshard_after_forward is None:
            self.sharding_strategy = os.environ.get(env_prefix + "SHARDING_STRATEGY", "FULL_SHARD")
        if self.sharding_strategy is not None:
            s = self.sharding_strategy
            if isinstance(s, int) or (isinstance(s, str) and s.isdigit()):
                s = FSDP_SHARDING_STRATEGY[int(s) - 1]
            s = getattr(s, "name", s)
            s = str(s).upper()
            if s not in FSDP_SHARDING_STRATEGY:
                raise ValueError(f"Unknown sharding strategy {s}; choose from {FSDP_SHARDING_STRATEGY}")
            self.sharding_strategy = s
        if self.reshard_after_forward is None:
            if self.sharding_strategy is not None:
                self.reshard_after_forward = self.sharding_strategy in ("FULL_SHARD", "HYBRID_SHARD")
            else:
                raf = os.environ.get(env_prefix + "RESHARD_AFTER_FORWARD", "true" if self.fsdp_version == 2 else "FULL_SHARD")
                self.reshard_after_forward = raf
        if isinstance(self.reshard_after_forward, str):
            raf = self.reshard_after_forward.upper()
            if raf in FSDP_SHARDING_STRATEGY or raf.isdigit():
                if raf.isdigit():
                    raf = FSDP_SHARDING_STRATEGY[int(raf) - 1]
                if self.sharding_strategy is None:
                    self.sharding_strategy = raf
                self.reshard_after_forward = raf in ("FULL_SHARD", "HYBRID_SHARD")
            else:
                self.reshard_after_forward = str_to_bool(raf.lower(), to_bool=True)
        if self.fsdp_version == 2 and not isinstance(self.reshard_after_forward, bool):
            raise ValueError(f"reshard_after_forward must be a bool with FSDP2, got {self.reshard_after_forward}")

        if self.cpu_offload is None:
            self.cpu_offload = str_to_bool(os.environ.get(env_prefix + "OFFLOAD_PARAMS", "False")) == 1
        if isinstance(self.cpu_offload, bool):
            self.cpu_offload = CPUOffloadPolicy() if self.cpu_offload else None

        if self.backward_prefetch is None:
            self.backward_prefetch = os.environ.get(env_prefix + "BACKWARD_PREFETCH", None)
        if isinstance(self.backward_prefetch, str):
            bp = self.backward_prefetch.upper()
            if bp == "NO_PREFETCH":
                self.backward_prefetch = None
            elif bp in FSDP_BACKWARD_PREFETCH or bp.isdigit():
                self.backward_prefetch = FSDP_BACKWARD_PREFETCH[int(bp) - 1] if bp.isdigit() else bp
            else:
                raise ValueError(f"Unknown backward_prefetch {bp}")

        self.set_state_dict_type()

        if self.auto_wrap_policy is None:
            self.auto_wrap_policy = os.environ.get(env_prefix + "AUTO_WRAP_POLICY", "NO_WRAP")
        if isinstance(self.auto_wrap_policy, str):
            p = self.auto_wrap_policy.upper()
            if p not in FSDP_AUTO_WRAP_POLICY:
                raise ValueError(f"Invalid auto wrap policy {p}; choose from {FSDP_AUTO_WRAP_POLICY}")
            self.auto_wrap_policy = p
            if p == "TRANSFORMER_BASED_WRAP" and self.transformer_cls_names_to_wrap is None:
                names = os.environ.get(env_prefix + "TRANSFORMER_CLS_TO_WRAP", None)
                if names:
                    self.transformer_cls_names_to_wrap = [n.strip() for n in names.split(",")]
            elif p == "SIZE_BASED_WRAP" and self.min_num_params is None:
                self.min_num_params = int(os.environ.get(env_prefix + "MIN_NUM_PARAMS", 0))

        if self.use_orig_params is None:
            self.use_orig_params = str_to_bool(os.environ.get(env_prefix + "USE_ORIG_PARAMS", "False")) == 1
        if self.sync_module_states is None:
            self.sync_module_states = str_to_bool(os.environ.get(env_prefix + "SYNC_MODULE_STATES", "False")) == 1
        if self.forward_prefetch is None:
            self.forward_prefetch = str_to_bool(os.environ.get(env_prefix + "FORWARD_PREFETCH", "False")) == 1
        if self.activation_checkpointing is None:
            self.activation_checkpointing = str_to_bool(os.environ.get(env_prefix + "ACTIVATION_CHECKPOINTING", "False")) == 1
        if self.cpu_ram_efficient_loading is None:
            self.cpu_ram_efficient_loading = (
                str_to_bool(os.environ.get(env_prefix + "CPU_RAM_EFFICIENT_LOADING", "False")) == 1
            )
        if self.ignored_modules is None:
            self.ignored_modules = _parse_ignored_modules(os.environ.get(env_prefix + "IGNORED_MODULES", None))
        if isinstance(self.mixed_precision_policy, (dict, str, torch.dtype)):
            self.set_mixed_precision(self.mixed_precision_policy, override=True)

    # -- state dict ---------------------------------------------------------------------------------
    def set_state_dict_type(self, state_dict_type=None):
        if state_dict_type is not None:
            self.state_dict_type = state_dict_type
        if self.state_dict_type is None:
            self.state_dict_type = os.environ.get(
                "FSDP_STATE_DICT_TYPE", "FULL_STATE_DICT" if self.fsdp_version == 1 else "SHARDED_STATE_DICT"
            )
        if isinstance(self.state_dict_type, int) or (isinstance(self.state_dict_type, str) and self.state_dict_type.isdigit()):
            self.state_dict_type = FSDP_STATE_DICT_TYPE[int(self.state_dict_type) - 1]
        self.state_dict_type = str(getattr(self.state_dict_type, "name", self.state_dict_type)).upper()
        if self.state_dict_type not in FSDP_STATE_DICT_TYPE:
            raise ValueError(f"Unknown state_dict_type {self.state_dict_type}")
        if self.fsdp_version == 2 and self.state_dict_type not in FSDP2_STATE_DICT_TYPE:
            raise ValueError(f"FSDP2 supports {FSDP2_STATE_DICT_TYPE}, got {self.state_dict_type}")
        if self.state_dict_config is None:
            self.state_dict_config = {"offload_to_cpu": True, "rank0_only": True}
        if self.optim_state_dict_config is None:
            self.optim_state_dict_config = {"offload_to_cpu": True, "rank0_only": True}

    # -- wrapping -----------------------------------------------------------------------------------
    def set_auto_wrap_policy(self, model):
        """Resolve the wrap policy into a predicate `fn(module) -> bool` used by the engine."""
        if callable(self.auto_wrap_policy) and not isinstance(self.auto_wrap_policy, str):
            return self.auto_wrap_policy
        policy = self.auto_wrap_policy
        if policy == "TRANSFORMER_BASED_WRAP":
            names = self.transformer_cls_names_to_wrap
            if not names:
                names = list(getattr(model, "_no_split_modules", None) or [])
            classes = set()
            for n in names:
                cls = get_module_class_from_name(model, n)
                if cls is None:
                    raise ValueError(f"Could not find the transformer layer class {n} in the model.")
                classes.add(cls)
            self.transformer_cls_names_to_wrap = names
            self._wrap_classes = classes
            fn = lambda m: isinstance(m, tuple(classes))  # noqa: E731
        elif policy == "SIZE_BASED_WRAP":
            threshold = self.min_num_params or 0
            if threshold <= 0:
                fn = None
            else:
                fn = lambda m: sum(p.numel() for p in m.parameters(recurse=True)) >= threshold  # noqa: E731
        else:
            fn = None
        self._wrap_fn = fn
        return fn

    def set_mixed_precision(self, mixed_precision, buffer_autocast=False, override=False):
        mapping = {"fp8": torch.bfloat16, "fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32, "no": torch.float32}
        if isinstance(mixed_precision, dict):
            mp = {k: (mapping[v] if isinstance(v, str) else v) for k, v in mixed_precision.items()}
            self.mixed_precision_policy = MixedPrecisionPolicy(**mp)
            return
        if isinstance(mixed_precision, MixedPrecisionPolicy):
            self.mixed_precision_policy = mixed_precision
            return
        dtype = mapping.get(mixed_precision, None) if isinstance(mixed_precision, str) else mixed_precision
        if dtype is None:
            raise ValueError(f"Invalid mixed precision {mixed_precision}")
        if override or self.mixed_precision_policy is None:
            self.mixed_precision_policy = MixedPrecisionPolicy(param_dtype=dtype, reduce_dtype=dtype, output_dtype=dtype)

    def set_cpu_offload(self):
        pass

    def validate_cpu_offload(self):
        pass


@dataclass
class TorchTensorParallelPlugin:
    """Deprecated alias kept for parity (reference `dataclasses.py:2170-2182`)."""

    tp_size: int = 1
    torch_device_mesh: Any = None


@dataclass
class TorchContextParallelConfig:
    """Ring-attention context parallel config. `allgather` gathers K/V once per layer over the `cp`
    communicator; `alltoall` rotates K/V around a P2P ring overlapped with the local block."""

    cp_comm_strategy: Literal["allgather", "alltoall"] = None

    def __post_init__(self):
        if self.cp_comm_strategy is None:
            self.cp_comm_strategy = os.environ.get("PARALLELISM_CONFIG_CP_COMM_STRATEGY", "allgather")
        if self.cp_comm_strategy not in ("allgather", "alltoall"):
            raise ValueError(f"cp_comm_strategy must be 'allgather' or 'alltoall', got {self.cp_comm_strategy}")


@dataclass
class DeepSpeedSequenceParallelConfig:
    """Ulysses sequence-parallel config; served by our RCCL all-to-all implementation (parallel/ulysses.py)."""

    sp_seq_length: Optional[int] = None
    sp_seq_length_is_variable: Optional[bool] = None
    sp_attn_implementation: Optional[str] = None

    def __post_init__(self):
        prefix = "PARALLELISM_CONFIG_SP_"
        if self.sp_seq_length_is_variable is None:
            self.sp_seq_length_is_variable = os.environ.get(prefix + "SEQ_LENGTH_IS_VARIABLE", "true").lower() == "true"
        if self.sp_seq_length is None and prefix + "SEQ_LENGTH" in os.environ:
            self.sp_seq_length = int(os.environ[prefix + "SEQ_LENGTH"])
        if self.sp_attn_implementation is None:
            self.sp_attn_implementation = os.environ.get(prefix + "ATTN_IMPLEMENTATION", "sdpa")


@dataclass
class TorchTensorParallelConfig:
    """TP options (parity: reference dataclasses.py:2263-2282). `sequence_parallel` keeps the residual stream
    sequence-sharded between TP regions (all-gather / reduce-scatter instead of all-reduce)."""

    enable_async_tp: bool = False
    sequence_parallel: bool = False


@dataclass
class MegatronLMPlugin:
    """Accepted for config compatibility. Megatron-LM is not a dependency; its capabilities
    (TP/CP/SP/EP) are provided by `ParallelismConfig` + parallel/*. Instantiating raises."""

    tp_degree: int = None
    pp_degree: int = None
    num_micro_batches: int = None

    def __post_init__(self):
        raise NotImplementedError(
            "Megatron-LM is not supported on this MI355X framework; use ParallelismConfig(tp_size=..., cp_size=...)."
        )


@dataclass
class BnbQuantizationConfig:
    """bitsandbytes has no MI355X build here; accepted for import compatibility only."""

    load_in_8bit: bool = False
    load_in_4bit: bool = False

    def __post_init__(self):
        if self.load_in_8bit or self.load_in_4bit:
            raise NotImplementedError("bitsandbytes quantization is not available on MI355X.")


def get_module_class_from_name(module: torch.nn.Module, name: str):
    """Find the class named `name` among `module` and its descendants (reference `dataclasses.py:3179-3196`)."""
    modules_children = list(module.children())
    if module.__class__.__name__ == name:
        return module.__class__
    if len(modules_children) == 0:
        return None
    for child_module in modules_children:
        module_class = get_module_class_from_name(child_module, name)
        if module_class is not None:
            return module_class
    return None


def add_model_config_to_megatron_parser(*args, **kwargs):  # pragma: no cover - API stub
    raise NotImplementedError("Megatron-LM is not supported.")
