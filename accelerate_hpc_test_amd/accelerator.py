"""`Accelerator`: the public facade of the framework.

Parity: `/root/reference/src/accelerate/accelerator.py:184-4324`. Same constructor arguments, properties and methods
(`prepare`, `backward`, `accumulate`, `no_sync`, `gather(_for_metrics)`, `reduce`, `clip_grad_norm_`,
`save_state`/`load_state`, `save_model`, `unwrap_model`, `autocast`, `profile`, trackers, ...), the same
gradient-accumulation semantics (`_do_sync`, loss division, scheduler interplay) and the same checkpoint layout.

What the methods drive is MI355X-native:
* DDP → `parallel/ddp.py` (own bucketed RCCL reducer; 128 MB xGMI-sized buckets, comm stream overlap);
* FSDP (v1 flags mapped to v2 semantics) → `parallel/fsdp.py` (flat-shard engine, RCCL all-gather /
  reduce-scatter on side streams, fp32 master shards, fused HIP AdamW writing the bf16 all-gather source);
* `clip_grad_norm_` → HIP multi-tensor L2 norm + device-side clip (+ one all-reduce when sharded), no host sync;
* AdamW/Adam → HIP multi-tensor kernel (`ops/multi_tensor.py`);
* fp8 (`mixed_precision="fp8"`) → our `Fp8Linear` (HIP amax / cast / MX-MFMA GEMM) swapped into the model;
* dataloaders → `DataLoaderShard` with a copy-stream device prefetcher;
* context / sequence / tensor parallelism → `parallel/context_parallel.py`, `parallel/ulysses.py`, `parallel/tensor_parallel.py`.
"""

from __future__ import annotations

import contextlib
import functools
import json
import math
import os
import re
import shutil
import warnings
from collections import OrderedDict
from functools import partial
from types import MethodType
from typing import Any, Callable, Optional, Union

import torch
import torch.utils.hooks as hooks

from .checkpointing import load_accelerator_state, load_custom_state, save_accelerator_state, save_custom_state
from .data_loader import DataLoaderDispatcher, DataLoaderShard, prepare_data_loader, skip_first_batches
from .logging import get_logger
from .optimizer import AcceleratedOptimizer
from .parallelism_config import ParallelismConfig
from .scheduler import AcceleratedScheduler
from .state import AcceleratorState, GradientState, PartialState
from .tracking import LOGGER_TYPE_TO_CLASS, GeneralTracker, filter_trackers
from .utils.constants import (
    FSDP_MODEL_NAME,
    PROFILE_PATTERN_NAME,
    SAFE_WEIGHTS_INDEX_NAME,
    SAFE_WEIGHTS_NAME,
    SAFE_WEIGHTS_PATTERN_NAME,
    WEIGHTS_INDEX_NAME,
    WEIGHTS_NAME,
    WEIGHTS_PATTERN_NAME,
)
from .utils.dataclasses import (
    AORecipeKwargs,
    AutocastKwargs,
    DataLoaderConfiguration,
    DeepSpeedPlugin,
    DistributedDataParallelKwargs,
    DistributedType,
    DynamoBackend,
    FP8RecipeKwargs,
    FullyShardedDataParallelPlugin,
    GradientAccumulationPlugin,
    GradScalerKwargs,
    InitProcessGroupKwargs,
    KwargsHandler,
    LoggerType,
    MegatronLMPlugin,
    MSAMPRecipeKwargs,
    PrecisionType,
    ProfileKwargs,
    ProjectConfiguration,
    RcclKwargs,
    RNGType,
    TERecipeKwargs,
    TorchDynamoPlugin,
)
from .utils.environment import parse_choice_from_env, parse_flag_from_env, str_to_bool
from .utils.memory import clear_device_cache, release_memory
from .utils.modeling import convert_file_size_to_int, get_mixed_precision_context_manager, id_tensor_storage
from .utils.operations import (
    convert_outputs_to_fp32,
    gather,
    gather_object,
    pad_across_processes,
    recursively_apply,
    reduce,
    send_to_device,
)
from .utils.other import (
    check_os_kernel,
    clean_state_dict_for_safetensors,
    compile_regions,
    extract_model_from_parallel,
    has_compiled_regions,
    is_compiled_module,
    save,
)

from .utils.fault_tolerance import FaultInjector, StepWatchdog, check_collective_sequence  # noqa: E402

logger = get_logger(__name__)

_split_batches = object()  # sentinel, as in the reference
_dispatch_batches = object()
_even_batches = object()
_use_seedable_sampler = object()




def _delegate(path: str, settable: bool = False) -> property:
    """A property reading (and, when `settable`, writing) `self.<owner>.<attr>` for `path` = "owner.attr" (or a plain
    attribute name)."""
    owner, _, attr = path.rpartition(".")

    def _target(self):
        return getattr(self, owner) if owner else self

    def fget(self):
        return getattr(_target(self), attr)

    def fset(self, value):
        setattr(_target(self), attr, value)

    return property(fget, fset if settable else None, doc=f"`{path}`")

class _CheckpointRotation:
    """Automatic checkpoint naming of `ProjectConfiguration`: `<project_dir>/checkpoints/checkpoint_<k>` directories,
    ordered by the number in their name, at most `total_limit` kept."""

    _NUM = re.compile(r"(\d+)(?!.*\d)")

    def __init__(self, project_configuration):
        self.cfg = project_configuration
        self.enabled = bool(project_configuration.automatic_checkpoint_naming)
        self.root = os.path.join(project_configuration.project_dir or ".", "checkpoints")

    def existing(self) -> list:
        if not os.path.isdir(self.root):
            return []
        dirs = [os.path.join(self.root, d) for d in os.listdir(self.root)]
        return sorted((d for d in dirs if self._NUM.search(os.path.basename(d))),
                      key=lambda d: int(self._NUM.search(os.path.basename(d)).group(1)))

    def prune_for_one_more(self):
        limit = self.cfg.total_limit
        have = self.existing()
        if limit is not None and len(have) + 1 > limit:
            drop = have[: len(have) + 1 - limit]
            logger.warning(f"Deleting {len(drop)} checkpoints to make room for new checkpoint.")
            for d in drop:
                shutil.rmtree(d)

    def next_dir(self, iteration: int) -> str:
        out = os.path.join(self.root, f"checkpoint_{iteration}")
        if os.path.exists(out):
            raise ValueError(f"Checkpoint directory {out} ({iteration}) already exists. Please manually override "
                             "`self.save_iteration` with what iteration to start with.")
        return out

    def latest(self) -> str:
        have = self.existing()
        if not have:
            raise ValueError(f"No checkpoints found in {self.root}")
        return have[-1]

    @staticmethod
    def custom_state_files(folder: str) -> list:
        return [f for f in os.listdir(folder) if re.fullmatch(r"custom_checkpoint_\d+\.pkl", f)]


def _only_tensors(data) -> bool:
    """True when `data` is a (nested) structure of tensors only."""
    try:
        recursively_apply(lambda x: x, data, error_on_other_type=True)
    except TypeError:
        return False
    return True

def _any_dtensor(params) -> bool:
    try:
        from torch.distributed.tensor import DTensor
    except ImportError:  # pragma: no cover
        return False
    return any(isinstance(p, DTensor) or isinstance(p.grad, DTensor) for p in params)


class Accelerator:
    def __init__(
        self,
        device_placement: bool = True,
        split_batches: bool = _split_batches,
        mixed_precision: Union[PrecisionType, str, None] = None,
        gradient_accumulation_steps: int = 1,
        cpu: bool = False,
        dataloader_config: Optional[DataLoaderConfiguration] = None,
        deepspeed_plugin: Optional[Union[DeepSpeedPlugin, dict]] = None,
        fsdp_plugin: Optional[FullyShardedDataParallelPlugin] = None,
        torch_tp_plugin=None,
        megatron_lm_plugin: Optional[MegatronLMPlugin] = None,
        rng_types: Optional[list[Union[str, RNGType]]] = None,
        log_with: Optional[Union[str, LoggerType, GeneralTracker, list]] = None,
        project_dir: Optional[Union[str, os.PathLike]] = None,
        project_config: Optional[ProjectConfiguration] = None,
        gradient_accumulation_plugin: Optional[GradientAccumulationPlugin] = None,
        step_scheduler_with_optimizer: bool = True,
        kwargs_handlers: Optional[list[KwargsHandler]] = None,
        dynamo_backend: Union[DynamoBackend, str, None] = None,
        dynamo_plugin: Optional[TorchDynamoPlugin] = None,
        deepspeed_plugins=None,
        parallelism_config: Optional[ParallelismConfig] = None,
    ):
        self.trackers = []
        if project_config is not None:
            self.project_configuration = project_config
        else:
            self.project_configuration = ProjectConfiguration(project_dir=project_dir)
        if project_dir is not None and self.project_dir is None:
            self.project_configuration.set_directories(project_dir)
        if mixed_precision is not None:
            mixed_precision = str(mixed_precision)
            if mixed_precision not in PrecisionType:
                raise ValueError(f"Unknown mixed_precision mode: {mixed_precision}. Choose between {PrecisionType.list()}")
        if torch_tp_plugin is not None:
            warnings.warn("`torch_tp_plugin` is deprecated; use `parallelism_config=ParallelismConfig(tp_size=...)`.", FutureWarning)
        if dynamo_plugin is not None and dynamo_backend is not None:
            raise ValueError("You cannot pass in both `dynamo_plugin` and `dynamo_backend`, please only pass in one.")
        if dynamo_backend is not None:
            dynamo_plugin = TorchDynamoPlugin(backend=dynamo_backend)
        elif dynamo_plugin is None:
            dynamo_plugin = TorchDynamoPlugin()
        if deepspeed_plugins is not None and deepspeed_plugin is None:
            deepspeed_plugin = deepspeed_plugins if not isinstance(deepspeed_plugins, dict) else next(iter(deepspeed_plugins.values()))
        if deepspeed_plugin is None and parse_flag_from_env("ACCELERATE_USE_DEEPSPEED"):
            deepspeed_plugin = DeepSpeedPlugin()
        if isinstance(deepspeed_plugin, dict):
            deepspeed_plugin = DeepSpeedPlugin(hf_ds_config=deepspeed_plugin)
        if os.environ.get("ACCELERATE_USE_FSDP", "false").lower() == "true" or isinstance(fsdp_plugin, FullyShardedDataParallelPlugin):
            if fsdp_plugin is None:
                fsdp_plugin = FullyShardedDataParallelPlugin()
        if megatron_lm_plugin is None and parse_flag_from_env("ACCELERATE_USE_MEGATRON_LM"):
            megatron_lm_plugin = MegatronLMPlugin()

        # kwargs handlers
        self.ddp_handler = None
        self.scaler_handler = None
        self.init_handler = None
        self.fp8_recipe_handler = None
        self.ao_recipe_handler = None
        self.te_recipe_handler = None
        self.autocast_handler = None
        self.profile_handler = None
        self.has_lomo_optimizer = False
        self.rccl_handler = RcclKwargs()
        found_handlers = set()
        handler_class_to_attr = {
            DistributedDataParallelKwargs: "ddp_handler",
            GradScalerKwargs: "scaler_handler",
            InitProcessGroupKwargs: "init_handler",
            FP8RecipeKwargs: "fp8_recipe_handler",
            AutocastKwargs: "autocast_handler",
            ProfileKwargs: "profile_handler",
            AORecipeKwargs: "ao_recipe_handler",
            TERecipeKwargs: "te_recipe_handler",
            RcclKwargs: "rccl_handler",
        }
        if kwargs_handlers is not None:
            for handler in kwargs_handlers:
                assert isinstance(handler, KwargsHandler), f"Unsupported kwargs handler passed: {handler}, must be one that inherits `accelerate.utils.KwargsHandler`."
                handler_class = handler.__class__
                if isinstance(handler, MSAMPRecipeKwargs):
                    raise NotImplementedError("MS-AMP is not supported on MI355X.")
                for cls, attr in handler_class_to_attr.items():
                    if handler_class is cls or (cls is FP8RecipeKwargs and isinstance(handler, FP8RecipeKwargs)):
                        if handler_class in found_handlers:
                            raise ValueError(f"You can only pass one {handler_class} in `kwargs_handlers`.")
                        found_handlers.add(handler_class)
                        setattr(self, attr, handler)
        if parallelism_config is None and parse_flag_from_env("ACCELERATE_USE_PARALLELISM_CONFIG"):
            parallelism_config = ParallelismConfig()
        kwargs = self.init_handler.to_kwargs() if self.init_handler is not None else {}
        self.state = AcceleratorState(
            mixed_precision=mixed_precision,
            cpu=cpu,
            dynamo_plugin=dynamo_plugin,
            deepspeed_plugin=deepspeed_plugin,
            fsdp_plugin=fsdp_plugin,
            torch_tp_plugin=torch_tp_plugin,
            megatron_lm_plugin=megatron_lm_plugin,
            parallelism_config=parallelism_config,
            _from_accelerator=True,
            **kwargs,
        )
        self.parallelism_config = parallelism_config
        if parallelism_config is not None:
            parallelism_config._validate_accelerator(self)
            self.state.device_mesh = parallelism_config.get_device_mesh(self.device.type) if self.use_distributed else None
        self.delayed_fp8_autocast = False
        self._fp8_backend = None
        if self.state.mixed_precision == "fp8":
            if self.te_recipe_handler is not None or self.fp8_recipe_handler is not None:
                self._fp8_backend = "TE"
            else:
                self._fp8_backend = "AO"
                if self.ao_recipe_handler is None:
                    self.ao_recipe_handler = AORecipeKwargs()

        trackers = filter_trackers(log_with, self.logging_dir)
        if len(trackers) < 1 and log_with is not None:
            warnings.warn(f"`log_with={log_with}` was passed but no supported trackers are currently installed.")
        self.log_with = trackers

        if (
            (mixed_precision != "bf16")
            and getattr(self.state, "downcast_bfloat", False)
            and (self.state.distributed_type != DistributedType.XLA)
        ):
            raise ValueError("Can only use `downcast_bf16` when using `mixed_precision='bf16'` and on a TPU")

        if gradient_accumulation_plugin is not None:
            if gradient_accumulation_steps != 1:
                raise ValueError(
                    "You can only pass one of `gradient_accumulation_steps` and `gradient_accumulation_plugin`. Please only pass in the created `GradientAccumulationPlugin` object."
                )
        else:
            gradient_accumulation_steps = int(
                parse_choice_from_env("ACCELERATE_GRADIENT_ACCUMULATION_STEPS", gradient_accumulation_steps)
            )
            gradient_accumulation_plugin = GradientAccumulationPlugin(num_steps=gradient_accumulation_steps)
        self.gradient_state = GradientState(gradient_accumulation_plugin=gradient_accumulation_plugin)

        self.device_placement = device_placement
        if dataloader_config is None:
            dataloader_config = DataLoaderConfiguration()
        self.dataloader_config = dataloader_config
        if split_batches is not _split_batches:
            warnings.warn("Passing `split_batches` to Accelerator is deprecated; use DataLoaderConfiguration.", FutureWarning)
            self.dataloader_config.split_batches = split_batches
        self.step_scheduler_with_optimizer = step_scheduler_with_optimizer

        # Mixed precision attributes
        self.scaler = None
        self.native_amp = False
        if self.state.mixed_precision == "fp16" and self.device.type != "cpu":
            self.native_amp = True
            kwargs = self.scaler_handler.to_kwargs() if self.scaler_handler is not None else {}
            from .ops._ext import native_enabled

            if native_enabled():
                from .ops.amp import HipGradScaler  # unscale + overflow check on the multi-tensor HIP kernel

                self.scaler = HipGradScaler("cuda", **kwargs)
            else:
                self.scaler = torch.amp.GradScaler("cuda", **kwargs)
        elif self.state.mixed_precision in ("bf16", "fp8"):
            self.native_amp = True
        elif self.state.mixed_precision == "fp16" and self.device.type == "cpu":
            self.native_amp = True

        self.step = 0
        self._optimizers = []
        self._models = []
        self._schedulers = []
        self._dataloaders = []
        self._custom_objects = []
        self._fsdp_engines = []
        self._save_model_state_pre_hook = OrderedDict()
        self._load_model_state_pre_hook = OrderedDict()
        self.rng_types = rng_types
        if self.rng_types is None:
            self.rng_types = ["generator"]
        self.flag_tensor = None
        self._cp_context = None
        # failure detection / fault drills (utils/fault_tolerance.py)
        self._backward_calls = 0
        self._watchdog = StepWatchdog.from_env(self.rccl_handler.watchdog_timeout, rank=self.process_index)
        self._fault_injector = FaultInjector.from_env(self.process_index)
        check_os_kernel()
        if (self.device.type == "cuda" and self.num_processes > 1
                and os.environ.get("ACCELERATE_CHECK_TOPOLOGY", "1") != "0"):
            # xGMI links between this node's GPUs, P2P / IPC switches (parallel/topology.py). Local rank 0
            # inspects (rocm-smi once per node); with ACCELERATE_STRICT_TOPOLOGY=1 the verdict is all-reduced so that
            # EVERY rank raises, instead of the others hanging at their first collective
            from .parallel.topology import validate_comm_environment

            strict = os.environ.get("ACCELERATE_STRICT_TOPOLOGY", "0") == "1"
            problems = []
            if self.local_process_index == 0:
                problems = validate_comm_environment(
                    int(os.environ.get("LOCAL_WORLD_SIZE", self.num_processes) or self.num_processes), strict=False)
            if strict:
                flag = torch.tensor([1.0 if problems else 0.0], device=self.device)
                torch.distributed.all_reduce(flag)
                if flag.item() > 0:
                    raise RuntimeError("communication environment check failed on a node (ACCELERATE_STRICT_TOPOLOGY=1)"
                                       + (": " + "; ".join(problems) if problems else ""))

    # ============================================================================== properties
    # Read-through views of the process state and the dataloader / project configurations (`_delegate`, module
    # level); derived properties follow.
    use_distributed = _delegate("state.use_distributed")
    distributed_type = _delegate("state.distributed_type")
    num_processes = _delegate("state.num_processes")
    process_index = _delegate("state.process_index")
    local_process_index = _delegate("state.local_process_index")
    device = _delegate("state.device")
    is_main_process = _delegate("state.is_main_process")
    is_local_main_process = _delegate("state.is_local_main_process")
    mixed_precision = _delegate("state.mixed_precision")
    torch_device_mesh = _delegate("state.device_mesh")
    split_batches = _delegate("dataloader_config.split_batches")
    dispatch_batches = _delegate("dataloader_config.dispatch_batches")
    even_batches = _delegate("dataloader_config.even_batches", settable=True)
    use_seedable_sampler = _delegate("dataloader_config.use_seedable_sampler")
    non_blocking = _delegate("dataloader_config.non_blocking")
    use_stateful_dataloader = _delegate("dataloader_config.use_stateful_dataloader")
    project_dir = _delegate("project_configuration.project_dir")
    logging_dir = _delegate("project_configuration.logging_dir")
    save_iteration = _delegate("project_configuration.iteration")
    sync_gradients = _delegate("gradient_state.sync_gradients", settable=True)
    fp8_backend = _delegate("_fp8_backend")

    @property
    def deepspeed_plugin(self):
        return None  # DeepSpeed is not part of this build

    @property
    def multi_device(self):
        return self.use_distributed and self.distributed_type in (DistributedType.MULTI_GPU, DistributedType.FSDP)

    @property
    def is_last_process(self):
        return self.process_index == self.num_processes - 1

    @property
    def is_fsdp2(self):
        return self.state.distributed_type == DistributedType.FSDP and self.state.fsdp_plugin.fsdp_version == 2

    @property
    def is_composable_parallelism_enabled(self):
        return self.is_fsdp2

    @property
    def should_save_model(self):
        return True

    @property
    def tensor_parallel_rank(self) -> int:
        if self.parallelism_config and self.parallelism_config.tp_enabled:
            return self.torch_device_mesh.local_rank("tp")
        raise RuntimeError("Tensor parallelism is not enabled. Please check your configuration.")

    @property
    def pipeline_parallel_rank(self) -> int:
        raise NotImplementedError("Pipeline parallelism is currently not supported in Accelerate.")

    @property
    def context_parallel_rank(self) -> int:
        if self.parallelism_config and self.parallelism_config.cp_enabled:
            return self.torch_device_mesh.local_rank("cp")
        raise RuntimeError("Context parallelism is not enabled. Please check your configuration.")

    @property
    def data_parallel_rank(self) -> int:
        if self.parallelism_config and self.torch_device_mesh is not None:
            return self.torch_device_mesh.local_rank("dp")
        return self.process_index

    @property
    def data_parallel_shard_rank(self) -> int:
        if self.parallelism_config and self.parallelism_config.dp_shard_enabled:
            return self.torch_device_mesh.local_rank("dp_shard")
        raise RuntimeError("Data parallelism sharding is not enabled. Please check your configuration.")

    @property
    def gradient_accumulation_steps(self):
        return self.gradient_state.num_steps

    @gradient_accumulation_steps.setter
    def gradient_accumulation_steps(self, gradient_accumulation_steps):
        self.gradient_state.plugin_kwargs.update({"num_steps": gradient_accumulation_steps})

    @property
    def optimizer_step_was_skipped(self):
        for optimizer in self._optimizers:
            if optimizer.step_was_skipped:
                return True
        return False

    # ============================================================================== process control
    def on_main_process(self, function: Callable[..., Any] = None):
        if function is None:
            if "Accelerator." in self.__class__.__name__:
                function = self
            else:
                raise ValueError("The `on_main_process` decorator must be called with a function on an instantiated `Accelerator` object.")

        def _inner(*args, **kwargs):
            return PartialState().on_main_process(function)(*args, **kwargs)

        return _inner

    def on_local_main_process(self, function: Callable[..., Any] = None):
        def _inner(*args, **kwargs):
            return PartialState().on_local_main_process(function)(*args, **kwargs)

        return _inner

    def on_last_process(self, function: Callable[..., Any]):
        def _inner(*args, **kwargs):
            return PartialState().on_last_process(function)(*args, **kwargs)

        return _inner

    def on_process(self, function: Callable[..., Any] = None, process_index: int = None):
        if function is None:
            return partial(self.on_process, process_index=process_index)

        def _inner(*args, **kwargs):
            return PartialState().on_process(function, process_index)(*args, **kwargs)

        return _inner

    def on_local_process(self, function: Callable[..., Any] = None, local_process_index: int = None):
        if function is None:
            return partial(self.on_local_process, local_process_index=local_process_index)

        def _inner(*args, **kwargs):
            return PartialState().on_local_process(function, local_process_index)(*args, **kwargs)

        return _inner

    @contextlib.contextmanager
    def main_process_first(self):
        with self.state.main_process_first():
            yield

    @contextlib.contextmanager
    def local_main_process_first(self):
        with self.state.local_main_process_first():
            yield

    @contextlib.contextmanager
    def split_between_processes(self, inputs, apply_padding: bool = False):
        with PartialState().split_between_processes(inputs, apply_padding=apply_padding) as inputs:
            yield inputs

    def print(self, *args, **kwargs):
        self.state.print(*args, **kwargs)

    def wait_for_everyone(self):
        PartialState().wait_for_everyone()

    # ============================================================================== gradient sync control
    @contextlib.contextmanager
    def no_sync(self, model):
        context = contextlib.nullcontext
        if self.use_distributed or self.distributed_type == DistributedType.FSDP:
            if hasattr(model, "no_sync"):
                context = getattr(model, "no_sync")
        with context():
            yield

    @staticmethod
    @contextlib.contextmanager
    def trigger_sync_in_backward(model):
        if not hasattr(model, "require_backward_grad_sync") and not hasattr(model, "set_requires_gradient_sync"):
            yield
            return
        if hasattr(model, "set_requires_gradient_sync"):
            old = model.engine.requires_grad_sync
            model.set_requires_gradient_sync(True)
            try:
                yield
            finally:
                model.set_requires_gradient_sync(old)
            return
        old = model.require_backward_grad_sync
        model.require_backward_grad_sync = True
        if hasattr(model, "trigger_sync"):
            model.trigger_sync()
        try:
            yield
        finally:
            model.require_backward_grad_sync = old

    def _do_sync(self):
        if self.gradient_state.sync_with_dataloader and self.gradient_state.end_of_dataloader:
            self.step = 0
            self.gradient_state._set_sync_gradients(True)
        else:
            self.step += 1
            self.gradient_state._set_sync_gradients((self.step % self.gradient_state.num_steps) == 0)

    @contextlib.contextmanager
    def accumulate(self, *models):
        self._do_sync()
        allow_gradient_sync = self.sync_gradients or (
            self.use_distributed and self.gradient_state.plugin_kwargs.get("sync_each_batch", False)
        )
        with contextlib.ExitStack() as cm_stack:
            for m in models:
                cm_stack.enter_context(contextlib.nullcontext() if allow_gradient_sync else self.no_sync(m))
            yield

    @contextlib.contextmanager
    def join_uneven_inputs(self, joinables, even_batches=None):
        """Train on uneven per-rank inputs (reference accelerator.py:1298-1379): optionally override `even_batches`
        on the prepared loaders and enter each DDP joinable's `join()` — ranks that finish early shadow the
        others' gradient all-reduces with zeros until everyone is done (parallel/ddp.py)."""
        if self.distributed_type in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU):
            with contextlib.ExitStack() as stack:
                for j in joinables:
                    if hasattr(j, "join") and hasattr(j, "buckets"):
                        stack.enter_context(j.join())
                with self._override_even_batches(even_batches):
                    yield
        else:
            if self.distributed_type != DistributedType.NO:
                warnings.warn("Joining uneven inputs is only supported for multi-GPU training, as a result `join_uneven_inputs` will have no effect.")
            yield

    @contextlib.contextmanager
    def _override_even_batches(self, even_batches):
        saved = []
        if even_batches is not None:
            iterable_seen = False
            for dl in self._dataloaders:
                if isinstance(dl, DataLoaderDispatcher):
                    iterable_seen = True
                    continue
                bs = getattr(dl, "batch_sampler", None)
                if bs is not None and hasattr(bs, "even_batches"):
                    saved.append((bs, bs.even_batches))
                    bs.even_batches = even_batches
            if iterable_seen:
                warnings.warn("Overriding even_batches is only supported for map-style datasets, yet some dataloaders given were iterable")
        try:
            yield
        finally:
            for bs, value in saved:
                bs.even_batches = value

    # ============================================================================== prepare
    def _prepare_one(self, obj, first_pass=False, device_placement=None):
        if first_pass:
            if isinstance(obj, torch.utils.data.DataLoader):
                return self.prepare_data_loader(obj, device_placement=device_placement)
            elif isinstance(obj, torch.nn.Module):
                return self.prepare_model(obj, device_placement=device_placement)
            elif isinstance(obj, torch.optim.Optimizer):
                optimizer = self.prepare_optimizer(obj, device_placement=device_placement)
                return optimizer
        elif isinstance(obj, torch.optim.lr_scheduler.LRScheduler):
            scheduler = self.prepare_scheduler(obj)
            return scheduler
        return obj

    def prepare(self, *args, device_placement=None):
        """Prepare models, optimizers, dataloaders and schedulers for the configured distributed setup."""
        if device_placement is None:
            device_placement = [None for _ in args]
        elif len(device_placement) != len(args):
            raise ValueError(f"`device_placement` should be a list with {len(args)} elements (the number of objects passed).")
        for obj in args:
            if isinstance(obj, torch.nn.Module) and self.verify_device_map(obj) and self.distributed_type != DistributedType.NO:
                raise ValueError(
                    "You can't train a model that has been loaded with `device_map='auto'` in any distributed mode."
                    " Please rerun your script specifying `--num_processes=1` or by launching with `python {{myscript.py}}`."
                )
        if self.distributed_type == DistributedType.FSDP:
            models = [o for o in args if isinstance(o, torch.nn.Module)]
            if len(models) > 1:
                raise AssertionError("You can't use same `Accelerator()` instance with multiple models when using FSDP2")
        if self.state.mixed_precision == "fp8":
            for obj in args:
                if isinstance(obj, torch.nn.Module) and not getattr(obj, "_acc_fp8_converted", False):
                    self._convert_fp8(obj)

        # Pass 1: dataloaders + models; optimizers are remapped to sharded params before being wrapped.
        result = []
        for obj, d in zip(args, device_placement):
            if isinstance(obj, (torch.utils.data.DataLoader, torch.nn.Module)):
                result.append(self._prepare_one(obj, first_pass=True, device_placement=d))
            else:
                result.append(obj)
        for i, (obj, d) in enumerate(zip(result, device_placement)):
            if isinstance(obj, torch.optim.Optimizer) and not isinstance(obj, AcceleratedOptimizer):
                self._remap_optimizer_params(obj)
                result[i] = self._prepare_one(obj, first_pass=True, device_placement=d)
        # Pass 2: schedulers (they need the wrapped optimizers)
        result = tuple(self._prepare_one(obj, device_placement=d) for obj, d in zip(result, device_placement))
        for item in result:
            if any(item in container for container in (self._dataloaders, self._models, self._optimizers, self._schedulers)):
                item._is_accelerate_prepared = True
        if self.parallelism_config is not None and self.parallelism_config.sp_enabled:
            # reference accelerator.py:2393-2409: sequence-parallel data-loader adapter after the model is prepared
            result = tuple(self.deepspeed_ulysses_dl_adapter(x, None) if isinstance(x, (DataLoaderShard, DataLoaderDispatcher)) else x for x in result)
        return result if len(result) > 1 else result[0]

    def deepspeed_ulysses_dl_adapter(self, dl, model=None):
        """Cut batches along the sequence for Ulysses SP (parity name with reference accelerator.py:2458-2476)."""
        if self.parallelism_config is None or not self.parallelism_config.sp_enabled:
            return dl
        from .parallel.ulysses import UlyssesSPDataLoaderAdapter

        mesh = self.torch_device_mesh
        return UlyssesSPDataLoaderAdapter(dl, sp_rank=mesh.local_rank("sp"), sp_group=mesh.group("sp"),
                                          sp_world_size=mesh.size("sp"), device=self.device)

    def _remap_optimizer_params(self, optimizer):
        """An optimizer created on the original parameters is pointed at the FSDP shard parameters (replaces the
        reference's `data_ptr` patching, accelerator.py:1690-1744). TP re-sharding maps are applied first."""
        for m in self._models:
            inner = extract_model_from_parallel(m)
            for attr in ("_tp_param_map", "_ep_param_map"):
                tmap = getattr(inner, attr, None) or getattr(m, attr, None)
                if tmap:
                    for group in optimizer.param_groups:
                        group["params"] = [tmap.get(p, p) for p in group["params"]]
        for eng in self._fsdp_engines:
            pmap = eng.param_map()
            for group in optimizer.param_groups:
                group["params"] = [pmap.get(p, p) for p in group["params"]]
            optimizer._acc_fsdp_engine = eng

    def _convert_fp8(self, model):
        from .ops.fp8 import convert_model_to_fp8

        recipe = self.ao_recipe_handler or self.te_recipe_handler or self.fp8_recipe_handler
        convert_model_to_fp8(model, recipe=recipe, backend=self._fp8_backend)
        model._acc_fp8_converted = True

    def prepare_model(self, model: torch.nn.Module, device_placement: Optional[bool] = None, evaluation_mode: bool = False):
        if device_placement is None:
            device_placement = self.device_placement and self.distributed_type != DistributedType.FSDP
        self._models.append(model)
        if self.verify_device_map(model) and self.distributed_type != DistributedType.NO:
            raise ValueError("You can't train a model that has been loaded with `device_map='auto'` in any distributed mode.")
        if self.native_amp and self.distributed_type != DistributedType.FSDP:
            model._original_forward = model.forward
            autocast_context = get_mixed_precision_context_manager(self.native_amp, self.autocast_handler)
            model_forward_func = model.forward.__func__ if hasattr(model.forward, "__func__") else model.forward
            new_forward = autocast_context(model_forward_func)
            if hasattr(model.forward, "__func__"):
                model.forward = MethodType(new_forward, model)
                model.forward = MethodType(convert_outputs_to_fp32(model.forward.__func__), model)
            else:
                model.forward = convert_outputs_to_fp32(new_forward)
        if device_placement and not self.verify_device_map(model):
            model = model.to(self.device)
        if self.parallelism_config is not None and self.parallelism_config.tp_enabled:
            model = self._prepare_tp(model)
        if self.parallelism_config is not None and self.parallelism_config.sp_enabled:
            from .parallel.ulysses import install_ulysses

            if self.distributed_type != DistributedType.FSDP:
                raise ValueError("Ulysses sequence parallelism needs the FSDP2 engine (params are sharded over dp_shard x sp).")
            if install_ulysses(model, self.torch_device_mesh.group("sp")) == 0:
                raise ValueError("Ulysses SP: the model exposes no `attention_impl` hook; wrap the step in "
                                 "`parallel.ulysses.ulysses_sdpa_context` for SDPA-based models.")
        if not evaluation_mode:
            # RcclKwargs.ddp_force: one process with an initialised group still gets the reducer (nranks=1 RCCL)
            force_ddp = (self.rccl_handler.ddp_force and self.num_processes == 1 and self.distributed_type == DistributedType.NO
                         and torch.distributed.is_available() and torch.distributed.is_initialized())
            if self.distributed_type in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU) or force_ddp:
                dp_size = self.parallelism_config.data_parallel_size if self.parallelism_config is not None else self.num_processes
                if any(p.requires_grad for p in model.parameters()) and (force_ddp or (self.num_processes > 1 and dp_size > 1)):
                    kwargs = self.ddp_handler.to_kwargs() if self.ddp_handler is not None else {}
                    from .parallel.ddp import DistributedDataParallel

                    bucket_mb = kwargs.pop("bucket_cap_mb", None)
                    if bucket_mb is None:
                        bucket_mb = self.rccl_handler.ddp_bucket_mb
                    comm_hook = self.ddp_handler.comm_hook if self.ddp_handler is not None else None
                    comm_wrapper = self.ddp_handler.comm_wrapper if self.ddp_handler is not None else None
                    group = None
                    if self.torch_device_mesh is not None and self.parallelism_config.dp_replicate_enabled:
                        group = self.torch_device_mesh.group("dp_replicate")
                    model = DistributedDataParallel(
                        model,
                        process_group=group,
                        bucket_cap_mb=bucket_mb,
                        broadcast_buffers=kwargs.get("broadcast_buffers", True),
                        find_unused_parameters=kwargs.get("find_unused_parameters", False),
                        comm_hook=comm_hook,
                        comm_wrapper=comm_wrapper,
                        comm_state_option=self.ddp_handler.comm_state_option if self.ddp_handler is not None else None,
                        own_communicator=force_ddp,
                    )
                    self._models[-1] = model
            elif self.distributed_type == DistributedType.FSDP:
                model = self._prepare_fsdp(model)
                self._models[-1] = model
        if self.state.dynamo_plugin is not None and self.state.dynamo_plugin.backend != DynamoBackend.NO and not is_compiled_module(model):
            kw = self.state.dynamo_plugin.to_kwargs()
            if self.state.dynamo_plugin.use_regional_compilation:
                model = compile_regions(model, **kw)
            else:
                model = torch.compile(model, **kw)
            self._models[-1] = model
        return model

    def _prepare_tp(self, model):
        """Shard the model over the `tp` mesh dim with its TP plan (parity: reference accelerator.py:1579-1639,
        which defers to transformers' `tp_plan`; here parallel/tensor_parallel.py does the sharding)."""
        if getattr(model, "_tp_group", None) is not None:
            return model
        from .parallel.tensor_parallel import parallelize_module

        handler = self.parallelism_config.tp_handler
        return parallelize_module(
            model, self.torch_device_mesh.group("tp"), sequence_parallel=bool(getattr(handler, "sequence_parallel", False))
        )

    def _prepare_fsdp(self, model):
        from .parallel.fsdp import FullyShardedModule, fully_shard

        if isinstance(model, FullyShardedModule):
            return model
        plugin = self.state.fsdp_plugin
        if self.state.mixed_precision != "no" and plugin.mixed_precision_policy is None:
            plugin.set_mixed_precision(self.state.mixed_precision)
        group = replicate_group = None
        mesh = self.torch_device_mesh
        if mesh is not None:
            group = mesh.group("dp_shard_cp") if self.parallelism_config.fsdp_dim_names else None
            if self.parallelism_config.dp_replicate_enabled:
                replicate_group = mesh.group("dp_replicate")
        elif self.num_processes > 1 and plugin.sharding_strategy in ("NO_SHARD", "HYBRID_SHARD", "HYBRID_SHARD_ZERO2"):
            group, replicate_group = self._fsdp1_strategy_groups(plugin.sharding_strategy)
        init_fn = getattr(model, "init_weights", None)
        init_fn = (lambda m, _f=init_fn: _f(m)) if init_fn is not None else (lambda m: [getattr(c, "reset_parameters", lambda: None)() for c in m.modules()])
        if self.parallelism_config is not None and self.parallelism_config.ep_enabled:
            # Expert parallelism: experts are sharded over the FSDP group by the model itself and stay outside the
            # flat FSDP units (models/moe.py). Old→new parameter map lets a pre-built optimizer follow.
            if not hasattr(model, "enable_expert_parallel"):
                raise ValueError("ep_size > 1 needs a model with `enable_expert_parallel(group)` (e.g. MixtralForCausalLM).")
            old_by_name = dict(model.named_parameters())
            ep_modules = model.enable_expert_parallel(group, device=self.device)
            new_by_name = dict(model.named_parameters())
            model._ep_param_map = {old_by_name[n]: new_by_name[n] for n in old_by_name if new_by_name.get(n) is not old_by_name[n]}
            existing = list(plugin.ignored_modules or []) if not isinstance(plugin.ignored_modules, str) else []
            plugin.ignored_modules = existing + list(ep_modules)
        wrapped = fully_shard(
            model,
            plugin=plugin,
            device=self.device,
            process_group=group,
            replicate_group=replicate_group,
            init_fn=init_fn,
            prefetch_depth=self.rccl_handler.fsdp_prefetch_depth,
            force_sharded=self.rccl_handler.fsdp_force_sharded,
            fp8_all_gather=self._fsdp_fp8_all_gather(),
        )
        self._fsdp_engines.append(wrapped.engine)
        return wrapped

    def _fsdp1_strategy_groups(self, strategy: str):
        """(shard group, replicate group) for the FSDP1 strategies that are not a plain full shard over the world
        (reference accelerator.py:1909-1925 hands `sharding_strategy` to torch FSDP1; `commands/to_fsdp2.py:50-66`
        maps it onto FSDP2): NO_SHARD -> every rank its own shard group (the engine's unsharded path) and one
        replicate all-reduce over the world, i.e. DDP on the FSDP engine; HYBRID_SHARD / HYBRID_SHARD_ZERO2 -> shard
        within a node (LOCAL_WORLD_SIZE ranks over xGMI), replicate across nodes (the HSDP path). Groups are created
        collectively, in the same order on every rank, and cached."""
        cached = getattr(self, "_fsdp1_groups", None)
        if cached is not None and cached[0] == strategy:
            return cached[1], cached[2]
        W, r = self.num_processes, self.process_index
        shard = 1 if strategy == "NO_SHARD" else int(os.environ.get("LOCAL_WORLD_SIZE", W) or W)
        if shard <= 0 or W % shard:
            raise ValueError(f"{strategy}: world size {W} is not a multiple of the node size {shard} (LOCAL_WORLD_SIZE)")
        reps = W // shard
        shard_group = replicate_group = None
        for n in range(reps):  # shard groups: consecutive node-local blocks
            ranks = list(range(n * shard, (n + 1) * shard))
            g = torch.distributed.new_group(ranks) if shard < W else torch.distributed.group.WORLD
            if r in ranks:
                shard_group = g
        if reps > 1:
            for k in range(shard):  # replicate groups: the same local rank on every node
                ranks = list(range(k, W, shard))
                g = torch.distributed.new_group(ranks) if reps < W else torch.distributed.group.WORLD
                if r in ranks:
                    replicate_group = g
        self._fsdp1_groups = (strategy, shard_group, replicate_group)
        return shard_group, replicate_group

    def _fsdp_fp8_all_gather(self) -> bool:
        """torchao-style fp8 all-gather of the FSDP shards (reference examples/torch_native_parallelism/fsdp2_fp8.py:69-75):
        on with the AO (dynamic scaling) fp8 backend when `enable_fsdp_float8_all_gather` is set."""
        if self.state.mixed_precision != "fp8" or self._fp8_backend != "AO" or self.ao_recipe_handler is None:
            return False
        return bool(self.ao_recipe_handler.enable_fsdp_float8_all_gather)

    def prepare_data_loader(self, data_loader: torch.utils.data.DataLoader, device_placement=None, slice_fn_for_dispatch=None):
        if getattr(data_loader, "_is_accelerate_prepared", False):
            if data_loader not in self._dataloaders:
                self._dataloaders.append(data_loader)
            return data_loader
        if device_placement is None:
            device_placement = self.device_placement
        prepared = prepare_data_loader(
            data_loader,
            self.device,
            num_processes=self.num_processes,
            process_index=self.process_index,
            split_batches=self.split_batches,
            put_on_device=device_placement,
            rng_types=self.rng_types.copy() if self.rng_types else None,
            dispatch_batches=self.dispatch_batches,
            even_batches=self.even_batches,
            slice_fn_for_dispatch=slice_fn_for_dispatch,
            use_seedable_sampler=self.use_seedable_sampler,
            data_seed=self.dataloader_config.data_seed,
            non_blocking=self.non_blocking,
            use_stateful_dataloader=self.use_stateful_dataloader,
            torch_device_mesh=self.torch_device_mesh,
            prefetch_to_device=self.dataloader_config.prefetch_to_device,
        )
        self._dataloaders.append(prepared)
        return prepared

    def prepare_optimizer(self, optimizer: torch.optim.Optimizer, device_placement=None):
        if getattr(optimizer, "_is_accelerate_prepared", False):
            if optimizer not in self._optimizers:
                self._optimizers.append(optimizer)
            return optimizer
        if device_placement is None:
            device_placement = self.device_placement
        if self.distributed_type == DistributedType.FSDP:
            device_placement = False
        optimizer = AcceleratedOptimizer(optimizer, device_placement=device_placement, scaler=self.scaler)
        eng = getattr(optimizer.optimizer, "_acc_fsdp_engine", None)
        if eng is not None:
            optimizer.optimizer._accelerate_post_step = lambda _o=optimizer, _e=eng: _e.on_optimizer_step(
                bool(getattr(_o.optimizer, "_acc_last_step_fused", False))
            )
            if self.rccl_handler.fsdp_optimizer_overlap:
                optimizer.enable_overlap(eng)
        self._optimizers.append(optimizer)
        return optimizer

    def prepare_scheduler(self, scheduler):
        """Wrap an LR scheduler so it steps with its (prepared) optimizer; an already-wrapped one is only registered."""
        if not getattr(scheduler, "_is_accelerate_prepared", False):
            inner = getattr(scheduler, "optimizer", None)
            owner = next((o for o in self._optimizers if o.optimizer == inner), self._optimizers)
            scheduler = AcceleratedScheduler(scheduler, owner, step_with_optimizer=self.step_scheduler_with_optimizer,
                                             split_batches=self.split_batches)
        if scheduler not in self._schedulers:
            self._schedulers.append(scheduler)
        return scheduler

    # ============================================================================== training step helpers
    def backward(self, loss, **kwargs):
        learning_rate = kwargs.pop("learning_rate", None)
        step = self._backward_calls
        self._backward_calls += 1
        if self._fault_injector is not None:
            loss = self._fault_injector.before_backward(step, loss)
        loss = loss / self.gradient_accumulation_steps
        if self.scaler is not None:
            self.scaler.scale(loss).backward(**kwargs)
        elif learning_rate is not None and self.has_lomo_optimizer:
            self.lomo_backward(loss, learning_rate)
        else:
            loss.backward(**kwargs)
        self.heartbeat("backward")
        interval = self.rccl_handler.collective_check_interval
        if self.state.debug and self.use_distributed and interval and self._backward_calls % interval == 0:
            check_collective_sequence()

    def heartbeat(self, tag: str = "step"):
        """Tell the step watchdog (RcclKwargs.watchdog_timeout / ACCELERATE_WATCHDOG_TIMEOUT) this rank progressed."""
        if self._watchdog is not None:
            self._watchdog.beat(tag)

    def set_trigger(self):
        self.flag_tensor = torch.tensor(1, device=self.device)

    def check_trigger(self):
        if self.flag_tensor is None:
            self.flag_tensor = torch.tensor(0, device=self.device)
        flag_tensor = self.reduce(self.flag_tensor, reduction="sum")
        if flag_tensor.item() >= 1:
            self.flag_tensor = torch.tensor(0, device=self.device)
            return True
        return False

    def unscale_gradients(self, optimizer=None):
        if self.native_amp and self.mixed_precision == "fp16" and self.scaler is not None:
            if optimizer is None:
                optimizer = self._optimizers
            elif not isinstance(optimizer, (tuple, list)):
                optimizer = [optimizer]
            for opt in optimizer:
                while isinstance(opt, AcceleratedOptimizer):
                    opt = opt.optimizer
                self.scaler.unscale_(opt)

    def _fsdp_model_for(self, parameters):
        from .parallel.fsdp import FullyShardedModule

        ids = {id(p) for p in parameters}
        for m in self._models:
            if isinstance(m, FullyShardedModule):
                if any(id(p) in ids for p in m.parameters()):
                    return m
        return None

    def clip_grad_norm_(self, parameters, max_norm, norm_type=2):
        """Clip the global gradient norm. GPU: HIP multi-tensor L2 norm + device-side scaling (no host sync); FSDP:
        norm over the local shards + one all-reduce. Returns the total norm (0-d tensor)."""
        if isinstance(parameters, torch.Tensor):
            parameters = [parameters]
        parameters = [p for p in parameters]
        if self.distributed_type == DistributedType.FSDP:
            self.unscale_gradients()
            m = self._fsdp_model_for(parameters)
            if m is not None:
                return m.clip_grad_norm_(max_norm, norm_type)
        self.unscale_gradients()
        grads_params = [p for p in parameters if p.grad is not None]
        if _any_dtensor(grads_params):
            return self._clip_grad_norm_dtensor(grads_params, float(max_norm), float(norm_type))
        tp_sharded = [p for p in grads_params if getattr(getattr(p, "_tp_spec", None), "size", 1) > 1]
        if tp_sharded:
            return self._clip_grad_norm_tp(grads_params, tp_sharded, float(max_norm), float(norm_type))
        if grads_params and grads_params[0].grad.is_cuda and float(norm_type) == 2.0:
            from .ops.multi_tensor import clip_grads_by_total_sq, grad_sq_norm

            total = grad_sq_norm(grads_params)
            clip_grads_by_total_sq(grads_params, total, float(max_norm))
            return total.sqrt().reshape(())
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm, norm_type=norm_type)

    @staticmethod
    def _clip_grad_norm_tp(grads_params, sharded, max_norm, norm_type=2.0):
        """Tensor parallel: each rank holds 1/tp of a sharded parameter's gradient, so those squares are summed over
        the tp group, while replicated parameters (norms, biases of rowwise layers, ...) hold the whole gradient on
        every rank and count once. (The plain local norm under-counts the sharded part by 1/tp.) norm_type inf: the
        sharded part's max is MAX-reduced over tp; other finite orders are not supported here."""
        import torch.distributed as dist

        group = sharded[0]._tp_spec.group
        ids = {id(p) for p in sharded}
        rest = [p for p in grads_params if id(p) not in ids]
        dev = grads_params[0].grad.device
        native = grads_params[0].grad.is_cuda
        if norm_type == float("inf"):
            def amax(ps):
                return torch.stack([p.grad.detach().abs().max().float() for p in ps]).max().reshape(1) if ps else torch.zeros(1, device=dev)

            total = amax(sharded)
            dist.all_reduce(total, op=dist.ReduceOp.MAX, group=group)
            total = torch.maximum(total, amax(rest))
            coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
            for p in grads_params:
                p.grad.mul_(coef.to(p.grad.dtype))
            return total.reshape(())
        if norm_type != 2.0:
            raise NotImplementedError(f"clip_grad_norm_ with tensor-parallel parameters supports norm_type 2 and inf, not {norm_type}")

        def sq(ps):
            if not ps:
                return torch.zeros(1, dtype=torch.float32, device=dev)
            if native:
                from .ops.multi_tensor import grad_sq_norm

                return grad_sq_norm(ps)
            return sum(p.grad.detach().float().pow(2).sum() for p in ps).reshape(1)

        total = sq(sharded)
        dist.all_reduce(total, group=group)
        total = total + sq(rest)
        if native:
            from .ops.multi_tensor import clip_grads_by_total_sq

            clip_grads_by_total_sq(grads_params, total, max_norm)
        else:
            coef = (max_norm / (total.sqrt() + 1e-6)).clamp(max=1.0)
            for p in grads_params:
                p.grad.mul_(coef.to(p.grad.dtype))
        return total.sqrt().reshape(())

    @staticmethod
    @torch.no_grad()
    def _clip_grad_norm_dtensor(grads_params, max_norm, norm_type=2.0):
        """Parameters already sharded as DTensors (transformers `tp_plan="auto"` / torch `parallelize_module`): the
        reference clips with DTensor-aware `torch.nn.utils.clip_grad_norm_` (accelerator.py:2943-2953). Here the
        squares (or maxima) of Shard-placed gradients are reduced over their mesh, Replicate-placed and plain ones
        count once, Partial ones are first reduced to Replicate; the scale is applied to the local shards."""
        import torch.distributed as dist
        from torch.distributed.tensor import DTensor, Replicate

        inf = norm_type == float("inf")
        if not inf and norm_type != 2.0:
            raise NotImplementedError(f"clip_grad_norm_ on DTensor parameters supports norm_type 2 and inf, not {norm_type}")
        dev = grads_params[0].grad.device
        rest_part = torch.zeros(1, dtype=torch.float32, device=dev)
        # one partial per (mesh, set of sharded mesh dims): a gradient sharded on dims {0, 1} of a 2-D mesh is summed
        # over both groups, one sharded on dim 1 only over that group (summing it over dim 0 too would count it once
        # per dim-0 replica)
        partials = {}
        for p in grads_params:
            g = p.grad
            if isinstance(g, DTensor):
                if any(pl.is_partial() for pl in g.placements):
                    g = p.grad = g.redistribute(placements=[Replicate() if pl.is_partial() else pl for pl in g.placements])
                local = g.to_local().detach().float()
                v = local.abs().max().reshape(1) if inf and local.numel() else local.pow(2).sum().reshape(1)
                dims = tuple(d for d, pl in enumerate(g.placements) if pl.is_shard())
                if dims:
                    key = (id(g.device_mesh), dims)
                    if key not in partials:
                        partials[key] = [g.device_mesh, dims, torch.zeros(1, dtype=torch.float32, device=dev)]
                    acc = partials[key]
                    acc[2] = torch.maximum(acc[2], v) if inf else acc[2] + v
                    continue
            else:
                local = g.detach().float()
                v = local.abs().max().reshape(1) if inf and local.numel() else local.pow(2).sum().reshape(1)
            rest_part = torch.maximum(rest_part, v) if inf else rest_part + v
        total = rest_part
        for mesh, dims, part in partials.values():
            for d in dims:
                dist.all_reduce(part, op=dist.ReduceOp.MAX if inf else dist.ReduceOp.SUM, group=mesh.get_group(d))
            total = torch.maximum(total, part) if inf else total + part
        if not inf:
            total = total.sqrt()
        coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
        for p in grads_params:
            g = p.grad.to_local() if isinstance(p.grad, DTensor) else p.grad
            g.mul_(coef.to(g.dtype))
        return total.reshape(())

    def clip_grad_value_(self, parameters, clip_value):
        if self.distributed_type in (DistributedType.FSDP,):
            raise Exception("DeepSpeed and FSDP  do not support `clip_grad_value_`. Use `clip_grad_norm_` instead.")
        self.unscale_gradients()
        torch.nn.utils.clip_grad_value_(parameters, clip_value)

    # ============================================================================== collectives
    def gather(self, tensor):
        return gather(tensor)

    def gather_for_metrics(self, input_data, use_gather_object=False):
        """Gather `input_data` from every process for metric computation. On the last batch of a loader that
        `even_batches` padded, the duplicated samples are dropped (`GradientState.remainder` real samples are kept).
        Anything that is not purely tensors goes through `gather_object` (a flat list)."""
        as_objects = use_gather_object or not _only_tensors(input_data)
        data = gather_object(input_data) if as_objects else self.gather(input_data)
        if not self.gradient_state.end_of_dataloader:
            return data
        keep = self.gradient_state.remainder
        if keep == -1:
            logger.info("gather_for_metrics: the loader has no length, so padding duplicates in its last batch "
                        "cannot be dropped here; returning everything gathered")
        if keep is None or keep <= 0:
            return data
        return data[:keep] if as_objects else recursively_apply(lambda t: t[:keep], data)

    def reduce(self, tensor, reduction="sum", scale=1.0):
        return reduce(tensor, reduction, scale)

    def pad_across_processes(self, tensor, dim=0, pad_index=0, pad_first=False):
        return pad_across_processes(tensor, dim=dim, pad_index=pad_index, pad_first=pad_first)

    def unwrap_model(self, model, keep_fp32_wrapper: bool = True, keep_torch_compile: bool = True):
        return extract_model_from_parallel(model, keep_fp32_wrapper, keep_torch_compile)

    # ============================================================================== trackers
    def init_trackers(self, project_name: str, config: Optional[dict] = None, init_kwargs: Optional[dict] = {}):
        for tracker in self.log_with:
            if issubclass(type(tracker), GeneralTracker):
                self.trackers.append(tracker)
            else:
                tracker_init = LOGGER_TYPE_TO_CLASS[str(tracker)]
                if tracker_init.requires_logging_directory:
                    self.trackers.append(tracker_init(project_name, self.logging_dir, **init_kwargs.get(str(tracker), {})))
                else:
                    self.trackers.append(tracker_init(project_name, **init_kwargs.get(str(tracker), {})))
        for tracker in self.trackers:
            if self.is_main_process or not getattr(tracker, "main_process_only", True):
                tracker.start()
        if config is not None:
            for tracker in self.trackers:
                if self.is_main_process or not getattr(tracker, "main_process_only", True):
                    tracker.store_init_configuration(config)

    def get_tracker(self, name: str, unwrap: bool = False):
        if len(self.trackers) > 0:
            for tracker in self.trackers:
                if tracker.name == name:
                    return tracker.tracker if unwrap else tracker
            raise ValueError(f"{name} is not an available tracker stored inside the `Accelerator`.")
        return GeneralTracker(_blank=True)

    def log(self, values: dict, step: Optional[int] = None, log_kwargs: Optional[dict] = {}):
        for tracker in self.trackers:
            if self.is_main_process or not getattr(tracker, "main_process_only", True):
                tracker.log(values, step=step, **log_kwargs.get(tracker.name, {}))

    def end_training(self):
        from .utils.async_checkpoint import wait_pending_saves

        wait_pending_saves()
        if getattr(self, "_watchdog", None) is not None:
            self._watchdog.stop()
            self._watchdog = None
        for tracker in self.trackers:
            if self.is_main_process or not getattr(tracker, "main_process_only", True):
                tracker.finish()
        self.state.destroy_process_group()

    # ============================================================================== saving
    def save(self, obj, f, safe_serialization=False):
        save(obj, f, save_on_each_node=self.project_configuration.save_on_each_node, safe_serialization=safe_serialization)

    def save_model(self, model: torch.nn.Module, save_directory: Union[str, os.PathLike], max_shard_size: Union[int, str] = "10GB", safe_serialization: bool = True):
        """Save the full (unwrapped) weights, split into shards with an index file when above `max_shard_size`."""
        if os.path.isfile(save_directory):
            logger.error(f"Provided path ({save_directory}) should be a directory, not a file")
            return
        state_dict = self.get_state_dict(model)
        if not self.is_main_process:
            self.wait_for_everyone()
            return
        os.makedirs(save_directory, exist_ok=True)
        if safe_serialization:
            state_dict = clean_state_dict_for_safetensors(state_dict)
        weights_name = SAFE_WEIGHTS_NAME if safe_serialization else WEIGHTS_NAME
        filename_pattern = SAFE_WEIGHTS_PATTERN_NAME if safe_serialization else WEIGHTS_PATTERN_NAME
        max_bytes = convert_file_size_to_int(max_shard_size)
        shards, cur, cur_size = [], OrderedDict(), 0
        for k, v in state_dict.items():
            nbytes = v.numel() * v.element_size()
            if cur and cur_size + nbytes > max_bytes:
                shards.append(cur)
                cur, cur_size = OrderedDict(), 0
            cur[k] = v
            cur_size += nbytes
        if cur:
            shards.append(cur)
        # clean up stale weight files with the same prefix
        for filename in os.listdir(save_directory):
            full = os.path.join(save_directory, filename)
            base = weights_name.split(".")[0]
            if filename.startswith(base) and os.path.isfile(full) and filename.endswith(weights_name.split(".")[-1]):
                os.remove(full)
        index = None
        if len(shards) == 1:
            names = [weights_name]
        else:
            n = len(shards)
            names = [filename_pattern.format(suffix=f"-{i + 1:05d}-of-{n:05d}") for i in range(n)]
            weight_map = {k: names[i] for i, s in enumerate(shards) for k in s}
            index = {"metadata": {"total_size": sum(v.numel() * v.element_size() for v in state_dict.values())}, "weight_map": weight_map}
        for shard, name in zip(shards, names):
            path = os.path.join(save_directory, name)
            if safe_serialization:
                from safetensors.torch import save_file

                save_file({k: v.contiguous() for k, v in shard.items()}, path, metadata={"format": "pt"})
            else:
                torch.save(shard, path)
        if index is not None:
            idx_name = SAFE_WEIGHTS_INDEX_NAME if safe_serialization else WEIGHTS_INDEX_NAME
            with open(os.path.join(save_directory, idx_name), "w", encoding="utf-8") as f:
                f.write(json.dumps(index, indent=2, sort_keys=True) + "\n")
            logger.info(f"The model is bigger than the maximum size per checkpoint ({max_shard_size}) and is going to be split in {len(shards)} checkpoint shards.")
        self.wait_for_everyone()

    def register_save_state_pre_hook(self, hook: Callable[..., None]) -> hooks.RemovableHandle:
        handle = hooks.RemovableHandle(self._save_model_state_pre_hook)
        self._save_model_state_pre_hook[handle.id] = hook
        return handle

    def register_load_state_pre_hook(self, hook: Callable[..., None]) -> hooks.RemovableHandle:
        handle = hooks.RemovableHandle(self._load_model_state_pre_hook)
        self._load_model_state_pre_hook[handle.id] = hook
        return handle

    # --- checkpoints: automatic naming / rotation lives in `_CheckpointRotation`, file names in checkpointing.py
    def _split_for_checkpoint(self):
        """(fsdp models, other models, engine-managed optimizers, other optimizers): FSDP-wrapped models and the
        optimizers over their shard parameters are saved by utils/fsdp_utils.py (per-rank shards or a gathered full
        state), everything else by checkpointing.py."""
        from .parallel.fsdp import FullyShardedModule

        fsdp = [(i, m) for i, m in enumerate(self._models) if isinstance(m, FullyShardedModule)]
        plain = [m for m in self._models if not isinstance(m, FullyShardedModule)]
        eng_opts, plain_opts = [], []
        for i, opt in enumerate(self._optimizers):
            managed = fsdp and getattr(opt.optimizer, "_acc_fsdp_engine", None) is not None
            (eng_opts if managed else plain_opts).append((i, opt) if managed else opt)
        return fsdp, plain, eng_opts, plain_opts

    def save_state(self, output_dir: str = None, safe_serialization: bool = True, **save_model_func_kwargs):
        """Save model(s), optimizer(s), scheduler(s), dataloader positions, scaler, RNG and registered custom states.
        With `ProjectConfiguration(automatic_checkpoint_naming=True)` the state goes to
        `<project_dir>/checkpoints/checkpoint_<iteration>` and the oldest checkpoints beyond `total_limit` are pruned."""
        from .utils.async_checkpoint import wait_pending_saves
        from .utils.fsdp_utils import save_fsdp_model, save_fsdp_optimizer

        wait_pending_saves()  # the previous non-blocking save's files are complete before rotation / overwrite
        rot = _CheckpointRotation(self.project_configuration)
        if rot.enabled:
            if self.is_main_process:
                rot.prune_for_one_more()
            output_dir = rot.next_dir(self.save_iteration)
            self.wait_for_everyone()
        os.makedirs(output_dir, exist_ok=True)
        logger.info(f"Saving current state to {output_dir}")
        fsdp, plain, eng_opts, plain_opts = self._split_for_checkpoint()
        for i, model in fsdp:
            save_fsdp_model(self.state.fsdp_plugin, self, model, output_dir, i)
        for i, opt in eng_opts:
            save_fsdp_optimizer(self.state.fsdp_plugin, self, opt, fsdp[0][1], output_dir, i)
        weights = [self.get_state_dict(m, unwrap=False) for m in plain]
        for hook in self._save_model_state_pre_hook.values():
            hook(self._models, weights, output_dir)
        node_kw = {"save_on_each_node": self.project_configuration.save_on_each_node}
        location = save_accelerator_state(output_dir, weights, plain_opts, self._schedulers, self._dataloaders,
                                          self.state.process_index, self.step, self.scaler,
                                          safe_serialization=safe_serialization, **node_kw)
        for i, obj in enumerate(self._custom_objects):
            save_custom_state(obj, output_dir, i, **node_kw)
        self.project_configuration.iteration += 1
        return location

    def load_state(self, input_dir: str = None, load_kwargs: dict | None = None, **load_model_func_kwargs):
        """Restore what `save_state` wrote (the newest automatic checkpoint when `input_dir` is None)."""
        from .utils.async_checkpoint import wait_pending_saves
        from .utils.fsdp_utils import load_fsdp_model, load_fsdp_optimizer

        wait_pending_saves()  # a non-blocking save of this process may still be writing the files
        self.wait_for_everyone()
        if input_dir is not None:
            input_dir = os.path.expanduser(input_dir)
            if not os.path.isdir(input_dir):
                raise ValueError(f"Tried to find {input_dir} but folder does not exist")
        else:
            rot = _CheckpointRotation(self.project_configuration)
            if not rot.enabled:
                raise ValueError("No input_dir provided and automatic checkpoint naming is disabled.")
            input_dir = rot.latest()
        logger.info(f"Loading states from {input_dir}")
        fsdp, plain, eng_opts, plain_opts = self._split_for_checkpoint()
        for i, model in fsdp:
            load_fsdp_model(self.state.fsdp_plugin, self, model, input_dir, i)
        for i, opt in eng_opts:
            load_fsdp_optimizer(self.state.fsdp_plugin, self, opt, fsdp[0][1], input_dir, i)
        for hook in self._load_model_state_pre_hook.values():
            hook(plain, input_dir)
        map_location = load_model_func_kwargs.pop("map_location", None)
        if map_location is None:  # multi-GPU: optimizer state straight onto the device
            map_location = "on_device" if self.num_processes > 1 and self.device.type == "cuda" else "cpu"
        overrides = load_accelerator_state(input_dir, [self.unwrap_model(m) for m in plain], plain_opts, self._schedulers,
                                           self._dataloaders, self.state.process_index, self.scaler, map_location,
                                           load_kwargs, **load_model_func_kwargs)
        self.step = overrides.get("step", self.step)
        found = _CheckpointRotation.custom_state_files(input_dir)
        if len(found) != len(self._custom_objects):
            raise RuntimeError(
                f"Number of custom checkpoints in folder {input_dir} does not match the number of registered objects:\n"
                f"\tFound checkpoints: {len(found)}\n\tRegistered objects: {len(self._custom_objects)}\n"
                "Load checkpoints only from folders written with the same set of registered objects, or keep other "
                "files named `custom_checkpoint_<k>.pkl` out of that folder.")
        logger.info(f"Loading in {len(found)} custom states")
        for index, obj in enumerate(self._custom_objects):
            load_custom_state(obj, input_dir, index)

    def free_memory(self, *objects):
        self._schedulers = []
        self._optimizers = []
        self._models = []
        self._dataloaders = []
        self._fsdp_engines = []
        self.step = 0
        release_memory(*objects)
        return [None for _ in objects] if objects else None

    def clear(self, *objects):
        return self.free_memory(*objects)

    def get_state_dict(self, model, unwrap=True):
        """Full state dict on the CPU (FSDP: gathered unit by unit, fp32 master weights)."""
        from .parallel.fsdp import FullyShardedModule

        if isinstance(model, FullyShardedModule):
            sd = model.engine.full_state_dict(rank0_only=False)
            return self._gather_tp(sd, model.engine.model)
        if unwrap:
            model = self.unwrap_model(model)
        state_dict = model.state_dict()
        sd = OrderedDict((k, v.detach().cpu() if isinstance(v, torch.Tensor) else v) for k, v in state_dict.items())
        return self._gather_tp(sd, model)

    @staticmethod
    def _gather_tp(sd, model):
        if getattr(model, "_tp_group", None) is None:
            return sd
        from .parallel.tensor_parallel import gather_tp_state_dict

        return OrderedDict(gather_tp_state_dict(sd, model))

    def register_for_checkpointing(self, *objects):
        invalid_objects = []
        for obj in objects:
            if not hasattr(obj, "state_dict") or not hasattr(obj, "load_state_dict"):
                invalid_objects.append(obj)
        if len(invalid_objects) > 0:
            err = "All `objects` must include a `state_dict` and `load_state_dict` function to be stored. The following inputs are invalid:"
            for index, obj in enumerate(invalid_objects):
                err += f"\n\t- Item at index {index}, `{type(obj).__name__}`"
            raise ValueError(err)
        self._custom_objects.extend(objects)

    # ============================================================================== misc contexts
    @contextlib.contextmanager
    def maybe_context_parallel(self, buffers=None, buffer_seq_dims=None, no_restore_buffers=None):
        """Shard `buffers` along their sequence dims across the `cp` group and route attention through ring attention
        (parallel/context_parallel.py) for the duration of the block."""
        if self.parallelism_config is None or not self.parallelism_config.cp_enabled:
            yield
            return
        from .parallel.context_parallel import context_parallel

        with context_parallel(
            self.torch_device_mesh,
            self._models,
            buffers or [],
            buffer_seq_dims or [],
            no_restore_buffers or set(),
            strategy=self.parallelism_config.cp_handler.cp_comm_strategy,
        ):
            yield

    @contextlib.contextmanager
    def autocast(self, autocast_handler: AutocastKwargs = None):
        if autocast_handler is None:
            autocast_handler = self.autocast_handler
        autocast_context = get_mixed_precision_context_manager(self.native_amp, autocast_handler)
        autocast_context.__enter__()
        yield
        autocast_context.__exit__(*__import__("sys").exc_info())

    @contextlib.contextmanager
    def profile(self, profile_handler: ProfileKwargs | None = None):
        profile_handler = profile_handler or self.profile_handler or ProfileKwargs()
        with profile_handler.build() as profiler:
            yield profiler
        if profile_handler.output_trace_dir is None:
            return
        os.makedirs(profile_handler.output_trace_dir, exist_ok=True)
        profiler.export_chrome_trace(
            os.path.join(profile_handler.output_trace_dir, PROFILE_PATTERN_NAME.format(suffix=self.process_index))
        )
        self.wait_for_everyone()

    def skip_first_batches(self, dataloader, num_batches: int = 0):
        return skip_first_batches(dataloader, num_batches=num_batches)

    def __deepcopy__(self, memo):
        logger.info("Deep copying the `Accelerator` object, note that this will point to the same original object.")
        return self

    def verify_device_map(self, model: torch.nn.Module) -> bool:
        for m in model.modules():
            if hasattr(m, "hf_device_map") and len(m.hf_device_map) > 1:
                return True
        return False

    def lomo_backward(self, loss: torch.Tensor, learning_rate: float) -> None:
        raise NotImplementedError("LOMO optimizers are not available in this environment.")
