"""The remainder of the reference's `accelerate.utils` surface (`/root/reference/src/accelerate/utils/__init__.py`),
mapped onto this stack.

* fp8 back-end helpers (TransformerEngine / torchao names) → the native MX-MFMA fp8 path in `ops/fp8.py`.
* FSDP2 helpers (`fsdp2_prepare_model`, `fsdp2_load_full_state_dict`, ...) → the native engine in `parallel/fsdp.py`.
* DeepSpeed / Megatron-LM / bitsandbytes / XLA / SageMaker glue: those libraries are not part of the MI355X stack
  (SURVEY §7.5). The names exist so imports keep working; using them raises with the native alternative.
* availability probes report the truth for this environment.
"""

from __future__ import annotations

import functools
import importlib.util
import os
from contextlib import contextmanager
from typing import Any, Callable, Optional

import torch
import torch.nn as nn

from .constants import SAFE_WEIGHTS_NAME, WEIGHTS_NAME

# ------------------------------------------------------------------------------------------------ constants
SAFE_WEIGHTS_PATTERN_NAME = "model{suffix}.safetensors"
WEIGHTS_PATTERN_NAME = "pytorch_model{suffix}.bin"
TORCH_DISTRIBUTED_OPERATION_TYPES = ["MULTI_CPU", "MULTI_GPU", "FSDP", "DEEPSPEED", "MEGATRON_LM"]
MITA_PROFILING_AVAILABLE_PYTORCH_VERSION = "2.1.0"
XPU_PROFILING_AVAILABLE_PYTORCH_VERSION = "2.4.0"


def _has(mod: str) -> bool:
    return importlib.util.find_spec(mod) is not None


# ------------------------------------------------------------------------------------------------ availability
# Probes of optional libraries report the truth for this environment; probes of other vendors' devices / libraries
# (NVML, Moore Threads MUSA, Tecorigin SDAA, Intel XCCL, Habana, bitsandbytes, SageMaker) are constant False here.
_PROBED_MODULES = {
    "is_boto3_available": "boto3", "is_matplotlib_available": "matplotlib", "is_pytest_available": "pytest",
    "is_torchvision_available": "torchvision", "is_torchdata_available": "torchdata",
    "is_schedulefree_available": "schedulefree", "is_lomo_available": "lomo_optim",
    "is_import_timer_available": "import_timer",
    "is_triton_available": "triton",  # reported, never dispatched to
}
_NEVER_AVAILABLE = (
    "is_pynvml_available", "is_sagemaker_available", "is_musa_available", "is_sdaa_available", "is_xccl_available",
    "is_habana_gaudi1", "is_4bit_bnb_available", "is_8bit_bnb_available", "is_bitsandbytes_multi_backend_available",
)


def _make_probe(name: str, module: Optional[str]):
    def probe(*_args, **_kwargs):
        return module is not None and _has(module)

    probe.__name__ = probe.__qualname__ = name
    return probe


for _name, _module in list(_PROBED_MODULES.items()) + [(n, None) for n in _NEVER_AVAILABLE]:
    globals()[_name] = _make_probe(_name, _module)


def is_transformer_engine_mxfp8_available():
    """MX-fp8 block scaling is native on gfx950 (ops/fp8.py), no TransformerEngine needed."""
    from .environment import check_fp8_capability

    return check_fp8_capability()


def is_weights_only_available():
    return True


# ------------------------------------------------------------------------------------------------ env checks
def check_cuda_fp8_capability():
    """Name kept from the reference; on this stack: gfx950 (CDNA4) fp8 MFMA support."""
    from .environment import check_fp8_capability

    return check_fp8_capability()


def check_cuda_p2p_ib_support():
    """xGMI peer-to-peer is always available between MI355X GPUs of a node."""
    return True


def get_current_device_type():
    from .environment import get_current_device_type as f

    return f()


# ------------------------------------------------------------------------------------------------ decorators
def _requires(name: str, alt: str):
    def deco(func):
        @functools.wraps(func)
        def wrapper(*a, **k):
            raise NotImplementedError(f"`{func.__name__}` needs {name}, which is not part of the MI355X stack. {alt}")

        return wrapper

    return deco


def deepspeed_required(func):
    return _requires("DeepSpeed", "Use FullyShardedDataParallelPlugin (ZeRO-3 = FSDP2 full shard).")(func)


def torchao_required(func):
    @functools.wraps(func)
    def wrapper(*a, **k):
        return func(*a, **k)  # torchao's role is played by ops/fp8.py

    return wrapper


# ------------------------------------------------------------------------------------------------ fp8 back-end names
def convert_model_to_fp8_ao(model: nn.Module, config=None, module_filter_func: Optional[Callable] = None):
    from ..ops.fp8 import convert_model_to_fp8

    return convert_model_to_fp8(model, recipe=config, backend="AO", module_filter_func=module_filter_func)


def convert_model(model: nn.Module, to_transformer_engine: bool = True, _convert_linear: bool = True, _convert_ln: bool = True):
    """TransformerEngine module swap → native Fp8Linear swap (layer norms stay our fused RMSNorm)."""
    if to_transformer_engine and _convert_linear:
        from ..ops.fp8 import convert_model_to_fp8

        convert_model_to_fp8(model, backend="TE")
    return model


def has_transformer_engine_layers(model: nn.Module) -> bool:
    from ..ops.fp8 import has_fp8_layers

    return has_fp8_layers(model)


def has_ao_layers(model: nn.Module) -> bool:
    from ..ops.fp8 import has_fp8_layers

    return has_fp8_layers(model)


def filter_first_and_last_linear_layers(module: nn.Module, fqn: str) -> bool:
    from ..ops.fp8 import filter_first_and_last_linear_layers as f

    return f(module, fqn)


def apply_fp8_autowrap(model, fp8_recipe_handler=None):
    """TE wraps `forward` in `fp8_autocast`; our Fp8Linear layers are always-on, so this only converts."""
    from ..ops.fp8 import convert_model_to_fp8, has_fp8_layers

    if not has_fp8_layers(model):
        convert_model_to_fp8(model, recipe=fp8_recipe_handler, backend="TE")
    return model


def contextual_fp8_autocast(model_forward, fp8_recipe, use_during_eval: bool = False):
    """Disable fp8 in eval mode unless `use_during_eval` (reference semantics)."""

    @functools.wraps(model_forward)
    def forward(self, *args, **kwargs):
        from ..ops import fp8 as f8

        enabled = use_during_eval or self.training
        with f8.fp8_enabled(enabled):
            return model_forward(self, *args, **kwargs)

    forward.__wrapped__ = model_forward
    return forward


# ------------------------------------------------------------------------------------------------ FSDP2 helper names
def fsdp2_prepare_model(accelerator, model: nn.Module) -> nn.Module:
    return accelerator._prepare_fsdp(model)


def fsdp2_load_full_state_dict(accelerator, model: nn.Module, full_sd: dict, cpu_offload: bool = False):
    """Rank 0's full state dict → every rank's shards (the engine slices locally; no per-param broadcast)."""
    from ..parallel.fsdp import FullyShardedModule

    if isinstance(model, FullyShardedModule):
        return model.engine.load_full_state_dict(full_sd)
    return model.load_state_dict(full_sd)


def fsdp2_switch_optimizer_parameters(optimizer, mapping: dict):
    """Point an optimizer created on unsharded params at the sharded ones (`mapping`: old → new)."""
    for group in optimizer.param_groups:
        group["params"] = [mapping.get(p, p) for p in group["params"]]
    return optimizer


def fsdp2_apply_ac(accelerator, model: nn.Module):
    from ..parallel.fsdp import apply_activation_checkpointing

    return apply_activation_checkpointing(model, accelerator.state.fsdp_plugin)


def fsdp2_canonicalize_names(named_params: dict) -> dict:
    """Drop wrapper prefixes (`_orig_mod.`, `_checkpoint_wrapped_module.`, `module.`) from parameter names."""
    out = {}
    for k, v in named_params.items():
        for pre in ("_orig_mod.", "_checkpoint_wrapped_module.", "_fsdp_wrapped_module."):
            k = k.replace(pre, "")
        out[k] = v
    return out


def get_fsdp2_grad_scaler(**kwargs):
    """bf16/fp32 need no scaler; fp16 uses torch's GradScaler over the fp32 grad shards (finite-check is global)."""
    return torch.amp.GradScaler("cuda", **kwargs)


def enable_fsdp_ram_efficient_loading():
    os.environ["FSDP_CPU_RAM_EFFICIENT_LOADING"] = "True"


def disable_fsdp_ram_efficient_loading():
    os.environ["FSDP_CPU_RAM_EFFICIENT_LOADING"] = "False"


def model_has_dtensor(model: nn.Module) -> bool:
    from torch.distributed.tensor import DTensor

    return any(isinstance(p, DTensor) for p in model.parameters())


# ------------------------------------------------------------------------------------------------ tied weights
from .device_map import find_tied_parameters  # noqa: E402,F401
from .placement import retie_parameters  # noqa: E402,F401


def check_tied_parameters_in_config(model: nn.Module) -> bool:
    cfg = getattr(model, "config", None)
    return bool(getattr(cfg, "tie_word_embeddings", False) or getattr(cfg, "tie_encoder_decoder", False))


def check_tied_parameters_on_same_device(tied_params, device_map):
    import logging

    for group in tied_params:
        devices = set()
        for name in group:
            parts = name.split(".")
            for i in range(len(parts), -1, -1):
                key = ".".join(parts[:i])
                if key in device_map:
                    devices.add(device_map[key])
                    break
        if len(devices) > 1:
            logging.getLogger(__name__).warning(f"Tied parameters are on different devices: {group} -> {devices}")


def ensure_weights_retied(param_init_fn, model: nn.Module, device):
    tied = find_tied_parameters(model)
    if not tied:
        return param_init_fn

    @functools.wraps(param_init_fn)
    def wrapper(module):
        out = param_init_fn(module)
        retie_parameters(model, tied)
        return out

    return wrapper


def load_offloaded_weights(model, index, offload_folder):
    from .offload import load_offloaded_weight
    from .placement import set_module_tensor_to_device

    for name, meta in index.items():
        w = load_offloaded_weight(os.path.join(offload_folder, f"{name}.dat"), meta)
        set_module_tensor_to_device(model, name, "cpu", value=w)


# ------------------------------------------------------------------------------------------------ data-parallel helpers
def gather_across_data_parallel_groups(tensor):
    """All-gather `tensor` over the data-parallel group of the active mesh (world when no mesh)."""
    from ..state import AcceleratorState
    from .operations import gather

    st = AcceleratorState()
    mesh = getattr(st, "torch_device_mesh", None) if hasattr(st, "torch_device_mesh") else None
    if mesh is None or mesh.group("dp") is None:
        return gather(tensor)
    import torch.distributed as dist

    from ..parallel.comm import all_gather_dim

    return all_gather_dim(tensor if tensor.dim() else tensor.reshape(1), 0, mesh.group("dp"))


def avg_losses_across_data_parallel_group(losses: list):
    averaged = torch.cat([l.clone().detach().view(1) for l in losses])
    g = gather_across_data_parallel_groups(averaged)
    return g.view(-1, len(losses)).mean(0)


def is_peft_model(model) -> bool:
    return _has("peft") and type(model).__module__.startswith("peft")


def has_4bit_bnb_layers(model) -> bool:
    return False


# ------------------------------------------------------------------------------------------------ unsupported glue
def _unsupported(name: str, alt: str):
    class _Stub:
        def __init__(self, *a, **k):
            raise NotImplementedError(f"`{name}` belongs to a library that is not part of the MI355X stack. {alt}")

    _Stub.__name__ = name
    return _Stub


def _unsupported_fn(name: str, alt: str):
    def f(*a, **k):
        raise NotImplementedError(f"`{name}` is not available on the MI355X stack. {alt}")

    f.__name__ = name
    return f


_DS = "ZeRO stages are provided by the native FSDP2 engine (FullyShardedDataParallelPlugin)."
_MG = "TP/CP/SP/EP/PP are provided natively (ParallelismConfig, parallel/*, prepare_pippy)."

DeepSpeedEngineWrapper = _unsupported("DeepSpeedEngineWrapper", _DS)
DeepSpeedOptimizerWrapper = _unsupported("DeepSpeedOptimizerWrapper", _DS)
DeepSpeedSchedulerWrapper = _unsupported("DeepSpeedSchedulerWrapper", _DS)
HfDeepSpeedConfig = _unsupported("HfDeepSpeedConfig", _DS)
MegatronEngine = _unsupported("MegatronEngine", _MG)
MegatronLMDummyDataLoader = _unsupported("MegatronLMDummyDataLoader", _MG)
MegatronLMDummyScheduler = _unsupported("MegatronLMDummyScheduler", _MG)
MegatronLMOptimizerWrapper = _unsupported("MegatronLMOptimizerWrapper", _MG)
MegatronLMSchedulerWrapper = _unsupported("MegatronLMSchedulerWrapper", _MG)
AbstractTrainStep = _unsupported("AbstractTrainStep", _MG)
BertTrainStep = _unsupported("BertTrainStep", _MG)
GPTTrainStep = _unsupported("GPTTrainStep", _MG)
T5TrainStep = _unsupported("T5TrainStep", _MG)
add_model_config_to_megatron_parser = _unsupported_fn("add_model_config_to_megatron_parser", _MG)
megatron_lm_initialize = _unsupported_fn("megatron_lm_initialize", _MG)
megatron_lm_prepare_data_loader = _unsupported_fn("megatron_lm_prepare_data_loader", _MG)
megatron_lm_prepare_model_optimizer_scheduler = _unsupported_fn("megatron_lm_prepare_model_optimizer_scheduler", _MG)
megatron_lm_prepare_optimizer = _unsupported_fn("megatron_lm_prepare_optimizer", _MG)
megatron_lm_prepare_scheduler = _unsupported_fn("megatron_lm_prepare_scheduler", _MG)
load_and_quantize_model = _unsupported_fn("load_and_quantize_model", "bitsandbytes is not available on ROCm here; use fp8 (ops/fp8.py).")
install_xla = _unsupported_fn("install_xla", "TPU/XLA is out of scope.")
prepare_tpu = _unsupported_fn("prepare_tpu", "TPU/XLA is out of scope.")
prepare_sagemager_args_inputs = _unsupported_fn("prepare_sagemager_args_inputs", "SageMaker launches are out of scope.")


class DummyOptim:
    """Placeholder optimizer for DeepSpeed-config-driven training (reference utils/deepspeed.py:339-359). With the
    native engine it just records its arguments; `Accelerator.prepare` maps a DeepSpeed plugin to FSDP, where a real
    torch optimizer is required."""

    def __init__(self, params, lr=0.001, weight_decay=0, **kwargs):
        self.params, self.lr, self.weight_decay, self.kwargs = params, lr, weight_decay, kwargs


class DummyScheduler:
    def __init__(self, optimizer, total_num_steps=None, warmup_num_steps=0, lr_scheduler_callable=None, **kwargs):
        self.optimizer, self.total_num_steps, self.warmup_num_steps = optimizer, total_num_steps, warmup_num_steps
        self.lr_scheduler_callable, self.kwargs = lr_scheduler_callable, kwargs


def map_pytorch_optim_to_deepspeed(optimizer):
    return optimizer


def get_active_deepspeed_plugin(state):
    plugins = getattr(state, "deepspeed_plugins", None)
    if not plugins:
        raise ValueError("No DeepSpeed plugin is configured.")
    return next(p for p in plugins.values() if getattr(p, "selected", True))
