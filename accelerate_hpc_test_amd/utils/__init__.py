"""`accelerate_hpc_test_amd.utils` — the utility surface (parity with `accelerate.utils`, reference
`src/accelerate/utils/__init__.py:14-303`)."""

from .constants import (
    MODEL_NAME,
    OPTIMIZER_NAME,
    PROFILE_PATTERN_NAME,
    RNG_STATE_NAME,
    SAFE_MODEL_NAME,
    SAFE_WEIGHTS_INDEX_NAME,
    SAFE_WEIGHTS_NAME,
    SAMPLER_NAME,
    SCALER_NAME,
    SCHEDULER_NAME,
    TORCH_LAUNCH_PARAMS,
    WEIGHTS_INDEX_NAME,
    WEIGHTS_NAME,
)
from .dataclasses import (
    AORecipeKwargs,
    AutocastKwargs,
    BnbQuantizationConfig,
    ComputeEnvironment,
    CPUOffloadPolicy,
    CustomDtype,
    DataLoaderConfiguration,
    DDPCommunicationHookType,
    DeepSpeedPlugin,
    DeepSpeedSequenceParallelConfig,
    DistributedDataParallelKwargs,
    DistributedType,
    DynamoBackend,
    Float8LinearConfig,
    FP8BackendType,
    FP8RecipeKwargs,
    FullyShardedDataParallelPlugin,
    GradientAccumulationPlugin,
    GradScalerKwargs,
    InitProcessGroupKwargs,
    KwargsHandler,
    LoggerType,
    MegatronLMPlugin,
    MixedPrecisionPolicy,
    MSAMPRecipeKwargs,
    PrecisionType,
    ProfileKwargs,
    ProjectConfiguration,
    RcclKwargs,
    RNGType,
    SageMakerDistributedType,
    TensorInformation,
    TERecipeKwargs,
    TorchContextParallelConfig,
    TorchDynamoPlugin,
    TorchTensorParallelConfig,
    TorchTensorParallelPlugin,
    get_module_class_from_name,
)
from .environment import (
    are_libraries_initialized,
    check_fp8_capability,
    clear_environment,
    convert_dict_to_env_variables,
    get_cpu_distributed_information,
    get_gpu_arch,
    get_gpu_info,
    get_int_from_env,
    is_gfx950,
    parse_choice_from_env,
    parse_flag_from_env,
    patch_environment,
    purge_accelerate_environment,
    set_numa_affinity,
    str_to_bool,
)
from .imports import (
    is_aim_available,
    is_bf16_available,
    is_bnb_available,
    is_clearml_available,
    is_comet_ml_available,
    is_cuda_available,
    is_datasets_available,
    is_deepspeed_available,
    is_dvclive_available,
    is_fp8_available,
    is_fp16_available,
    is_hip_available,
    is_hpu_available,
    is_megatron_lm_available,
    is_mlflow_available,
    is_mlu_available,
    is_mps_available,
    is_msamp_available,
    is_npu_available,
    is_pandas_available,
    is_peft_available,
    is_pippy_available,
    is_rich_available,
    is_rocm_available,
    is_safetensors_available,
    is_swanlab_available,
    is_tensorboard_available,
    is_timm_available,
    is_torch_xla_available,
    is_torchao_available,
    is_torchdata_stateful_dataloader_available,
    is_tqdm_available,
    is_trackio_available,
    is_transformer_engine_available,
    is_transformers_available,
    is_wandb_available,
    is_xpu_available,
)
from .memory import clear_device_cache, find_executable_batch_size, release_memory, should_reduce_batch_size
from .modeling import (
    compute_module_sizes,
    convert_file_size_to_int,
    dtype_byte_size,
    get_grad_scaler,
    get_mixed_precision_context_manager,
    id_tensor_storage,
    named_module_tensors,
)
from .operations import (
    CannotPadNestedTensorWarning,
    ConvertOutputsToFp32,
    DistributedOperationException,
    GatheredParameters,
    broadcast,
    broadcast_object_list,
    concatenate,
    convert_outputs_to_fp32,
    convert_to_fp32,
    copy_tensor_to_devices,
    find_batch_size,
    find_device,
    gather,
    gather_object,
    get_data_structure,
    honor_type,
    ignorant_find_batch_size,
    initialize_tensors,
    is_namedtuple,
    is_tensor_information,
    is_torch_tensor,
    listify,
    pad_across_processes,
    pad_input_tensors,
    recursively_apply,
    reduce,
    send_to_device,
    slice_tensors,
)
from .other import (
    check_os_kernel,
    clean_state_dict_for_safetensors,
    compile_regions,
    compile_regions_deepspeed,
    convert_bytes,
    extract_model_from_parallel,
    get_module_children_bottom_up,
    get_pretty_name,
    has_compiled_regions,
    is_compiled_module,
    is_port_in_use,
    load,
    merge_dicts,
    recursive_getattr,
    save,
    wait_for_everyone,
)
from .random import set_seed, synchronize_rng_state, synchronize_rng_states
from .versions import compare_versions, is_torch_version
from .compat_api import *  # noqa: F401,F403 - remainder of the reference's utils surface (see compat_api.py)
from .compat_api import (  # noqa: F401 - explicit for linters / IDEs
    SAFE_WEIGHTS_PATTERN_NAME,
    TORCH_DISTRIBUTED_OPERATION_TYPES,
    WEIGHTS_PATTERN_NAME,
    DummyOptim,
    DummyScheduler,
    check_cuda_fp8_capability,
    fsdp2_prepare_model,
    gather_across_data_parallel_groups,
)


def __getattr__(name):
    # Heavier submodules are imported lazily (avoid import cycles with the package root).
    if name in ("merge_fsdp_weights", "save_fsdp_model", "load_fsdp_model", "save_fsdp_optimizer", "load_fsdp_optimizer"):
        from . import fsdp_utils

        return getattr(fsdp_utils, name)
    if name in (
        "infer_auto_device_map",
        "get_balanced_memory",
        "get_max_memory",
        "load_checkpoint_in_model",
        "set_module_tensor_to_device",
        "get_max_layer_size",
        "check_device_map",
        "load_state_dict",
        "calculate_maximum_sizes",
        "align_module_device",
        "has_offloaded_params",
        "find_tied_parameters",
        "retie_parameters",
        "clean_device_map",
        "get_module_leaves",
    ):
        from . import checkpoint_io, device_map, placement

        for mod in (device_map, placement, checkpoint_io):
            if hasattr(mod, name):
                return getattr(mod, name)
    if name in ("offload_weight", "load_offloaded_weight", "save_offload_index", "offload_state_dict", "OffloadedWeightsLoader", "PrefixedDataset", "extract_submodules_state_dict"):
        from . import offload

        return getattr(offload, name)
    if name in ("write_basic_config",):
        from ..commands.config.default import write_basic_config

        return write_basic_config
    if name in ("PrepareForLaunch", "prepare_multi_gpu_env", "prepare_simple_launcher_cmd_env", "get_launch_prefix",
                "prepare_deepspeed_cmd_env", "_filter_args", "setup_fp8_env", "_convert_nargs_to_dict", "env_var_path_add"):
        from . import launch

        return getattr(launch, name)
    if name == "ParallelismConfig":
        from ..parallelism_config import ParallelismConfig

        return ParallelismConfig
    if name == "tqdm":
        from .tqdm import tqdm

        return tqdm
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
