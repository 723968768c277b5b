"""Feature detection, collapsed to what matters on an MI355X (ROCm) stack.

Parity: `/root/reference/src/accelerate/utils/imports.py:50-518`. The reference probes a dozen vendor
back-ends; here there are two: CPU (gloo) and ROCm GPUs (RCCL). Optional Python integrations
(transformers, datasets, trackers) are probed lazily with importlib so nothing is imported eagerly.
"""

from __future__ import annotations

import functools
import importlib.util
import os


def _is_package_available(name: str) -> bool:
    return importlib.util.find_spec(name) is not None


@functools.lru_cache
def is_torch_available() -> bool:
    return _is_package_available("torch")


@functools.lru_cache
def is_rocm_available() -> bool:
    import torch

    return getattr(torch.version, "hip", None) is not None


def is_cuda_available() -> bool:
    """True when a ROCm GPU is usable (PyTorch exposes HIP devices under the `cuda` device type)."""
    import torch

    return torch.cuda.is_available()


def is_hip_available() -> bool:
    return is_rocm_available() and is_cuda_available()


def is_bf16_available(ignore_tpu: bool = True) -> bool:
    # Every CDNA GPU and every x86 CPU supported by PyTorch handles bf16.
    return True


def is_fp16_available() -> bool:
    return True


def is_fp8_available() -> bool:
    """fp8 training runs on our own HIP kernels (no torchao/TE dependency); needs gfx950."""
    from .environment import check_fp8_capability

    return check_fp8_capability()


def is_torchao_available() -> bool:
    return _is_package_available("torchao")


def is_transformer_engine_available() -> bool:
    return False  # not used: fp8 is served by our own kernels (ops/fp8.py)


def is_msamp_available() -> bool:
    return False


def is_deepspeed_available() -> bool:
    return False  # capabilities re-provided natively (parallel/fsdp.py, parallel/ulysses.py)


def is_megatron_lm_available() -> bool:
    return False


def is_bnb_available() -> bool:
    return False


def is_torch_xla_available(*args, **kwargs) -> bool:
    return False


def is_npu_available(*args, **kwargs) -> bool:
    return False


def is_xpu_available(*args, **kwargs) -> bool:
    return False


def is_mps_available(*args, **kwargs) -> bool:
    return False


def is_mlu_available(*args, **kwargs) -> bool:
    return False


def is_hpu_available(*args, **kwargs) -> bool:
    return False


def is_transformers_available() -> bool:
    return _is_package_available("transformers")


def is_datasets_available() -> bool:
    return _is_package_available("datasets")


def is_safetensors_available() -> bool:
    return _is_package_available("safetensors")


def is_rich_available() -> bool:
    if _is_package_available("rich"):
        from .environment import parse_flag_from_env

        return parse_flag_from_env("ACCELERATE_ENABLE_RICH", False)
    return False


def is_tqdm_available() -> bool:
    return _is_package_available("tqdm")


def is_tensorboard_available() -> bool:
    return _is_package_available("tensorboard") or _is_package_available("tensorboardX")


def is_wandb_available() -> bool:
    return _is_package_available("wandb")


def is_comet_ml_available() -> bool:
    return _is_package_available("comet_ml")


def is_aim_available() -> bool:
    return _is_package_available("aim")


def is_mlflow_available() -> bool:
    return _is_package_available("mlflow")


def is_clearml_available() -> bool:
    return _is_package_available("clearml")


def is_dvclive_available() -> bool:
    return _is_package_available("dvclive")


def is_swanlab_available() -> bool:
    return _is_package_available("swanlab")


def is_trackio_available() -> bool:
    return _is_package_available("trackio")


def is_pandas_available() -> bool:
    return _is_package_available("pandas")


def is_torchdata_stateful_dataloader_available() -> bool:
    if not _is_package_available("torchdata"):
        return False
    try:
        from torchdata.stateful_dataloader import StatefulDataLoader  # noqa: F401

        return True
    except Exception:
        return False


def is_timm_available() -> bool:
    return _is_package_available("timm")


def is_psutil_available() -> bool:
    return _is_package_available("psutil")


def is_native_extension_available() -> bool:
    """True when the in-tree HIP extension (`accelerate_hpc_test_amd._C`) imports."""
    from ..ops import _ext

    return _ext.available()


def is_ccl_available() -> bool:
    return False


def is_mpi_available() -> bool:
    import torch.distributed as dist

    return dist.is_mpi_available()


def is_pippy_available() -> bool:
    # Pipeline inference is implemented natively in inference.py (no torch.distributed.pipelining needed).
    return True


def is_import_timer_available() -> bool:
    return False


def torch_distributed_available() -> bool:
    import torch.distributed as dist

    return dist.is_available()


def get_ccl_version():
    return None


def is_boto3_available() -> bool:
    return _is_package_available("boto3")


def is_sagemaker_available() -> bool:
    return False


def is_triton_available() -> bool:
    # Deliberately unused on the perf path (north star: no Triton).
    return False


def is_peft_available() -> bool:
    return _is_package_available("peft")


def is_schedulefree_available() -> bool:
    return _is_package_available("schedulefree")


def is_lomo_available() -> bool:
    return _is_package_available("lomo_optim")


def is_matplotlib_available() -> bool:
    return _is_package_available("matplotlib")


def use_native_kernels() -> bool:
    """Global switch for the HIP kernels (`ACCELERATE_NATIVE_KERNELS=0` forces the PyTorch reference path
    for debugging; on a GPU the default is the HIP path and missing kernels raise)."""
    return os.environ.get("ACCELERATE_NATIVE_KERNELS", "1") != "0"
