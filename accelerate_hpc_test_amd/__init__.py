"""accelerate_hpc_test_amd — an MI355X-native (gfx950, ROCm, RCCL/xGMI) training-loop framework with the public
API of 🤗 Accelerate (`/root/reference/src/accelerate/__init__.py:14-51`).

    from accelerate_hpc_test_amd import Accelerator
    accelerator = Accelerator(mixed_precision="bf16", fsdp_plugin=FullyShardedDataParallelPlugin(fsdp_version=2))
    model, optimizer, loader = accelerator.prepare(model, optimizer, loader)

Scripts written for `accelerate` run unchanged under `accelerate-amd launch` (which aliases the `accelerate`
module name to this package, see `compat.py`).
"""

__version__ = "0.1.0"

from .accelerator import Accelerator
from .big_modeling import (
    cpu_offload,
    cpu_offload_with_hook,
    disk_offload,
    dispatch_model,
    init_empty_weights,
    init_on_device,
    load_checkpoint_and_dispatch,
)
from .data_loader import skip_first_batches
from .inference import prepare_pippy
from .launchers import debug_launcher, notebook_launcher
from .parallelism_config import ParallelismConfig
from .state import PartialState
from .utils import (
    AutocastKwargs,
    DataLoaderConfiguration,
    DDPCommunicationHookType,
    DeepSpeedPlugin,
    DistributedDataParallelKwargs,
    DistributedType,
    FullyShardedDataParallelPlugin,
    GradScalerKwargs,
    InitProcessGroupKwargs,
    ProfileKwargs,
    find_executable_batch_size,
    is_rich_available,
    synchronize_rng_states,
)
from .utils.checkpoint_io import load_checkpoint_in_model
from .utils.device_map import infer_auto_device_map

if is_rich_available():
    from .utils import rich  # noqa: F401
