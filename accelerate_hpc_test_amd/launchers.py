"""In-process launchers: `notebook_launcher` (elastic, fork) and `debug_launcher` (CPU gloo fake cluster).

Parity: `/root/reference/src/accelerate/launchers.py:41-309`. `notebook_launcher` starts one worker per GPU through
torch's elastic agent (so `max_restarts` / `monitor_interval` fault tolerance works), binding each worker to one
MI355X via LOCAL_RANK. `debug_launcher` forks N CPU processes sharing a gloo FileStore rendezvous — the harness
for multi-rank semantics tests without GPUs.
"""

from __future__ import annotations

import os
import sys
import tempfile

import torch

from .state import AcceleratorState, PartialState
from .utils.environment import are_libraries_initialized, patch_environment
from .utils.other import get_free_port, is_port_in_use


def test_launch():
    """Sanity entry used by `accelerate-amd test`."""
    _ = PartialState()


def notebook_launcher(
    function,
    args=(),
    num_processes=None,
    mixed_precision="no",
    use_port="29500",
    master_addr="127.0.0.1",
    node_rank=0,
    num_nodes=1,
    rdzv_backend="static",
    rdzv_endpoint="",
    rdzv_conf=None,
    rdzv_id="none",
    max_restarts=0,
    monitor_interval=0.1,
    log_line_prefix_template=None,
):
    """Launch `function(*args)` on `num_processes` local workers (one per GPU) with elastic fault tolerance."""
    problematic_imports = are_libraries_initialized("bitsandbytes")
    if problematic_imports:
        raise RuntimeError(
            "Could not start distributed process. Libraries known to initialize the device upon import have been "
            f"imported already: {', '.join(problematic_imports)}. Import them inside the launched function instead."
        )
    if num_processes is None:
        num_processes = max(1, torch.cuda.device_count())
    if num_processes == 1 and num_nodes == 1:  # nothing to launch: run in this process
        with patch_environment(accelerate_mixed_precision=mixed_precision):
            function(*args)
        return
    if AcceleratorState._shared_state:
        raise ValueError(
            "To launch a multi-GPU training from your notebook, the `Accelerator` should only be initialized inside your "
            "training function. Restart your notebook and make sure no cells initializes an `Accelerator`."
        )
    if rdzv_backend == "static" and num_nodes == 1 and is_port_in_use(int(use_port)):
        use_port = str(get_free_port())
    config = _elastic_config(num_processes, num_nodes, node_rank, master_addr, use_port, rdzv_backend, rdzv_endpoint,
                             rdzv_conf, rdzv_id, max_restarts, monitor_interval, log_line_prefix_template)
    from torch.distributed.launcher.api import elastic_launch

    worker_env = {
        "nproc": num_processes, "node_rank": node_rank, "world_size": num_nodes * num_processes,
        "master_addr": master_addr, "master_port": use_port, "mixed_precision": mixed_precision,
        "accelerate_mixed_precision": mixed_precision, "fork_launched": "1",
        # dmabuf IPC: RCCL peer buffers and HIP-tensor sharing between the forked workers
        "hsa_enable_ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    }
    with patch_environment(**worker_env):
        elastic_launch(config=config, entrypoint=function)(*args)


def _elastic_config(nproc, nnodes, node_rank, master_addr, port, backend, endpoint, conf, run_id, max_restarts,
                    monitor_interval, log_line_prefix_template):
    """torch elastic LaunchConfig for `nproc` forked workers per node: a static rendezvous gets this node's rank and
    defaults its endpoint to master_addr:port; restarts / monitoring follow the caller's fault-tolerance settings."""
    from torch.distributed.launcher.api import LaunchConfig

    conf = dict(conf or {})
    if backend == "static":
        conf["rank"] = node_rank
        endpoint = endpoint or f"{master_addr}:{port}"
    extra = {} if log_line_prefix_template is None else {"log_line_prefix_template": log_line_prefix_template}
    return LaunchConfig(min_nodes=nnodes, max_nodes=nnodes, nproc_per_node=nproc, run_id=run_id, rdzv_endpoint=endpoint,
                        rdzv_backend=backend, rdzv_configs=conf, max_restarts=max_restarts,
                        monitor_interval=monitor_interval, start_method="fork", **extra)


def debug_launcher(function, args=(), num_processes=2):
    """Run `function(*args)` on `num_processes` forked CPU processes (gloo over a FileStore)."""
    from torch.multiprocessing import start_processes

    with tempfile.NamedTemporaryFile() as tmp_file:
        with patch_environment(
            world_size=num_processes,
            master_addr="127.0.0.1",
            master_port=str(get_free_port()),
            accelerate_debug_rdv_file=tmp_file.name,
            accelerate_use_cpu="yes",
        ):
            launcher = _DebugWorker(function)
            start_processes(launcher, args=args, nprocs=num_processes, start_method="fork")


class _DebugWorker:
    """Sets RANK/LOCAL_RANK from the process index and initialises gloo on a FileStore (utils/launch.py parity)."""

    def __init__(self, launcher):
        self.launcher = launcher

    def __call__(self, index, *args):
        os.environ["LOCAL_RANK"] = str(index)
        os.environ["RANK"] = str(index)
        os.environ["FORK_LAUNCHED"] = str(1)
        # A forked child inherits the parent's OpenMP pool bookkeeping but not its threads: the first parallel
        # region would wait forever on workers that do not exist. The fake cluster runs tiny models, so run
        # each rank single-threaded.
        torch.set_num_threads(1)
        rdv_file = os.environ.get("ACCELERATE_DEBUG_RDV_FILE")
        if rdv_file:
            torch.distributed.init_process_group(
                "gloo",
                rank=index,
                store=torch.distributed.FileStore(rdv_file, int(os.environ["WORLD_SIZE"])),
                world_size=int(os.environ["WORLD_SIZE"]),
            )
        self.launcher(*args)
