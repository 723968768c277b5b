"""Process / device runtime singletons: `PartialState`, `AcceleratorState`, `GradientState`.

Parity: `/root/reference/src/accelerate/state.py:122-1365`. Semantics kept: shared-state (Borg) singletons,
`_reset_state`, `wait_for_everyone`, `split_between_processes`, the `on_*_process` decorators,
`main_process_first`, the AttributeError raised when a reset state is accessed. What differs:

* Only two executable back-ends: CPU (gloo; `MULTI_CPU` when WORLD_SIZE>1) and ROCm GPUs (RCCL through
  `torch.distributed`'s "nccl" backend, `MULTI_GPU`/`FSDP`). There is no multi-vendor backend ladder.
* One process per GPU: `cuda:{LOCAL_RANK % device_count}`, bound before the process group is created so
  RCCL communicators are created on the right device. When FSDP needs CPU collectives (offload, full
  state dicts) the group is created as `cuda:nccl,cpu:gloo`.
"""

from __future__ import annotations

import os
import threading
import warnings
from contextlib import contextmanager
from typing import Any, Callable

import torch

from .utils.dataclasses import DistributedType, GradientAccumulationPlugin, SageMakerDistributedType
from .utils.environment import (
    get_cpu_distributed_information,
    get_int_from_env,
    parse_choice_from_env,
    parse_flag_from_env,
    set_numa_affinity,
    str_to_bool,
)


def is_initialized() -> bool:
    """Whether an `AcceleratorState` has been created in this process."""
    return AcceleratorState._shared_state != {}


def do_nothing(*args, **kwargs):
    return None


class ThreadLocalSharedDict(threading.local):
    """Per-thread shared dict (used when `ACCELERATE_THREAD_LOCAL_STATE=1`)."""

    def __init__(self, thread_local: bool = False):
        self._storage = {}

    def __get__(self, obj, objtype=None):
        return self._storage

    def __set__(self, obj, value):
        self._storage = value


SharedDict = ThreadLocalSharedDict if parse_flag_from_env("ACCELERATE_THREAD_LOCAL_STATE") else dict

# Attributes every initialised state carries: reading one of them after `_reset_state()` is a use-after-reset, reported
# with a hint instead of the bare AttributeError.
_PARTIAL_ATTRS = frozenset(
    "_cpu _mixed_precision _shared_state backend debug device distributed_type fork_launched local_process_index "
    "num_processes process_index".split()
)
_ACCELERATOR_ATTRS = _PARTIAL_ATTRS | frozenset(
    "deepspeed_plugin use_ipex fsdp_plugin megatron_lm_plugin dynamo_plugin parallelism_config device_mesh".split()
)


def _missing_attribute(owner: str, name: str, known) -> AttributeError:
    if name in known:
        return AttributeError(
            f"`{owner}` object has no attribute `{name}`. This happens if `{owner}._reset_state()` was called and an "
            "`Accelerator` or `PartialState` was not reinitialized."
        )
    return AttributeError(f"'{owner}' object has no attribute '{name}'")


class PartialState:
    """Process-level singleton: distributed environment, device, process indices.

    Creating it initialises `torch.distributed` when the launcher set `WORLD_SIZE>1` (torchrun /
    `accelerate launch` / `debug_launcher`). All instances share one dict of attributes.
    """

    _shared_state = SharedDict()
    _known_attrs = _PARTIAL_ATTRS

    def __init__(self, cpu: bool = False, **kwargs):
        self.__dict__ = self._shared_state
        if self.initialized:
            return
        self._cpu = cpu
        self.backend = None
        env_device = os.environ.get("ACCELERATE_TORCH_DEVICE", None)
        self.device = torch.device(env_device) if env_device is not None else None
        self.debug = parse_flag_from_env("ACCELERATE_DEBUG_MODE")
        use_cpu = cpu or parse_flag_from_env("ACCELERATE_USE_CPU") or not torch.cuda.is_available()
        self._use_cpu = use_cpu

        backend, distributed_type = self._prepare_backend(use_cpu, kwargs.pop("backend", None))
        self.backend = backend
        self.distributed_type = distributed_type
        timeout = kwargs.pop("timeout", None)
        init_method = kwargs.pop("init_method", None)

        world_size = get_int_from_env(["WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE"], 1)
        if distributed_type == DistributedType.NO:
            self.num_processes = 1
            self.process_index = 0
            self.local_process_index = 0
        else:
            if distributed_type == DistributedType.MULTI_CPU:
                info = get_cpu_distributed_information()
                os.environ.setdefault("RANK", str(info.rank))
                os.environ.setdefault("WORLD_SIZE", str(info.world_size))
                os.environ.setdefault("LOCAL_RANK", str(info.local_rank))
                os.environ.setdefault("LOCAL_WORLD_SIZE", str(info.local_world_size))
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
            # Bind the device BEFORE the process group so RCCL comms land on the right GPU.
            if not use_cpu:
                local_rank = int(os.environ.get("LOCAL_RANK", "0"))
                self.device = torch.device("cuda", local_rank % torch.cuda.device_count())
                torch.cuda.set_device(self.device)
            if not torch.distributed.is_initialized():
                pg_kwargs = {"backend": backend}
                if timeout is not None:
                    pg_kwargs["timeout"] = timeout
                if init_method is not None:
                    pg_kwargs["init_method"] = init_method
                if backend == "nccl" and self.device is not None:
                    pg_kwargs["device_id"] = self.device
                torch.distributed.init_process_group(**pg_kwargs)
            self.num_processes = torch.distributed.get_world_size()
            self.process_index = torch.distributed.get_rank()
            self.local_process_index = int(os.environ.get("LOCAL_RANK", -1))
            if self.local_process_index < 0:
                self.local_process_index = self.process_index % max(1, get_int_from_env(["LOCAL_WORLD_SIZE"], 1))
        if self.device is None:
            self.device = torch.device("cpu") if use_cpu else torch.device("cuda", 0)
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device)
        if (
            parse_flag_from_env("ACCELERATE_CPU_AFFINITY", False)
            and self.device.type == "cuda"
            and distributed_type != DistributedType.NO
        ):
            set_numa_affinity(self.local_process_index)
        self.fork_launched = parse_flag_from_env("FORK_LAUNCHED", 0)
        _ = world_size

    # ------------------------------------------------------------------------------------------
    def _prepare_backend(self, cpu: bool, backend: str | None = None) -> tuple[str | None, DistributedType]:
        """Decide the collective backend. Reference ladder `state.py:753-812`, collapsed to gloo/RCCL."""
        world_size = get_int_from_env(["WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE"], 1)
        if world_size <= 1:
            return None, DistributedType.NO
        if cpu:
            if backend is None or backend == "nccl":
                backend = "gloo"
            return backend, DistributedType.MULTI_CPU
        if backend is None:
            backend = "nccl"  # RCCL on ROCm
        if backend == "nccl" and parse_flag_from_env("ACCELERATE_FSDP_CPU_COLLECTIVES", False):
            backend = "cuda:nccl,cpu:gloo"
        return backend, DistributedType.MULTI_GPU

    def __repr__(self) -> str:
        return (
            f"Distributed environment: {self.distributed_type}{('  Backend: ' + self.backend) if self.backend else ''}\n"
            f"Num processes: {self.num_processes}\n"
            f"Process index: {self.process_index}\n"
            f"Local process index: {self.local_process_index}\n"
            f"Device: {self.device}\n"
        )

    @staticmethod
    def _reset_state():
        PartialState._shared_state.clear()

    @property
    def initialized(self) -> bool:
        return self._shared_state != {}

    @property
    def use_distributed(self):
        return self.distributed_type != DistributedType.NO and self.num_processes > 1

    @property
    def is_last_process(self) -> bool:
        return self.process_index == self.num_processes - 1

    @property
    def is_main_process(self) -> bool:
        return self.process_index == 0

    @property
    def is_local_main_process(self) -> bool:
        return self.local_process_index == 0

    def wait_for_everyone(self):
        """Barrier across all processes (no-op single-process). On RCCL the barrier is device-bound."""
        if (
            self.distributed_type in (DistributedType.MULTI_GPU, DistributedType.MULTI_CPU, DistributedType.FSDP)
            and torch.distributed.is_initialized()
            and self.num_processes > 1
        ):
            if self.backend == "nccl" and self.device is not None and self.device.type == "cuda":
                torch.distributed.barrier(device_ids=[self.device.index])
            else:
                torch.distributed.barrier()

    def _goes_first(self, is_main: bool):
        if not is_main:
            self.wait_for_everyone()
        yield
        if is_main:
            self.wait_for_everyone()

    @contextmanager
    def split_between_processes(self, inputs: list | tuple | dict | torch.Tensor, apply_padding: bool = False):
        """Hand process i the i-th contiguous block of `inputs` (reference `state.py:423-512`): n items over p processes
        give the first n % p processes one extra item. Lists, tuples, tensors (dim 0), dicts of those (split
        key-wise, every value the same length) and `datasets.Dataset` (index selection) are split; anything else is
        handed over whole. `apply_padding` makes every block as long as the longest, repeating the block's last item
        (lists / datasets) or the input's last element along dim 0 (tensors), so a later `gather` is rectangular."""
        if self.num_processes == 1:
            yield inputs
            return
        if isinstance(inputs, dict):
            lengths = {len(v) for v in inputs.values()}
            if len(lengths) > 1:
                raise ValueError("All values in the dictionary must have the same length")
            total = lengths.pop() if lengths else 0
        else:
            total = len(inputs)
        base, extra = divmod(total, self.num_processes)
        i = self.process_index
        lo = i * base + min(i, extra)
        hi = lo + base + (i < extra)
        longest = base + (extra > 0)
        yield self._split_block(inputs, lo, hi, longest, apply_padding)

    def _split_block(self, inputs, lo: int, hi: int, longest: int, pad: bool):
        if isinstance(inputs, dict):
            for key in inputs:
                inputs[key] = self._split_block(inputs[key], lo, hi, longest, pad)
            return inputs
        if isinstance(inputs, torch.Tensor):
            block = inputs[lo:hi] if lo < inputs.shape[0] else inputs[-1:]
            if pad and block.shape[0] < longest:
                filler = inputs[-1:].expand(longest - block.shape[0], *inputs.shape[1:])
                block = torch.cat([block, filler.to(block.device)])
            return block.to(self.device) if pad else block
        if isinstance(inputs, (list, tuple)):
            block = inputs[lo:hi] if lo < len(inputs) else inputs[-1:]
            if pad and len(block) < longest:
                block = block + type(block)([block[-1]]) * (longest - len(block))
            return block
        try:
            from datasets import Dataset
        except ImportError:
            return inputs
        if isinstance(inputs, Dataset):
            n = len(inputs)
            idx = list(range(min(lo, n - 1), min(hi, n)))
            if pad:
                idx += [idx[-1]] * (longest - len(idx))
            return inputs.select(idx)
        return inputs

    @contextmanager
    def main_process_first(self):
        yield from self._goes_first(self.is_main_process)

    @contextmanager
    def local_main_process_first(self):
        yield from self._goes_first(self.is_local_main_process)

    # ---- process-filter decorators: each returns `function` on the selected process(es) and a no-op elsewhere.
    # Outside a distributed run every filter selects the (only) process.
    def _selected(self, chosen: bool, function):
        return function if (chosen or not self.use_distributed) else do_nothing

    def on_main_process(self, function: Callable[..., Any] | None = None):
        if not self.initialized:
            raise ValueError("The `PartialState` or `Accelerator` must be initialized before calling this function.")
        return self._selected(self.is_main_process, function)

    def on_local_main_process(self, function: Callable[..., Any] | None = None):
        return self._selected(self.is_local_main_process, function)

    def on_last_process(self, function: Callable[..., Any]):
        return self._selected(self.is_last_process, function)

    def on_process(self, function: Callable[..., Any] | None = None, process_index: int | None = None):
        # usable bare (`@state.on_process(process_index=1)`) or applied directly
        if function is None:
            return lambda fn: self.on_process(fn, process_index=process_index)
        return self._selected(self.process_index == process_index, function)

    def on_local_process(self, function: Callable[..., Any] | None = None, local_process_index: int | None = None):
        if function is None:
            return lambda fn: self.on_local_process(fn, local_process_index=local_process_index)
        return self._selected(self.local_process_index == local_process_index, function)

    def print(self, *args, **kwargs):
        """`print` on the local main process only."""
        if self.is_local_main_process:
            print(*args, **kwargs)

    @property
    def default_device(self) -> torch.device:
        if torch.cuda.is_available() and not self._use_cpu:
            return torch.device("cuda")
        return torch.device("cpu")

    def set_device(self):
        if self.device is not None:
            return
        if self.distributed_type == DistributedType.NO:
            self.device = torch.device("cpu") if self._use_cpu else self.default_device
            return
        if self._use_cpu:
            self.device = torch.device("cpu")
            return
        self.device = torch.device("cuda", self.local_process_index % torch.cuda.device_count())
        torch.cuda.set_device(self.device)

    def destroy_process_group(self, group=None):
        if self.fork_launched and group is None:
            return
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group(group)

    def __getattr__(self, name: str):
        raise _missing_attribute("PartialState", name, self._known_attrs)


class AcceleratorState:
    """Training-level singleton: mixed precision, plugins, and the promoted distributed type."""

    _shared_state = SharedDict()
    _known_attrs = _ACCELERATOR_ATTRS

    def __init__(
        self,
        mixed_precision: str | None = None,
        cpu: bool = False,
        dynamo_plugin=None,
        deepspeed_plugin=None,
        fsdp_plugin=None,
        torch_tp_plugin=None,
        megatron_lm_plugin=None,
        parallelism_config=None,
        _from_accelerator: bool = False,
        **kwargs,
    ):
        self.__dict__ = self._shared_state
        cpu = cpu or parse_flag_from_env("ACCELERATE_USE_CPU")
        PartialState(cpu, **kwargs)  # creates the process state once; later calls just share it
        self.__dict__.update(PartialState._shared_state)
        already_set_up = self.initialized and getattr(self, "_mixed_precision", None) is not None
        if already_set_up:
            self._check_initialized(mixed_precision, cpu)
            return
        self._cpu = cpu
        mixed_precision = (
            parse_choice_from_env("ACCELERATE_MIXED_PRECISION", "no") if mixed_precision is None else mixed_precision.lower()
        )
        if mixed_precision == "fp8":
            from .utils.environment import check_fp8_capability

            if not cpu and torch.cuda.is_available() and not check_fp8_capability():
                warnings.warn("fp8 requires gfx950 (MI355X); falling back to bf16.")
                mixed_precision = "bf16"
        self.dynamo_plugin = dynamo_plugin
        self._mixed_precision = mixed_precision
        self.deepspeed_plugins = None
        self.use_ipex = False
        self.torch_tp_plugin = torch_tp_plugin
        self.parallelism_config = parallelism_config
        self.device_mesh = None
        self.megatron_lm_plugin = None
        if megatron_lm_plugin is not None:
            raise NotImplementedError("Megatron-LM is not supported on MI355X.")
        if deepspeed_plugin is not None:
            # ZeRO stages map onto our FSDP engine. Several named plugins may be given (reference
            # state.py:1178-1207); the first one is active until `select_deepspeed_plugin` switches.
            plugins = deepspeed_plugin if isinstance(deepspeed_plugin, dict) else {"default": deepspeed_plugin}
            for i, p in enumerate(plugins.values()):
                p.selected = i == 0
            self.deepspeed_plugins = plugins
            if fsdp_plugin is None:
                fsdp_plugin = next(iter(plugins.values())).to_fsdp_plugin()
        if os.environ.get("ACCELERATE_USE_FSDP", "false").lower() == "true" or fsdp_plugin is not None:
            self.fsdp_plugin = fsdp_plugin
        else:
            self.fsdp_plugin = None
        if parallelism_config is not None and parallelism_config.cp_enabled and fsdp_plugin is None:
            if not parse_flag_from_env("ACCELERATE_ALLOW_CP_STANDALONE", False):
                raise ValueError("Context parallelism requires FSDP2 (pass an `fsdp_plugin` with fsdp_version=2).")
        if self.fsdp_plugin is not None and self.distributed_type in (
            DistributedType.MULTI_GPU,
            DistributedType.MULTI_CPU,
            DistributedType.NO,
        ):
            # Single-device FSDP still runs the engine (fp32 master shards + bf16 compute params); on CPU the
            # engine uses gloo, which is how the sharding logic is tested without GPUs.
            self.distributed_type = DistributedType.FSDP
            if self._mixed_precision != "no" and self.fsdp_plugin.mixed_precision_policy is None:
                self.fsdp_plugin.set_mixed_precision(self._mixed_precision)
        PartialState._shared_state["distributed_type"] = self.distributed_type

    @property
    def initialized(self) -> bool:
        return self._shared_state != PartialState._shared_state

    def __repr__(self):
        return f"{PartialState()!r}\nMixed precision type: {self.mixed_precision}\n"

    def _check_initialized(self, mixed_precision=None, cpu=None):
        """A second Accelerator in the same process may not change the device kind or the precision."""
        if not (self.initialized and getattr(self, "_mixed_precision", None) is not None):
            return
        conflict = None
        if cpu and self.device.type != "cpu":
            conflict = "cpu=True"
        elif mixed_precision is not None and mixed_precision != self._mixed_precision:
            conflict = f"mixed_precision='{mixed_precision}'"
        if conflict:
            raise ValueError(
                "AcceleratorState has already been initialized and cannot be changed, restart your runtime completely "
                f"and pass `{conflict}` to `Accelerator()`."
            )

    @property
    def mixed_precision(self):
        return self._mixed_precision

    @staticmethod
    def _reset_state(reset_partial_state: bool = False):
        AcceleratorState._shared_state.clear()
        if reset_partial_state:
            PartialState._reset_state()

    @property
    def is_fsdp2(self) -> bool:
        return self.distributed_type == DistributedType.FSDP and self.fsdp_plugin.fsdp_version == 2

    # Process-level queries and helpers live on PartialState; AcceleratorState forwards them (see the loop after the
    # class body) so both singletons answer the same questions the same way.
    _FORWARDED_PROPERTIES = ("fork_launched", "use_distributed", "is_last_process", "is_main_process",
                             "is_local_main_process")
    _FORWARDED_METHODS = ("destroy_process_group", "wait_for_everyone", "split_between_processes",
                          "main_process_first", "local_main_process_first", "print")

    @property
    def deepspeed_plugin(self):
        """The active DeepSpeed plugin (its ZeRO semantics run on the FSDP engine), or None."""
        plugins = self.__dict__.get("deepspeed_plugins") or self._shared_state.get("deepspeed_plugins")
        if not plugins:
            return None
        return next((p for p in plugins.values() if getattr(p, "selected", False)), None)

    def get_deepspeed_plugin(self, name: str):
        return self.deepspeed_plugins[name]

    def select_deepspeed_plugin(self, name: str = None):
        if name not in (self.deepspeed_plugins or {}):
            raise ValueError(f"{name} is not a valid DeepSpeed plugin; choose from {list(self.deepspeed_plugins or {})}")
        for key, p in self.deepspeed_plugins.items():
            p.selected = key == name
        self.fsdp_plugin = self.deepspeed_plugins[name].to_fsdp_plugin()

    def __getattr__(self, name: str):
        raise _missing_attribute("AcceleratorState", name, self._known_attrs)


def _install_forwarders():
    for _name in AcceleratorState._FORWARDED_PROPERTIES:
        setattr(AcceleratorState, _name, property(lambda self, _n=_name: getattr(PartialState(), _n)))
    for _name in AcceleratorState._FORWARDED_METHODS:
        def _fwd(self, *args, _n=_name, **kwargs):
            return getattr(PartialState(), _n)(*args, **kwargs)

        _fwd.__name__ = _name
        _fwd.__doc__ = getattr(PartialState, _name).__doc__
        setattr(AcceleratorState, _name, _fwd)


_install_forwarders()


class GradientState:
    """Gradient-accumulation bookkeeping shared by the Accelerator, dataloaders, optimizer and scheduler (reference
    `state.py:1225-1365`): whether this step syncs gradients, the accumulation plugin's settings, and the stack of
    dataloaders being iterated (weak references; the innermost one decides `end_of_dataloader` / `remainder`)."""

    _shared_state = SharedDict()
    _PLUGIN_DEFAULTS = {"num_steps": 1, "adjust_scheduler": False, "sync_with_dataloader": True}

    def __init__(self, gradient_accumulation_plugin: GradientAccumulationPlugin | None = None):
        self.__dict__ = self._shared_state
        settings = gradient_accumulation_plugin.to_kwargs() if gradient_accumulation_plugin is not None else None
        if not self.initialized:
            self.sync_gradients = True
            self._dataloader_references_ref = [None]
            self.plugin_kwargs = settings or {}
        elif settings is not None:
            self.plugin_kwargs = settings  # a later plugin replaces the earlier settings

    def _setting(self, key):
        return self.plugin_kwargs.get(key, self._PLUGIN_DEFAULTS[key])

    num_steps = property(lambda self: self._setting("num_steps"))
    adjust_scheduler = property(lambda self: self._setting("adjust_scheduler"))
    sync_with_dataloader = property(lambda self: self._setting("sync_with_dataloader"))

    @property
    def initialized(self) -> bool:
        return GradientState._shared_state != {}

    @property
    def is_xla_gradients_synced(self) -> bool:
        """XLA-only flag in the reference; there is no XLA here, so gradients are always synced by our engines."""
        return True

    @is_xla_gradients_synced.setter
    def is_xla_gradients_synced(self, value):
        pass

    @property
    def end_of_dataloader(self) -> bool:
        dl = self.active_dataloader
        return dl.end_of_dataloader if dl is not None else False

    @property
    def remainder(self) -> int:
        dl = self.active_dataloader
        return dl.remainder if dl is not None else -1

    def __repr__(self):
        lines = [
            ("Sync Gradients", self.sync_gradients),
            ("At end of current dataloader", self.end_of_dataloader),
            ("Extra samples added", self.remainder),
            ("Gradient accumulation plugin", self.plugin_kwargs),
        ]
        return "".join(f"{k}: {v}\n" for k, v in lines)

    def _set_sync_gradients(self, sync_gradients):
        self.sync_gradients = sync_gradients

    def _add_dataloader(self, dataloader):
        import weakref

        self._dataloader_references_ref.append(weakref.ref(dataloader))

    def _remove_dataloader(self, dataloader):
        """Drop the innermost reference to `dataloader` (nested loops over one loader unwind one level)."""
        refs = self._dataloader_references_ref
        hit = next((i for i in reversed(range(len(refs))) if refs[i] is not None and refs[i]() is dataloader), None)
        if hit is not None:
            del refs[hit]

    @property
    def active_dataloader(self):
        ref = self._dataloader_references_ref[-1]
        return None if ref is None else ref()

    @property
    def dataloader_references(self):
        return self._dataloader_references_ref

    @dataloader_references.setter
    def dataloader_references(self, references):
        self._dataloader_references_ref = references

    @property
    def in_dataloader(self) -> bool:
        return self.active_dataloader is not None

    @staticmethod
    def _reset_state():
        GradientState._shared_state.clear()
