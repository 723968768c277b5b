"""N-D parallelism configuration and the rank mesh (one RCCL communicator per mesh dimension).

Parity: `/root/reference/src/accelerate/parallelism_config.py:33-398` — same fields (`dp_replicate_size`,
`dp_shard_size`, `cp_size`, `sp_size`, `tp_size`, handlers, `PARALLELISM_CONFIG_*` env vars), same canonical
dimension order (dp_replicate, dp_shard, cp, sp, tp — TP innermost so TP groups stay inside one node's xGMI mesh),
same flattened views (`dp` = replicate×shard, `dp_shard_cp`, `dp_cp`), same validation.

Instead of torch's DeviceMesh/DTensor, `RankMesh` builds the process groups directly with
`torch.distributed.new_group` (RCCL communicators on GPU, gloo on CPU) and exposes them by name.
"""

from __future__ import annotations

import itertools
import os
import warnings
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from .utils.dataclasses import DeepSpeedSequenceParallelConfig, TorchContextParallelConfig, TorchTensorParallelConfig

_DIM_ORDER = ("dp_replicate", "dp_shard", "cp", "sp", "tp")


class RankMesh:
    """Rank grid over the canonical dims; `group(name)` returns the process group this rank belongs to for a single
    dimension or a flattened combination (`dp`, `dp_shard_cp`, `dp_cp`)."""

    def __init__(self, sizes: dict[str, int], backend_device: str = "cuda"):
        self.sizes = {d: sizes.get(d, 1) for d in _DIM_ORDER}
        self.world_size = 1
        for s in self.sizes.values():
            self.world_size *= s
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.coords = self._coords_of(self.rank)
        self._groups: dict[str, object] = {}
        self.device_type = backend_device
        if dist.is_initialized():
            for name, dims in self._all_named_dims().items():
                self._groups[name] = self._make_groups(dims)

    def _coords_of(self, rank):
        coords, rem = {}, rank
        for d in reversed(_DIM_ORDER):
            coords[d] = rem % self.sizes[d]
            rem //= self.sizes[d]
        return coords

    def _rank_of(self, coords):
        r = 0
        for d in _DIM_ORDER:
            r = r * self.sizes[d] + coords[d]
        return r

    def _all_named_dims(self):
        named = {d: (d,) for d in _DIM_ORDER}
        named["dp"] = ("dp_replicate", "dp_shard")
        # Ranks that differ in cp or sp hold identical (replicated) parameters and see disjoint tokens of the same
        # batch, so FSDP shards over them and the loss is averaged over them — sp is folded in like cp.
        named["dp_shard_cp"] = ("dp_shard", "cp", "sp")
        named["dp_cp"] = ("dp_replicate", "dp_shard", "cp", "sp")
        return named

    def _make_groups(self, dims):
        """Create (collectively, on every rank) all groups varying over `dims`; return the one containing us."""
        others = [d for d in _DIM_ORDER if d not in dims]
        mine = None
        for fixed in itertools.product(*[range(self.sizes[d]) for d in others]):
            base = dict(zip(others, fixed))
            ranks = []
            for var in itertools.product(*[range(self.sizes[d]) for d in dims]):
                c = dict(base)
                c.update(dict(zip(dims, var)))
                ranks.append(self._rank_of(c))
            ranks.sort()
            g = dist.new_group(ranks) if len(ranks) < self.world_size else dist.group.WORLD
            if self.rank in ranks:
                mine = g
        return mine

    def group(self, name: str):
        return self._groups.get(name)

    def size(self, name: str) -> int:
        dims = self._all_named_dims()[name]
        n = 1
        for d in dims:
            n *= self.sizes[d]
        return n

    def local_rank(self, name: str) -> int:
        dims = self._all_named_dims()[name]
        r = 0
        for d in dims:
            r = r * self.sizes[d] + self.coords[d]
        return r

    def data_parallel_size_and_rank(self):
        """(size, rank) in the data-parallel sense: ranks that differ only in cp/sp/tp see the same batch."""
        return self.size("dp"), self.local_rank("dp")

    def __getitem__(self, name):
        return self.group(name if isinstance(name, str) else "_".join(name))

    @property
    def mesh_dim_names(self):
        return tuple(d for d in _DIM_ORDER if self.sizes[d] > 1)


@dataclass
class ParallelismConfig:
    dp_replicate_size: Optional[int] = None
    dp_shard_size: Optional[int] = None
    tp_size: Optional[int] = None
    cp_size: Optional[int] = None
    cp_backend: Optional[str] = None
    sp_size: Optional[int] = None
    sp_backend: Optional[str] = None
    tp_handler: Optional[TorchTensorParallelConfig] = None
    cp_handler: Optional[TorchContextParallelConfig] = None
    sp_handler: Optional[DeepSpeedSequenceParallelConfig] = None
    # Expert parallelism (MI355X extension; the reference reaches EP only through Megatron-LM). Experts are
    # sharded over the FSDP group (dp_shard × cp × sp), so ep_size is a sub-division, not an extra mesh dim:
    # it must be 1 or equal to that group's size.
    ep_size: Optional[int] = None
    device_mesh: Optional[RankMesh] = field(default=None, init=False)

    @property
    def ep_enabled(self):
        return (self.ep_size or 1) > 1

    def __repr__(self):
        return (
            "ParallelismConfig(\n "
            f"\tdp_replicate_size={self.dp_replicate_size},\n"
            f"\tdp_shard_size={self.dp_shard_size},\n"
            f"\ttp_size={self.tp_size},\n"
            f"\tcp_size={self.cp_size},\n"
            f"\tsp_size={self.sp_size},\n"
            f"\ttotal_size={self.total_size}\n)"
        )

    def to_json(self):
        return {
            "dp_replicate_size": self.dp_replicate_size,
            "dp_shard_size": self.dp_shard_size,
            "tp_size": self.tp_size,
            "cp_size": self.cp_size,
            "cp_backend": self.cp_backend,
            "sp_size": self.sp_size,
            "sp_backend": self.sp_backend,
        }

    @property
    def dp_dim_names(self):
        dims = []
        if self.dp_replicate_enabled:
            dims.append("dp_replicate")
        if self.dp_shard_enabled:
            dims.append("dp_shard")
        return dims

    @property
    def non_dp_dim_names(self):
        dims = []
        if self.cp_enabled:
            dims.append("cp")
        if self.sp_enabled:
            dims.append("sp")
        if self.tp_enabled:
            dims.append("tp")
        return dims

    @property
    def dp_shard_cp_dim_names(self):
        dims = []
        if self.dp_shard_enabled:
            dims.append("dp_shard")
        if self.cp_enabled:
            dims.append("cp")
        if self.sp_enabled:
            dims.append("sp")
        return dims

    @property
    def dp_cp_dim_names(self):
        return self.dp_dim_names + (["cp"] if self.cp_enabled else [])

    @property
    def fsdp_dim_names(self):
        dims = []
        if self.dp_shard_enabled:
            dims.append("dp_shard")
        if self.cp_enabled:
            dims.append("cp")
        if self.sp_enabled:
            dims.append("sp")
        return dims

    @property
    def total_size(self):
        return self.dp_replicate_size * self.dp_shard_size * self.tp_size * self.cp_size * self.sp_size

    @property
    def non_data_parallel_size(self):
        return self.tp_size * self.cp_size * self.sp_size

    @property
    def data_parallel_size(self):
        return self.dp_replicate_size * self.dp_shard_size

    @property
    def dp_replicate_enabled(self):
        return self.dp_replicate_size > 1

    @property
    def dp_shard_enabled(self):
        return self.dp_shard_size > 1

    @property
    def tp_enabled(self):
        return self.tp_size > 1

    @property
    def cp_enabled(self):
        return self.cp_size > 1

    @property
    def sp_enabled(self):
        return self.sp_size > 1

    @property
    def active_mesh_dims(self):
        return self.dp_dim_names + self.non_dp_dim_names

    def build_device_mesh(self, device_type: str = "cuda") -> RankMesh:
        mesh = RankMesh(
            {
                "dp_replicate": self.dp_replicate_size,
                "dp_shard": self.dp_shard_size,
                "cp": self.cp_size,
                "sp": self.sp_size,
                "tp": self.tp_size,
            },
            device_type,
        )
        self.device_mesh = mesh
        return mesh

    def get_device_mesh(self, device_type: Optional[str] = None):
        if self.device_mesh is None:
            if device_type is None:
                raise ValueError("You need to pass a device_type e.g cuda to build the device mesh")
            self.build_device_mesh(device_type)
        return self.device_mesh

    def __post_init__(self):
        env_prefix = "PARALLELISM_CONFIG_"
        if self.dp_replicate_size is None:
            self.dp_replicate_size = int(os.environ.get(env_prefix + "DP_REPLICATE_SIZE", "1"))
        if self.dp_shard_size is None:
            self.dp_shard_size = int(os.environ.get(env_prefix + "DP_SHARD_SIZE", "1"))
        if self.tp_size is None:
            self.tp_size = int(os.environ.get(env_prefix + "TP_SIZE", "1"))
        if self.cp_size is None:
            self.cp_size = int(os.environ.get(env_prefix + "CP_SIZE", "1"))
        if self.cp_backend is None:
            self.cp_backend = os.environ.get(env_prefix + "CP_BACKEND", "torch")
        if self.sp_size is None:
            self.sp_size = int(os.environ.get(env_prefix + "SP_SIZE", "1"))
        if self.sp_backend is None:
            self.sp_backend = os.environ.get(env_prefix + "SP_BACKEND", "deepspeed")
        if self.ep_size is None:
            self.ep_size = int(os.environ.get(env_prefix + "EP_SIZE", "1"))
        shard_group = self.dp_shard_size * self.cp_size * self.sp_size
        if self.ep_size > 1 and self.ep_size != shard_group:
            raise ValueError(f"ep_size ({self.ep_size}) must equal the FSDP shard group size dp_shard*cp*sp ({shard_group}).")
        if self.tp_size > 1 and self.tp_handler is None:
            self.tp_handler = TorchTensorParallelConfig()
        if self.cp_size > 1 and self.cp_handler is None:
            self.cp_handler = TorchContextParallelConfig()
        if self.sp_size > 1 and self.sp_handler is None:
            self.sp_handler = DeepSpeedSequenceParallelConfig()
        for name in ("dp_replicate_size", "dp_shard_size", "tp_size", "cp_size", "sp_size"):
            if getattr(self, name) < 1:
                raise ValueError(f"{name} must be at least 1, but got {getattr(self, name)}")
        if self.cp_size > 1 and self.sp_size > 1:
            raise ValueError("Context parallelism (cp_size) and sequence parallelism (sp_size) are mutually exclusive.")
        if self.cp_backend not in ("torch",):
            raise ValueError(f"cp_backend must be 'torch', got {self.cp_backend}")
        if self.sp_backend not in ("deepspeed", "native"):
            raise ValueError(f"sp_backend must be 'deepspeed' (served natively) or 'native', got {self.sp_backend}")

    def _set_size(self, parallelism: str, size: int):
        assert parallelism in ["dp_replicate", "dp_shard", "tp", "cp", "sp"]
        setattr(self, f"{parallelism}_size", size)

    def _validate_accelerator(self, accelerator):
        _warnings = set()
        if not accelerator.multi_device and self.total_size == 1:
            return
        if self.total_size != accelerator.num_processes:
            raise ValueError(
                f"ParallelismConfig total_size ({self.total_size}) does not match num_processes "
                f"({accelerator.num_processes}). Please adjust dp_replicate_size/ dp_shard_size/tp_size/cp_size/sp_size."
            )
        # MULTI_CPU is accepted too: the gloo fake cluster exercises the same mesh logic on CPU.
        if self.total_size > 1 and not (accelerator.is_fsdp2 or accelerator.multi_device or accelerator.distributed_type == "MULTI_CPU"):
            raise ValueError("ParallelismConfig is only compatible with DistributedType.FSDP (version 2), MULTI_GPU or MULTI_CPU.")
        for parallelism, size in self._sizes.items():
            if size == 1 and getattr(self, f"{parallelism}_handler", None) is not None:
                _warnings.add(f"ParallelismConfig.{parallelism}_handler is set, but {parallelism}_size is set to 1. This handler will be ignored.")
        if _warnings and accelerator.is_main_process:
            warnings.warn("ParallelismConfig has the following warnings:\n" + "\n".join(_warnings), UserWarning)

    @property
    def _sizes(self):
        return {"dp_replicate": self.dp_replicate_size, "dp_shard": self.dp_shard_size, "tp": self.tp_size, "cp": self.cp_size, "sp": self.sp_size}
