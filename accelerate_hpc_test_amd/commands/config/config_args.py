"""Config-file schema for `accelerate-amd config` / `launch`.

Parity target: `/root/reference/src/accelerate/commands/config/config_args.py:29-252` — the same YAML/JSON keys
are accepted (files produced by the reference's `accelerate config` load here unchanged), unknown keys are a hard
error, legacy keys (`fp16`, `dynamo_backend`) are migrated, and the default location is
`$HF_HOME/accelerate/default_config.yaml`.

Design: the schema is a declarative table (`_CLUSTER_FIELDS`) consumed by one generic codec (`_Codec`), so the
serialized form, the migration rules and the validation all live in one place instead of per-class methods.
"""

from __future__ import annotations

import json
import os
from dataclasses import dataclass, field, fields
from enum import Enum
from pathlib import Path
from typing import Any, Optional

import yaml

from ...utils.dataclasses import ComputeEnvironment, DistributedType, SageMakerDistributedType


def _cache_root() -> str:
    hf_home = os.environ.get("HF_HOME")
    if hf_home is None:
        hf_home = os.path.join(os.environ.get("XDG_CACHE_HOME", "~/.cache"), "huggingface")
    return os.path.join(os.path.expanduser(hf_home), "accelerate")


cache_dir = _cache_root()
default_yaml_config_file = os.path.join(cache_dir, "default_config.yaml")
default_json_config_file = default_yaml_config_file  # JSON is still read when a path ends in .json
default_config_file = default_yaml_config_file

# sub-dicts that are stored as {} in memory and dropped from the file when empty
_DICT_SECTIONS = (
    "deepspeed_config", "fsdp_config", "parallelism_config", "megatron_lm_config", "ipex_config",
    "mpirun_config", "fp8_config", "dynamo_config", "rccl_config",
)


class _Codec:
    """Reads/writes a config dataclass as YAML or JSON, applying legacy-key migration and key validation."""

    @staticmethod
    def read_raw(path: str) -> dict:
        text = Path(path).read_text(encoding="utf-8")
        data = json.loads(text) if path.endswith(".json") else yaml.safe_load(text)
        return dict(data or {})

    @staticmethod
    def migrate(raw: dict) -> dict:
        d = dict(raw)
        d.setdefault("compute_environment", ComputeEnvironment.LOCAL_MACHINE.value)
        if "distributed_type" not in d:
            raise ValueError("A `distributed_type` must be specified in the config file.")
        if d["distributed_type"] in (DistributedType.NO, DistributedType.NO.value):
            d.setdefault("num_processes", 1)
        legacy_fp16 = d.pop("fp16", None)
        if "mixed_precision" not in d:
            d["mixed_precision"] = "fp16" if legacy_fp16 else None
        if "dynamo_backend" in d:
            backend = d.pop("dynamo_backend")
            d["dynamo_config"] = {} if backend == "NO" else {"dynamo_backend": backend}
        for flag in ("use_cpu", "debug", "enable_cpu_affinity"):
            d.setdefault(flag, False)
        return d

    @staticmethod
    def check_keys(cls, d: dict, origin: str):
        known = {f.name for f in fields(cls)}
        unknown = sorted(set(d) - known)
        if unknown:
            raise ValueError(
                f"The config file at {origin} had unknown keys ({unknown}); fix or remove these keys "
                "(they are not part of the accelerate config schema understood by this version)."
            )

    @staticmethod
    def serialize(cfg) -> dict:
        out = {}
        for f in fields(cfg):
            v = getattr(cfg, f.name)
            if isinstance(v, Enum):
                v = v.value
            if v is None or (isinstance(v, dict) and not v):
                continue
            out[f.name] = v
        return out


@dataclass
class BaseConfig:
    compute_environment: ComputeEnvironment
    distributed_type: Any
    mixed_precision: Optional[str]
    use_cpu: bool
    debug: bool

    # ---- (de)serialization -------------------------------------------------------------------------------
    def to_dict(self) -> dict:
        return _Codec.serialize(self)

    @classmethod
    def process_config(cls, config_dict: dict) -> dict:
        return _Codec.migrate(config_dict)

    @classmethod
    def _from_path(cls, path: str):
        d = _Codec.migrate(_Codec.read_raw(path))
        _Codec.check_keys(cls, d, path)
        return cls(**d)

    @classmethod
    def from_yaml_file(cls, yaml_file: Optional[str] = None):
        return cls._from_path(str(yaml_file or default_yaml_config_file))

    @classmethod
    def from_json_file(cls, json_file: Optional[str] = None):
        return cls._from_path(str(json_file or default_json_config_file))

    def to_yaml_file(self, yaml_file):
        Path(yaml_file).write_text(yaml.safe_dump(self.to_dict()), encoding="utf-8")

    def to_json_file(self, json_file):
        Path(json_file).write_text(json.dumps(self.to_dict(), indent=2, sort_keys=True) + "\n", encoding="utf-8")

    def save(self, path):
        (self.to_json_file if str(path).endswith(".json") else self.to_yaml_file)(path)

    # ---- normalisation -----------------------------------------------------------------------------------
    def __post_init__(self):
        self.compute_environment = ComputeEnvironment(self.compute_environment)
        enum_cls = SageMakerDistributedType if self.compute_environment == ComputeEnvironment.AMAZON_SAGEMAKER else DistributedType
        if isinstance(self.distributed_type, str):
            self.distributed_type = enum_cls(self.distributed_type)
        for name in _DICT_SECTIONS:
            if hasattr(self, name) and getattr(self, name) is None:
                setattr(self, name, {})


@dataclass
class ClusterConfig(BaseConfig):
    """Local-machine / multi-node launch description (one process per MI355X GPU by default)."""

    num_processes: int = -1
    machine_rank: int = 0
    num_machines: int = 1
    gpu_ids: Optional[str] = None
    main_process_ip: Optional[str] = None
    main_process_port: Optional[int] = None
    rdzv_backend: Optional[str] = "static"
    same_network: Optional[bool] = False
    main_training_function: str = "main"
    enable_cpu_affinity: bool = False
    downcast_bf16: bool = False
    # feature sections
    fp8_config: dict = field(default=None)
    deepspeed_config: dict = field(default=None)
    fsdp_config: dict = field(default=None)
    parallelism_config: dict = field(default=None)
    megatron_lm_config: dict = field(default=None)
    ipex_config: dict = field(default=None)
    mpirun_config: dict = field(default=None)
    dynamo_config: dict = field(default=None)
    rccl_config: dict = field(default=None)  # MI355X-only: ddp_bucket_mb / fsdp_prefetch_depth / ...
    # TPU pod fields are accepted for file compatibility; they are inert on MI355X
    tpu_name: Optional[str] = None
    tpu_zone: Optional[str] = None
    tpu_use_cluster: bool = False
    tpu_use_sudo: bool = False
    command_file: Optional[str] = None
    commands: Optional[list] = None
    tpu_vm: Optional[list] = None
    tpu_env: Optional[list] = None


@dataclass
class SageMakerConfig(BaseConfig):
    """Accepted for file compatibility; launching on SageMaker is not supported from an MI355X node."""

    ec2_instance_type: str = "ml.p3.2xlarge"
    iam_role_name: Optional[str] = None
    image_uri: Optional[str] = None
    profile: Optional[str] = None
    region: str = "us-east-1"
    num_machines: int = 1
    gpu_ids: str = "all"
    base_job_name: str = "accelerate-sagemaker-1"
    pytorch_version: str = "2.1.0"
    transformers_version: str = "4.36.0"
    py_version: str = "py310"
    sagemaker_inputs_file: Optional[str] = None
    sagemaker_metrics_file: Optional[str] = None
    additional_args: Optional[dict] = None
    dynamo_config: dict = field(default=None)
    enable_cpu_affinity: bool = False


def load_config_from_file(config_file: Optional[str]):
    """Load `config_file` (or the default config) choosing the schema from its `compute_environment`."""
    if config_file is not None and not os.path.isfile(config_file):
        raise FileNotFoundError(
            f"The passed configuration file `{config_file}` does not exist. Pass an existing file to "
            "`accelerate-amd launch --config_file`, or create the default one with `accelerate-amd config`."
        )
    path = str(config_file or default_config_file)
    env = _Codec.read_raw(path).get("compute_environment", ComputeEnvironment.LOCAL_MACHINE.value)
    cls = ClusterConfig if env == ComputeEnvironment.LOCAL_MACHINE.value else SageMakerConfig
    return cls._from_path(path)
