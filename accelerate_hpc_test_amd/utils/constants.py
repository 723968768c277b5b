"""File names and tunables shared across the framework.

The checkpoint file names are part of the public contract: a checkpoint written by the reference
(`/root/reference/src/accelerate/utils/constants.py:19-33`) must be readable here and vice versa,
so the names are kept identical. The RCCL / xGMI tunables below are MI355X-specific additions.
"""

SCALER_NAME = "scaler.pt"
MODEL_NAME = "pytorch_model"
SAFE_MODEL_NAME = "model"
RNG_STATE_NAME = "random_states"
OPTIMIZER_NAME = "optimizer"
SCHEDULER_NAME = "scheduler"
SAMPLER_NAME = "sampler"
DATALOADER_STATE_NAME = "dl_state_dict"
PROFILE_PATTERN_NAME = "profile_{suffix}.json"
WEIGHTS_NAME = f"{MODEL_NAME}.bin"
WEIGHTS_PATTERN_NAME = "pytorch_model{suffix}.bin"
WEIGHTS_INDEX_NAME = f"{WEIGHTS_NAME}.index.json"
SAFE_WEIGHTS_NAME = f"{SAFE_MODEL_NAME}.safetensors"
SAFE_WEIGHTS_PATTERN_NAME = "model{suffix}.safetensors"
SAFE_WEIGHTS_INDEX_NAME = f"{SAFE_WEIGHTS_NAME}.index.json"
CUSTOM_CHECKPOINT_NAME = "custom_checkpoint_{i}.pkl"
FSDP_MODEL_NAME = "pytorch_model_fsdp"
FSDP_SHARD_INDEX_NAME = "shard_index.json"

# FSDP plugin vocabularies (same strings as the reference so YAML configs are portable).
FSDP_SHARDING_STRATEGY = ["FULL_SHARD", "SHARD_GRAD_OP", "NO_SHARD", "HYBRID_SHARD", "HYBRID_SHARD_ZERO2"]
FSDP_AUTO_WRAP_POLICY = ["TRANSFORMER_BASED_WRAP", "SIZE_BASED_WRAP", "NO_WRAP"]
FSDP_BACKWARD_PREFETCH = ["BACKWARD_PRE", "BACKWARD_POST", "NO_PREFETCH"]
FSDP_STATE_DICT_TYPE = ["FULL_STATE_DICT", "LOCAL_STATE_DICT", "SHARDED_STATE_DICT"]
FSDP2_STATE_DICT_TYPE = ["SHARDED_STATE_DICT", "FULL_STATE_DICT"]
FSDP_PYTORCH_VERSION = "2.1.0"
FSDP2_PYTORCH_VERSION = "2.6.0"

# torchrun arguments forwarded by `accelerate launch`.
TORCH_LAUNCH_PARAMS = [
    "nnodes",
    "nproc_per_node",
    "rdzv_backend",
    "rdzv_endpoint",
    "rdzv_id",
    "rdzv_conf",
    "standalone",
    "max_restarts",
    "monitor_interval",
    "start_method",
    "role",
    "module",
    "m",
    "no_python",
    "run_path",
    "log_dir",
    "r",
    "redirects",
    "t",
    "tee",
    "node_rank",
    "master_addr",
    "master_port",
]

ELASTIC_LOG_LINE_PREFIX_TEMPLATE_PYTORCH_VERSION = "2.2.0"

# ---------------------------------------------------------------------------------------------
# MI355X / xGMI tunables (env overridable, see utils/environment.py::get_int_from_env).
# ---------------------------------------------------------------------------------------------
# 8 x MI355X are fully connected by 7 point-to-point xGMI links of ~153 GB/s each. A single ring
# only drives one link per direction, so per-collective messages must be large enough that RCCL's
# multi-channel algorithms keep all 7 links busy: >= 8 MB per peer at world size 8.
DEFAULT_DDP_BUCKET_MB = 128
# FSDP gathers one transformer block per collective (~436 MB bf16 for a Llama-3-8B block), so no
# bucketing is needed; small units are coalesced up to this size.
DEFAULT_FSDP_MIN_UNIT_MB = 32
# Messages below this are latency bound (tens of us per RCCL launch); they are coalesced into a
# single flat collective (see utils/operations.py: reduce/gather of tensor lists).
SMALL_COLLECTIVE_BYTES = 1 << 20
# MI355X HBM per device (bytes) used by the device-map planner when the device cannot be queried.
MI355X_HBM_BYTES = 288 * (1 << 30)
