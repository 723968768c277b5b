"""Communication-environment validation for one MI355X node.

An 8×MI355X node is a fully connected xGMI mesh (7 point-to-point links per GPU). RCCL's all-gather / reduce-scatter
/ all-to-all reach their bandwidth only when every pair of the job's local GPUs is linked by xGMI and peer-to-peer is
not disabled; the HIP-IPC small all-reduce (parallel/small_allreduce.py) and CUDA-tensor sharing need dmabuf IPC.
The reference does no topology work beyond switching P2P off on RTX 40xx (`/root/reference/src/accelerate/utils/
environment.py:197-223`); here every rank's local view is checked once at start-up and problems are reported (or
raised with ACCELERATE_STRICT_TOPOLOGY=1):

* link type of every local GPU pair (`rocm-smi --showtopotype`): anything but XGMI means ring steps over PCIe;
* environment switches that silently cost bandwidth or break IPC: NCCL_P2P_DISABLE / NCCL_SHM_DISABLE /
  NCCL_P2P_LEVEL=LOC, HSA_ENABLE_IPC_MODE_LEGACY != 0, a RCCL channel cap below the link count.
The HIP-IPC all-reduce additionally self-tests its peer mappings at setup (parallel/small_allreduce.py).
"""

from __future__ import annotations

import os
import re
import warnings
from typing import Optional

from ..utils.environment import get_xgmi_topology

_LINKS_PER_GPU = 7  # MI355X: one xGMI link to each of the 7 peers


def parse_link_types(text: Optional[str]) -> dict:
    """{(i, j): link type} from `rocm-smi --showtopotype` (the "Link Type between two GPUs" matrix); {} if absent."""
    if not text:
        return {}
    types, header = {}, None
    for line in text.splitlines():
        toks = line.split()
        if not toks:
            continue
        if all(re.fullmatch(r"GPU\d+", t) for t in toks):
            header = [int(t[3:]) for t in toks]
            continue
        if header and re.fullmatch(r"GPU\d+", toks[0]) and len(toks) == len(header) + 1:
            i = int(toks[0][3:])
            for j, t in zip(header, toks[1:]):
                if i != j:
                    types[(i, j)] = t.upper()
    return types


def environment_problems(env=None) -> list:
    """Settings that cost xGMI bandwidth or break HIP IPC (strings, empty when clean)."""
    env = os.environ if env is None else env
    out = []
    if env.get("NCCL_P2P_DISABLE", "0") not in ("0", ""):
        out.append("NCCL_P2P_DISABLE is set: RCCL stops using direct xGMI peer transfers")
    if env.get("NCCL_SHM_DISABLE", "0") not in ("0", ""):
        out.append("NCCL_SHM_DISABLE is set")
    if env.get("NCCL_P2P_LEVEL", "").upper() == "LOC":
        out.append("NCCL_P2P_LEVEL=LOC disables peer-to-peer between GPUs")
    if env.get("HSA_ENABLE_IPC_MODE_LEGACY") not in (None, "0"):
        out.append("HSA_ENABLE_IPC_MODE_LEGACY must be 0 (dmabuf IPC) for RCCL peer buffers and the HIP-IPC all-reduce")
    for key in ("NCCL_MAX_NCHANNELS", "NCCL_MAX_CHANNELS"):
        v = env.get(key)
        if v is not None and v.isdigit() and int(v) < _LINKS_PER_GPU:
            out.append(f"{key}={v} caps RCCL below one channel per xGMI link ({_LINKS_PER_GPU})")
    return out


def link_problems(local_devices: list, types: dict) -> list:
    """Pairs of the job's local GPUs that are not linked by xGMI."""
    out = []
    for a in local_devices:
        for b in local_devices:
            if a < b:
                t = types.get((a, b)) or types.get((b, a))
                if t is not None and t != "XGMI":
                    out.append(f"GPU{a}-GPU{b} link type {t} (not XGMI): collectives between them cross {t}")
    return out


def _physical_devices(local_world: int, env) -> list:
    vis = env.get("HIP_VISIBLE_DEVICES") or env.get("ROCR_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    if vis:
        ids = [int(x) for x in vis.split(",") if x.strip().isdigit()]
        return ids[:local_world]
    return list(range(local_world))


def validate_comm_environment(local_world: int, topology_text: Optional[str] = None, strict: Optional[bool] = None,
                              env=None) -> list:
    """Check this node's communication setup for a job with `local_world` ranks on it (one GPU each). Returns the
    problems found; warns about them, or raises with `strict` (default: ACCELERATE_STRICT_TOPOLOGY=1)."""
    env = os.environ if env is None else env
    if strict is None:
        strict = env.get("ACCELERATE_STRICT_TOPOLOGY", "0") == "1"
    problems = environment_problems(env)
    if local_world > 1:
        text = topology_text if topology_text is not None else get_xgmi_topology()
        problems += link_problems(_physical_devices(local_world, env), parse_link_types(text))
    if problems:
        msg = "communication environment: " + "; ".join(problems)
        if strict:
            raise RuntimeError(msg)
        warnings.warn(msg)
    return problems
