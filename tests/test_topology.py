"""Communication-environment validation (parallel/topology.py): link-type matrix parsing, P2P / IPC
switches, strict mode."""

import pytest

from accelerate_hpc_test_amd.parallel import topology

SAMPLE = """
============================ ROCm System Management Interface ============================
=============================== Link Type between two GPUs ===============================
       GPU0         GPU1         GPU2         GPU3
GPU0   0            XGMI         XGMI         PCIE
GPU1   XGMI         0            XGMI         XGMI
GPU2   XGMI         XGMI         0            XGMI
GPU3   PCIE         XGMI         XGMI         0
================================== End of ROCm SMI Log ===================================
"""


def test_parse_link_types():
    t = topology.parse_link_types(SAMPLE)
    assert t[(0, 1)] == "XGMI" and t[(0, 3)] == "PCIE" and t[(3, 0)] == "PCIE" and (0, 0) not in t
    assert topology.parse_link_types(None) == {} and topology.parse_link_types("garbage\nlines") == {}


def test_link_problems_only_for_the_jobs_gpus():
    t = topology.parse_link_types(SAMPLE)
    assert topology.link_problems([0, 1, 2], t) == []
    probs = topology.link_problems([0, 1, 2, 3], t)
    assert len(probs) == 1 and "GPU0-GPU3" in probs[0] and "PCIE" in probs[0]


def test_environment_problems():
    assert topology.environment_problems({"HSA_ENABLE_IPC_MODE_LEGACY": "0"}) == []
    probs = topology.environment_problems({"NCCL_P2P_DISABLE": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "1",
                                           "NCCL_MAX_NCHANNELS": "4", "NCCL_P2P_LEVEL": "LOC"})
    assert len(probs) == 4


def test_validate_warns_or_raises():
    env = {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "HIP_VISIBLE_DEVICES": "0,3"}
    with pytest.warns(UserWarning, match="GPU0-GPU3"):
        probs = topology.validate_comm_environment(2, topology_text=SAMPLE, env=env)
    assert len(probs) == 1
    with pytest.raises(RuntimeError, match="not XGMI"):
        topology.validate_comm_environment(2, topology_text=SAMPLE, env=dict(env, ACCELERATE_STRICT_TOPOLOGY="1"))
    assert topology.validate_comm_environment(3, topology_text=SAMPLE, env={"HSA_ENABLE_IPC_MODE_LEGACY": "0"}) == []
