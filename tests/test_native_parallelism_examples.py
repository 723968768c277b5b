"""examples/torch_native_parallelism/nd_parallel.py on the CPU fake cluster: every parallel dimension the reference's
nd_parallel example exposes (dp_shard / HSDP, tp, cp) trains the toy Llama and its loss falls."""

import os
import sys

import pytest

from accelerate_hpc_test_amd import debug_launcher

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "examples", "torch_native_parallelism"))

import nd_parallel  # noqa: E402

BASE = ["--cpu", "--tiny", "--num-steps", "8", "--sequence-length", "64"]


def _run(argv):
    losses = nd_parallel.main(argv)
    assert losses[-1] < losses[0], losses


def test_nd_parallel_single_process():
    _run(BASE)


@pytest.mark.parametrize(
    "dims",
    [["--dp-shard-size", "2"], ["--tp-size", "2"], ["--cp-size", "2"], ["--dp-replicate-size", "2"],
     ["--tp-size", "2", "--hf"]],
    ids=["fsdp", "tp", "cp", "hsdp_replicate", "tp_hf_tp_plan"],
)
def test_nd_parallel_two_ranks(dims):
    debug_launcher(_run, args=(BASE + dims,), num_processes=2)
