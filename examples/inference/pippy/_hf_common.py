"""Shared driver of the transformers pippy examples (bert.py, gpt2.py, t5.py): build the model from its config with
random weights (offline: no Hub checkpoint), split it over the processes with `prepare_pippy`, run one micro-batched
forward and compare the last stage's logits (gathered to every rank) with the unsplit model."""

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

from accelerate_hpc_test_amd import PartialState  # noqa: E402
from accelerate_hpc_test_amd.inference import prepare_pippy  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def run(build, argv=None):
    """`build(full: bool) -> (model, inputs)`: the example's model (full-size config with `--full`, else a small one
    sized for the tests) and its example inputs (batch first)."""
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--full", action="store_true", help="the reference example's model size (random weights)")
    args = p.parse_args(argv)
    state = PartialState(cpu=args.cpu)
    set_seed(0)
    model, inputs = build(args.full)
    model.eval()
    ref = None
    if not args.full:
        with torch.no_grad():
            ref = model(**inputs).logits
    model = prepare_pippy(model, split_points="auto", gather_output=True, num_chunks=2)
    inputs = {k: v.to(state.device) for k, v in inputs.items()}
    with torch.no_grad():
        t0 = time.perf_counter()
        out = model(**inputs)
        dt = time.perf_counter() - t0
    if ref is not None:
        err = (out.logits.float().cpu() - ref.float()).abs().max().item()
        state.print(f"{type(model).__name__}: stages={state.num_processes} split_points={model.hf_split_points} "
                    f"max |staged - unsplit| = {err:.2e}")
        assert err < 1e-3, err
    state.print(f"pipeline forward in {dt * 1e3:.1f} ms")
    state.wait_for_everyone()
    return out
