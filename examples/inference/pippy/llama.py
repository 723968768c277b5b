"""Pipeline-parallel inference of a Llama model: one stage per process, micro-batched (parity: reference
examples/inference/pippy/llama.py, which splits a HF Llama with torch.distributed.pipelining).

Here `prepare_pippy` (inference.py, runtime in parallel/pipeline.py) cuts the decoder stack at `split_points` (or balances it, "auto"), each
rank materialises only its own stage, and activations move stage to stage over point-to-point sends (RCCL on GPUs,
gloo on CPU). Weights are random-init (offline); the example checks the staged logits against the unsplit model.

    accelerate-amd launch --num_processes 2 examples/inference/pippy/llama.py            # 2 GPUs
    accelerate-amd launch --cpu --num_processes 2 examples/inference/pippy/llama.py --cpu
"""

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

from accelerate_hpc_test_amd import PartialState  # noqa: E402
from accelerate_hpc_test_amd.inference import prepare_pippy  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--preset", default=None, help="a LLAMA_PRESETS name (default: a small model sized for the test)")
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--seq", type=int, default=32)
    args = p.parse_args(argv)
    state = PartialState(cpu=args.cpu)
    W = state.num_processes
    cfg = LLAMA_PRESETS[args.preset] if args.preset else LlamaConfig(
        vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2 * W, num_attention_heads=4,
        num_key_value_heads=2, max_position_embeddings=256)
    set_seed(0)
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    model.eval()
    ids = torch.randint(0, cfg.vocab_size, (args.batch, args.seq), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = model(ids).logits if not args.preset else None  # unsplit reference (small models only)
    model = prepare_pippy(model, split_points="auto", gather_output=True, num_chunks=2)
    with torch.no_grad():
        t0 = time.perf_counter()
        out = model(ids.to(state.device))
        dt = time.perf_counter() - t0
    if ref is not None:
        err = (out.logits.float().cpu() - ref.float()).abs().max().item()
        state.print(f"stages={W} split_points={model.hf_split_points} max |staged - unsplit| = {err:.2e}")
        assert err < 1e-3, err
    state.print(f"pipeline forward of {args.batch}x{args.seq} tokens in {dt * 1e3:.1f} ms")
    state.wait_for_everyone()
    return out


if __name__ == "__main__":
    main()
