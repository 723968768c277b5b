"""FSDP2 + fp8 Llama training (the reference's headline example).

Parity: the reference's `examples/torch_native_parallelism/fsdp2_fp8.py` (torchao `Float8Linear` via
`AORecipeKwargs`, FSDP2 transformer wrap of `LlamaDecoderLayer`, AdamW lr 1e-5, seq 8192, `PerformanceTracker`).
Here the fp8 linears are this framework's `Fp8Linear` (per-tensor dynamic scaling, HIP amax/cast kernels, MX-fp8
MFMA GEMMs) and the sharding is the native FSDP engine over RCCL. Synthetic tokens, random-init weights.

    accelerate-amd launch --num_processes 8 examples/torch_native_parallelism/fsdp2_fp8.py --precision fp8
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.utils import AORecipeKwargs, set_seed  # noqa: E402
from accelerate_hpc_test_amd.utils.tracing import ThroughputTracker  # noqa: E402

WARMUP_STEPS = 10


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--sequence-length", type=int, default=8192)
    p.add_argument("--num-steps", type=int, default=1000)
    p.add_argument("--precision", default="fp8", choices=["fp8", "bf16"])
    p.add_argument("--model", default="llama3.1-8b")
    p.add_argument("--log-with", default=None)
    return p.parse_args(argv)


def main(argv=None):
    set_seed(42)
    args = parse_args(argv)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    plugin.set_mixed_precision(args.precision)
    kwargs = [AORecipeKwargs()] if args.precision == "fp8" else []
    acc = Accelerator(fsdp_plugin=plugin, mixed_precision=args.precision, kwargs_handlers=kwargs, log_with=args.log_with)
    acc.init_trackers(project_name="FSDP2_fp8", config={"sequence_length": args.sequence_length, "num_steps": args.num_steps})
    cfg = LLAMA_PRESETS[args.model]
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5)
    model, opt = acc.prepare(model, opt)
    model.train()
    g = torch.Generator().manual_seed(acc.process_index)
    tracker = ThroughputTracker(warmup_steps=min(WARMUP_STEPS, max(1, args.num_steps - 1)))
    flops = cfg.flops_per_token(args.sequence_length)
    for step in range(args.num_steps):
        ids = torch.randint(0, cfg.vocab_size, (1, args.sequence_length), generator=g).to(acc.device)
        loss = model(ids, labels=ids, return_logits=False).loss
        acc.backward(loss)
        opt.step()
        opt.zero_grad()
        metrics = tracker.step(ids.numel(), flops)
        msg = f"Step {step}/{args.num_steps}, Loss: {loss.item():.4f}"
        if "warmup_completed" in metrics:
            acc.print("Warm up completed! Starting training")
        elif metrics:
            msg += f" | {metrics['tokens_per_second']:.0f} tokens/s/device | {metrics.get('tflops_per_device', 0):.0f} TFLOP/s/device"
        if step % 10 == 0 or step == args.num_steps - 1:
            acc.print(msg)
        acc.log(metrics)
    acc.wait_for_everyone()
    acc.end_training()
    acc.print("Training completed!")


if __name__ == "__main__":
    main()
