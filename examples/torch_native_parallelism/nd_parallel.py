"""N-d parallel Llama training: dp_replicate × dp_shard × cp × tp through `ParallelismConfig`.

Parity: the reference's `examples/torch_native_parallelism/nd_parallel.py` (HSDP + TP via transformers' `tp_plan`,
CP via `maybe_context_parallel`). Here every dimension is this framework's own: FSDP engine over dp_shard(×cp), HSDP
all-reduce over dp_replicate, Megatron-style TP layers, ring attention for CP — all on RCCL (gloo on CPU).
Synthetic tokens and random-init weights (no network).

    accelerate-amd launch --num_processes 8 examples/torch_native_parallelism/nd_parallel.py --dp-shard-size 4 --tp-size 2
    python examples/torch_native_parallelism/nd_parallel.py --cpu --tiny          # single process smoke run
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin, ParallelismConfig  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402
from accelerate_hpc_test_amd.utils.tracing import ThroughputTracker  # noqa: E402

TINY = LlamaConfig(vocab_size=128, hidden_size=64, intermediate_size=96, num_hidden_layers=2, num_attention_heads=4,
                   num_key_value_heads=2, max_position_embeddings=256)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--dp-replicate-size", type=int, default=1)
    p.add_argument("--dp-shard-size", type=int, default=1)
    p.add_argument("--tp-size", type=int, default=1)
    p.add_argument("--cp-size", type=int, default=1)
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--sequence-length", type=int, default=4096)
    p.add_argument("--num-steps", type=int, default=20)
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--tiny", action="store_true", help="2-layer toy Llama (CPU smoke runs / tests)")
    p.add_argument("--hf", action="store_true",
                   help="a transformers LlamaForCausalLM (as the reference example loads), TP-sharded by its own tp_plan")
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    pc = ParallelismConfig(dp_replicate_size=args.dp_replicate_size, dp_shard_size=args.dp_shard_size,
                           tp_size=args.tp_size, cp_size=args.cp_size)
    plugin = None
    if args.dp_shard_size * args.cp_size > 1 or args.dp_replicate_size > 1:
        plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                                transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(cpu=args.cpu, parallelism_config=pc, fsdp_plugin=plugin,
                      mixed_precision="no" if args.cpu else "bf16")
    set_seed(42)
    cfg = TINY if args.tiny else LLAMA_PRESETS[args.model]
    seq = min(args.sequence_length, cfg.max_position_embeddings) if args.tiny else args.sequence_length
    if args.hf:
        import transformers as tf

        hcfg = tf.LlamaConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                              num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                              num_key_value_heads=cfg.num_key_value_heads, max_position_embeddings=cfg.max_position_embeddings)
        model = tf.LlamaForCausalLM(hcfg)
        if args.dp_shard_size * args.cp_size > 1 or args.dp_replicate_size > 1:
            plugin.transformer_cls_names_to_wrap = ["LlamaDecoderLayer"]
    elif args.cpu:
        model = LlamaForCausalLM(cfg)
        model.init_weights()
    else:
        with torch.device("meta"):
            model = LlamaForCausalLM(cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=(1e-3 if args.hf else 1e-4) if args.tiny else 1e-5)
    model, opt = acc.prepare(model, opt)
    # every rank of one data-parallel replica sees the same batch; TP / CP ranks split the work inside it
    dp_rank = acc.process_index // (args.tp_size * args.cp_size)
    g = torch.Generator().manual_seed(1000 + dp_rank)
    tracker = ThroughputTracker(warmup_steps=min(5, max(1, args.num_steps - 1)))
    losses = []
    for step in range(args.num_steps):
        if args.tiny and step % 2 == 0:  # tiny runs revisit two batches so a falling loss shows learning
            g.manual_seed(1000 + dp_rank)
        ids = torch.randint(0, cfg.vocab_size, (1, seq), generator=g).to(acc.device)
        labels = ids.clone()
        if args.cp_size > 1:
            with acc.maybe_context_parallel(buffers=[ids, labels], buffer_seq_dims=[1, 1], no_restore_buffers={ids, labels}):
                loss = model(ids, shift_labels=labels).loss
                acc.backward(loss)
        else:
            loss = model(input_ids=ids, labels=labels).loss
            acc.backward(loss)
        opt.step()
        opt.zero_grad()
        loss = acc.reduce(loss.detach().reshape(1), reduction="mean")
        losses.append(loss.item())
        metrics = tracker.step(ids.numel(), cfg.flops_per_token(seq))
        if step % 5 == 0 or step == args.num_steps - 1:
            extra = f" | {metrics['tokens_per_second']:.0f} tok/s/rank" if "tokens_per_second" in metrics else ""
            acc.print(f"step {step} loss {losses[-1]:.4f}{extra}")
    acc.end_training()
    return losses


if __name__ == "__main__":
    main()
