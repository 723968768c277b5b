"""Long-sequence training with Ulysses sequence parallelism (parity: reference
examples/alst_ulysses_sequence_parallelism/sp-alst.py, which drives DeepSpeed ALST through `ParallelismConfig(sp_size,
sp_backend="deepspeed")`).

Here `ParallelismConfig(sp_size=N)` with the native FSDP2 engine: the prepared data loader hands every rank a
1/N slice of each sequence (plus its global `position_ids`), attention all-to-alls heads <-> sequence around the HIP
flash-attention kernel (parallel/ulysses.py), and the loss is averaged over the sp group. Labels are shifted on the
full sequence before sharding (`shift_labels`), as in the reference.

    accelerate-amd launch --num_processes 8 examples/alst_ulysses_sequence_parallelism/sp_ulysses.py --seq 65536
    accelerate-amd launch --cpu --num_processes 2 examples/alst_ulysses_sequence_parallelism/sp_ulysses.py --cpu
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin, ParallelismConfig  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--preset", default=None)
    p.add_argument("--seq", type=int, default=64)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--lr", type=float, default=1e-3)
    args = p.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    pc = ParallelismConfig(sp_size=world) if world > 1 else None
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(cpu=args.cpu, parallelism_config=pc, fsdp_plugin=plugin,
                      mixed_precision="no" if args.cpu else "bf16")
    cfg = LLAMA_PRESETS[args.preset] if args.preset else LlamaConfig(
        vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, max_position_embeddings=max(256, args.seq))
    set_seed(0)
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr)
    g = torch.Generator().manual_seed(5)
    data = []
    for _ in range(args.steps):
        ids = torch.randint(0, cfg.vocab_size, (args.seq,), generator=g)
        data.append({"input_ids": ids, "shift_labels": torch.cat([ids[1:], torch.tensor([-100])])})
    dl = torch.utils.data.DataLoader(data, batch_size=1)
    model, opt, dl = acc.prepare(model, opt, dl)
    losses = []
    for batch in dl:
        kw = {"position_ids": batch["position_ids"]} if "position_ids" in batch else {}
        out = model(batch["input_ids"], shift_labels=batch["shift_labels"], **kw)
        acc.backward(out.loss)
        opt.step()
        opt.zero_grad()
        losses.append(acc.reduce(out.loss.detach().reshape(1), reduction="mean").item())
        acc.print(f"step {len(losses)}: local tokens {batch['input_ids'].shape[-1]} of {args.seq}, loss {losses[-1]:.4f}")
    acc.end_training()
    return losses


if __name__ == "__main__":
    main()
