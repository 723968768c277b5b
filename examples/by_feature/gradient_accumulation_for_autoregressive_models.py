"""Token-correct gradient accumulation for causal LMs (reference:
examples/by_feature/gradient_accumulation_for_autoregressive_models.py).

Averaging per-micro-batch mean losses over-weights short sequences. Instead the loop counts the non-padded target
tokens of the whole accumulation window on every rank, all-reduces that count (`accelerator.reduce`), and sums the
per-token losses divided by the global count — scaled by `num_processes × gradient_accumulation_steps` to undo
the averaging that the gradient all-reduce and `backward` apply. Uses this framework's Llama (random init, synthetic
variable-length sequences).
"""

from _shared import base_parser  # noqa: I001  (also puts the repo on sys.path)

import torch
import torch.nn.functional as F

from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM
from accelerate_hpc_test_amd.utils import set_seed


def main(argv=None):
    p = base_parser("Token-normalised gradient accumulation (causal LM)")
    p.add_argument("--gradient_accumulation_steps", type=int, default=4)
    p.add_argument("--seq_len", type=int, default=128)
    p.add_argument("--steps", type=int, default=8)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision,
                              gradient_accumulation_steps=args.gradient_accumulation_steps)
    set_seed(0)
    cfg = LLAMA_PRESETS["llama-tiny"]
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr or 1e-3)
    model, optimizer = accelerator.prepare(model, optimizer)
    g = torch.Generator().manual_seed(accelerator.process_index)
    losses = []
    for step in range(args.steps):
        window = []
        for _ in range(args.gradient_accumulation_steps):
            ids = torch.randint(0, cfg.vocab_size, (2, args.seq_len), generator=g)
            lengths = torch.randint(args.seq_len // 4, args.seq_len, (2,), generator=g)
            labels = ids.clone()
            for i, n in enumerate(lengths.tolist()):
                labels[i, n:] = -100
            window.append((ids.to(accelerator.device), labels.to(accelerator.device)))
        local = sum(int((lab[:, 1:] != -100).sum()) for _, lab in window)
        n_tokens = accelerator.reduce(torch.tensor(local, device=accelerator.device), reduction="sum").item()
        total = 0.0
        for ids, labels in window:
            with accelerator.accumulate(model):
                logits = model(ids).logits.float()
                loss = F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), labels[:, 1:].reshape(-1),
                                       ignore_index=-100, reduction="sum") / n_tokens
                total += loss.item()
                accelerator.backward(loss * accelerator.num_processes * args.gradient_accumulation_steps)
                optimizer.step()
                optimizer.zero_grad()
        losses.append(accelerator.reduce(torch.tensor(total, device=accelerator.device), reduction="sum").item())
        accelerator.print(f"step {step}: loss per token {losses[-1]:.4f} over {int(n_tokens)} tokens")
    accelerator.end_training()
    return losses


if __name__ == "__main__":
    main()
