"""BERT sequence-pair classification (GLUE/MRPC shape) with the Accelerator API — BASELINE config #1.

Same training loop as the reference's `examples/nlp_example.py` (prepare → backward → gradient-accumulated step
→ gather_for_metrics evaluation), runnable on CPU (`--cpu`) or any number of MI355X ranks via
`accelerate-amd launch examples/nlp_example.py`.

Offline by construction: there is no network for `glue/mrpc` or the `bert-base-cased` checkpoint, so the data are
synthetic MRPC-shaped pairs (token ids, segment ids, padding masks; a label the model can learn: whether the two
segments share their first token) and the model is a randomly initialised `BertForSequenceClassification` with the
bert-base-cased configuration (use `--tiny` for a 2-layer model in tests). Metrics (accuracy / F1) are computed
without the `evaluate` package.
"""

import argparse
import os
import sys

import torch
from torch.utils.data import DataLoader, Dataset

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from accelerate_hpc_test_amd import Accelerator, DistributedType  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402

MAX_GPU_BATCH_SIZE = 16
EVAL_BATCH_SIZE = 32


class SyntheticMRPC(Dataset):
    """Sentence pairs of random length with a learnable paraphrase label."""

    def __init__(self, n, vocab, max_len=128, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.items = []
        for _ in range(n):
            la, lb = int(torch.randint(8, max_len // 2 - 2, (1,), generator=g)), int(torch.randint(8, max_len // 2 - 2, (1,), generator=g))
            label = int(torch.rand(1, generator=g) < 0.5)
            # "paraphrase" pairs draw both sentences from one topic band of the vocabulary, others from another
            lo, hi = (1000, 1000 + (vocab - 1000) // 2) if label else (1000 + (vocab - 1000) // 2, vocab)
            a = torch.randint(lo, hi, (la,), generator=g)
            b = torch.randint(lo, hi, (lb,), generator=g)
            ids = torch.cat([torch.tensor([101]), a, torch.tensor([102]), b, torch.tensor([102])])
            seg = torch.cat([torch.zeros(la + 2, dtype=torch.long), torch.ones(lb + 1, dtype=torch.long)])
            self.items.append({"input_ids": ids, "token_type_ids": seg, "labels": label})

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def collate_fn(examples, pad_to_multiple_of=None):
    L = max(len(e["input_ids"]) for e in examples)
    if pad_to_multiple_of:
        L = -(-L // pad_to_multiple_of) * pad_to_multiple_of
    ids = torch.zeros(len(examples), L, dtype=torch.long)
    seg = torch.zeros_like(ids)
    mask = torch.zeros_like(ids)
    for i, e in enumerate(examples):
        n = len(e["input_ids"])
        ids[i, :n], seg[i, :n], mask[i, :n] = e["input_ids"], e["token_type_ids"], 1
    return {"input_ids": ids, "token_type_ids": seg, "attention_mask": mask, "labels": torch.tensor([e["labels"] for e in examples])}


def get_dataloaders(accelerator: Accelerator, batch_size: int = 16, vocab: int = 28996, n_train: int = 3668, n_eval: int = 408):
    with accelerator.main_process_first():
        train, evals = SyntheticMRPC(n_train, vocab, seed=0), SyntheticMRPC(n_eval, vocab, seed=1)
    pad = 16 if accelerator.mixed_precision == "fp8" else (8 if accelerator.mixed_precision != "no" else None)
    col = lambda ex: collate_fn(ex, pad)  # noqa: E731
    train_dl = DataLoader(train, shuffle=True, collate_fn=col, batch_size=batch_size, drop_last=accelerator.mixed_precision == "fp8")
    eval_dl = DataLoader(evals, shuffle=False, collate_fn=col, batch_size=EVAL_BATCH_SIZE, drop_last=accelerator.mixed_precision == "fp8")
    return train_dl, eval_dl


def build_model(tiny: bool):
    from transformers import BertConfig, BertForSequenceClassification

    cfg = BertConfig(vocab_size=28996, num_labels=2)  # bert-base-cased shape
    if tiny:
        cfg.num_hidden_layers, cfg.hidden_size, cfg.num_attention_heads, cfg.intermediate_size = 2, 128, 2, 256
    return BertForSequenceClassification(cfg)


def binary_metrics(preds, refs):
    preds, refs = preds.long(), refs.long()
    acc = (preds == refs).float().mean().item()
    tp = ((preds == 1) & (refs == 1)).sum().item()
    fp = ((preds == 1) & (refs == 0)).sum().item()
    fn = ((preds == 0) & (refs == 1)).sum().item()
    f1 = 2 * tp / max(1, 2 * tp + fp + fn)
    return {"accuracy": acc, "f1": f1}


def training_function(config, args):
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    lr, num_epochs, seed, batch_size = config["lr"], int(config["num_epochs"]), int(config["seed"]), int(config["batch_size"])
    gradient_accumulation_steps = 1
    if batch_size > MAX_GPU_BATCH_SIZE and accelerator.distributed_type != DistributedType.NO:
        gradient_accumulation_steps = batch_size // MAX_GPU_BATCH_SIZE
        batch_size = MAX_GPU_BATCH_SIZE
    set_seed(seed)
    train_dl, eval_dl = get_dataloaders(accelerator, batch_size, n_train=args.n_train, n_eval=args.n_eval)
    model = build_model(args.tiny).to(accelerator.device)
    optimizer = torch.optim.AdamW(params=model.parameters(), lr=lr)
    total = (len(train_dl) * num_epochs) // gradient_accumulation_steps
    warmup = min(100, max(1, total // 10))  # linear warmup then linear decay (get_linear_schedule_with_warmup)
    lr_scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lambda s: min(1.0, (s + 1) / warmup) * max(0.0, 1 - s / max(1, total)))
    model, optimizer, train_dl, eval_dl, lr_scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, lr_scheduler)
    metric = None
    for epoch in range(num_epochs):
        model.train()
        for step, batch in enumerate(train_dl):
            outputs = model(**batch)
            loss = outputs.loss / gradient_accumulation_steps
            accelerator.backward(loss)
            if step % gradient_accumulation_steps == 0:
                optimizer.step()
                lr_scheduler.step()
                optimizer.zero_grad()
        model.eval()
        all_p, all_r = [], []
        for batch in eval_dl:
            with torch.no_grad():
                outputs = model(**batch)
            predictions = outputs.logits.argmax(dim=-1)
            predictions, references = accelerator.gather_for_metrics((predictions, batch["labels"]))
            all_p.append(predictions.cpu())
            all_r.append(references.cpu())
        metric = binary_metrics(torch.cat(all_p), torch.cat(all_r))
        accelerator.print(f"epoch {epoch}:", metric)
    accelerator.end_training()
    return metric


def main(argv=None):
    parser = argparse.ArgumentParser(description="Simple example of a training script (synthetic MRPC, random-init BERT).")
    parser.add_argument("--mixed_precision", type=str, default=None, choices=["no", "fp16", "bf16", "fp8"])
    parser.add_argument("--cpu", action="store_true", help="If passed, will train on the CPU.")
    parser.add_argument("--tiny", action="store_true", help="2-layer BERT (tests / smoke runs).")
    parser.add_argument("--num_epochs", type=int, default=3)
    parser.add_argument("--n_train", type=int, default=3668)
    parser.add_argument("--n_eval", type=int, default=408)
    args = parser.parse_args(argv)
    config = {"lr": 2e-5 if not args.tiny else 1e-3, "num_epochs": args.num_epochs, "seed": 42, "batch_size": 16}
    return training_function(config, args)


if __name__ == "__main__":
    main()
