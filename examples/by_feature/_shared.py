"""Shared scaffolding for the by_feature examples: the synthetic-MRPC data and random-init BERT of
`examples/nlp_example.py`, a common CLI, and the train / evaluate loops each feature example decorates.

Parity: the reference's `examples/by_feature/*.py` each copy `nlp_example.py` and add one feature
(`/root/reference/examples/by_feature/`). Here the copy lives once, below, and every example file shows only its
feature (offline: synthetic data, random-init model — there is no network for GLUE or checkpoints).
"""

import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))  # examples/ (nlp_example)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root (the package)

import nlp_example  # noqa: E402

from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def base_parser(description: str) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--mixed_precision", type=str, default=None, choices=["no", "fp16", "bf16", "fp8"])
    p.add_argument("--cpu", action="store_true", help="train on the CPU")
    p.add_argument("--tiny", action="store_true", help="2-layer BERT (tests / smoke runs)")
    p.add_argument("--num_epochs", type=int, default=3)
    p.add_argument("--n_train", type=int, default=3668)
    p.add_argument("--n_eval", type=int, default=408)
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--lr", type=float, default=None)
    return p


def build(accelerator, args, batch_size=None, seed: int = 42):
    """(model, optimizer, train_dl, eval_dl, scheduler) — NOT yet prepared."""
    set_seed(seed)
    train_dl, eval_dl = nlp_example.get_dataloaders(accelerator, batch_size or args.batch_size, n_train=args.n_train, n_eval=args.n_eval)
    model = nlp_example.build_model(args.tiny)
    lr = args.lr if args.lr is not None else (1e-3 if args.tiny else 2e-5)
    optimizer = torch.optim.AdamW(model.parameters(), lr=lr)
    total = max(1, len(train_dl) * args.num_epochs)
    scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lambda s: max(0.0, 1 - s / total))
    return model, optimizer, train_dl, eval_dl, scheduler


@torch.no_grad()
def evaluate(accelerator, model, eval_dl) -> dict:
    model.eval()
    preds, refs = [], []
    for batch in eval_dl:
        logits = model(**batch).logits
        p, r = accelerator.gather_for_metrics((logits.argmax(-1), batch["labels"]))
        preds.append(p.cpu())
        refs.append(r.cpu())
    model.train()
    return nlp_example.binary_metrics(torch.cat(preds), torch.cat(refs))
