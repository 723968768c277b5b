"""k-fold cross validation with one Accelerator (reference: examples/by_feature/cross_validation.py).

Each fold re-prepares a fresh model/optimizer/loaders; `accelerator.free_memory()` drops the previous fold's
prepared objects (and their FSDP/DDP buffers) first. Test-set logits of every fold are gathered and averaged.
"""

from _shared import base_parser, evaluate, nlp_example  # noqa: I001  (also puts the repo on sys.path)

import torch
from torch.utils.data import DataLoader, Subset

from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.utils import set_seed


def main(argv=None):
    p = base_parser("Cross-validation example")
    p.add_argument("--num_folds", type=int, default=3)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    data = nlp_example.SyntheticMRPC(args.n_train, 28996, seed=0)
    test = nlp_example.SyntheticMRPC(args.n_eval, 28996, seed=1)
    folds = torch.arange(len(data)).chunk(args.num_folds)
    test_logits, fold_metrics = [], []
    for k in range(args.num_folds):
        accelerator.free_memory()
        set_seed(42 + k)
        train_idx = torch.cat([f for i, f in enumerate(folds) if i != k]).tolist()
        train_dl = DataLoader(Subset(data, train_idx), batch_size=args.batch_size, shuffle=True, collate_fn=nlp_example.collate_fn)
        val_dl = DataLoader(Subset(data, folds[k].tolist()), batch_size=32, collate_fn=nlp_example.collate_fn)
        test_dl = DataLoader(test, batch_size=32, collate_fn=nlp_example.collate_fn)
        model = nlp_example.build_model(args.tiny)
        optimizer = torch.optim.AdamW(model.parameters(), lr=args.lr or (1e-3 if args.tiny else 2e-5))
        model, optimizer, train_dl, val_dl, test_dl = accelerator.prepare(model, optimizer, train_dl, val_dl, test_dl)
        for _ in range(args.num_epochs):
            model.train()
            for batch in train_dl:
                accelerator.backward(model(**batch).loss)
                optimizer.step()
                optimizer.zero_grad()
        fold_metrics.append(evaluate(accelerator, model, val_dl))
        model.eval()
        with torch.no_grad():
            logits = torch.cat([accelerator.gather_for_metrics(model(**b).logits).cpu() for b in test_dl])
        test_logits.append(logits)
        accelerator.print(f"fold {k}: {fold_metrics[-1]}")
    labels = torch.tensor([test[i]["labels"] for i in range(len(test))])
    ensemble = nlp_example.binary_metrics(torch.stack(test_logits).mean(0).argmax(-1), labels)
    accelerator.print("ensemble on the test set:", ensemble)
    accelerator.end_training()
    return ensemble


if __name__ == "__main__":
    main()
