"""Exact distributed evaluation with `gather_for_metrics` (reference: examples/by_feature/multi_process_metrics.py).

With `even_batches` the last batch is padded by wrapping around so every rank runs the same number of collectives;
`gather_for_metrics` drops those duplicates, so the metric is computed on exactly the evaluation set.
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator


def main(argv=None):
    p = base_parser("Multi-process metrics example")
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    seen = 0
    for epoch in range(args.num_epochs):
        model.train()
        for batch in train_dl:
            loss = model(**batch).loss
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
        model.eval()
        seen = 0
        for batch in eval_dl:
            refs = accelerator.gather_for_metrics(batch["labels"])
            seen += refs.shape[0]
        metric = evaluate(accelerator, model, eval_dl)
        accelerator.print(f"epoch {epoch}: {metric} over {seen} samples")
    accelerator.end_training()
    return seen


if __name__ == "__main__":
    main()
