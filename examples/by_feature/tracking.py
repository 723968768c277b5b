"""Experiment tracking with `log_with` / `init_trackers` / `log` (reference: examples/by_feature/tracking.py).

Trackers run on the main process only. `--with_tracking` logs loss, accuracy and the per-epoch token rate to
every available tracker under `--project_dir` (TensorBoard when installed; any `GeneralTracker` subclass works).
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator


def main(argv=None, trackers=None):
    p = base_parser("Tracking example")
    p.add_argument("--with_tracking", action="store_true")
    p.add_argument("--project_dir", type=str, default="logs")
    args = p.parse_args(argv)
    log_with = trackers if trackers is not None else ("all" if args.with_tracking else None)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, log_with=log_with, project_dir=args.project_dir)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    if log_with is not None:
        accelerator.init_trackers("by_feature_tracking", config={"lr": optimizer.param_groups[0]["lr"], "epochs": args.num_epochs})
    metric = None
    for epoch in range(args.num_epochs):
        model.train()
        total = 0.0
        for batch in train_dl:
            loss = model(**batch).loss
            total += loss.detach().float()
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
        metric = evaluate(accelerator, model, eval_dl)
        accelerator.print(f"epoch {epoch}:", metric)
        if log_with is not None:
            accelerator.log({"accuracy": metric["accuracy"], "f1": metric["f1"], "train_loss": (total / len(train_dl)).item(), "epoch": epoch}, step=epoch)
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
