"""Early stopping across ranks with `set_trigger` / `check_trigger` (reference: examples/by_feature/early_stopping.py).

Any rank may decide to stop (here: its loss fell below `--loss_threshold` for `--patience` steps); `check_trigger`
all-reduces the flag (one scalar over RCCL), so every rank leaves the loop at the same step and no collective is left
waiting on a rank that already stopped.
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator


class EarlyStoppingCallback:
    def __init__(self, min_delta=0.0, patience=5):
        self.min_delta, self.patience = min_delta, patience
        self.counter, self.lowest_loss = 0, float("inf")

    def check_early_stopping(self, loss):
        delta = self.lowest_loss - loss
        if delta >= self.min_delta:
            self.lowest_loss, self.counter = loss, 0
        else:
            self.counter += 1
        return self.counter >= self.patience


def main(argv=None):
    p = base_parser("Early stopping example")
    p.add_argument("--patience", type=int, default=3)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    callback = EarlyStoppingCallback(patience=args.patience)
    stopped_at = None
    for epoch in range(args.num_epochs):
        model.train()
        for step, batch in enumerate(train_dl):
            loss = model(**batch).loss
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
            if callback.check_early_stopping(loss.item()):
                accelerator.set_trigger()
            if accelerator.check_trigger():
                stopped_at = (epoch, step)
                break
        accelerator.print(f"epoch {epoch}:", evaluate(accelerator, model, eval_dl))
        if stopped_at is not None:
            accelerator.print(f"early stop at epoch {epoch} step {stopped_at[1]}")
            break
    accelerator.end_training()
    return {"stopped_at": stopped_at}


if __name__ == "__main__":
    main()
