"""Gradient accumulation with `accelerator.accumulate(model)` (reference: examples/by_feature/gradient_accumulation.py).

Inside `accumulate`, the data-parallel gradient sync (DDP bucket all-reduce / FSDP reduce-scatter over RCCL) only runs
on the last micro-batch of each accumulation window and on the last batch of the data loader; the wrapped optimizer
and scheduler skip their steps in between, so the loop reads like plain training.
"""


from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator


def main(argv=None):
    p = base_parser("Gradient accumulation example")
    p.add_argument("--gradient_accumulation_steps", type=int, default=2)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision,
                              gradient_accumulation_steps=args.gradient_accumulation_steps)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    metric = None
    for epoch in range(args.num_epochs):
        model.train()
        for batch in train_dl:
            with accelerator.accumulate(model):
                loss = model(**batch).loss
                accelerator.backward(loss)
                optimizer.step()
                scheduler.step()
                optimizer.zero_grad()
        metric = evaluate(accelerator, model, eval_dl)
        accelerator.print(f"epoch {epoch}:", metric)
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
