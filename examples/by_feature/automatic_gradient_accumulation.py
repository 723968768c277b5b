"""Keep the effective batch size while the per-step batch shrinks to fit memory
(reference: examples/by_feature/automatic_gradient_accumulation.py): `find_executable_batch_size` picks the largest
batch that runs, and the gradient-accumulation steps are set to `observed_batch_size // batch_size`.
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.utils import find_executable_batch_size


def main(argv=None):
    p = base_parser("Automatic gradient accumulation example")
    p.add_argument("--observed_batch_size", type=int, default=32)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)

    @find_executable_batch_size(starting_batch_size=args.observed_batch_size)
    def inner(batch_size):
        accelerator.free_memory()
        accelerator.gradient_accumulation_steps = max(1, args.observed_batch_size // batch_size)
        model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args, batch_size=batch_size)
        model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
        metric = None
        for epoch in range(args.num_epochs):
            model.train()
            for batch in train_dl:
                with accelerator.accumulate(model):
                    accelerator.backward(model(**batch).loss)
                    optimizer.step()
                    scheduler.step()
                    optimizer.zero_grad()
            metric = evaluate(accelerator, model, eval_dl)
            accelerator.print(f"epoch {epoch} (batch {batch_size} x {accelerator.gradient_accumulation_steps} steps):", metric)
        return metric

    metric = inner()
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
