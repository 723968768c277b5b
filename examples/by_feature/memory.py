"""Automatic batch-size search with `find_executable_batch_size` (reference: examples/by_feature/memory.py).

The decorated function is retried with 90 % of the batch size whenever it raises an out-of-memory error (the HIP
message included); the inner function must build everything that depends on the batch size. With
`ACCELERATE_FAULT_INJECT=0:0:oom` the first attempt fails on purpose (utils/fault_tolerance.py) so the retry path can
be exercised on any machine.
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.utils import find_executable_batch_size


def main(argv=None):
    p = base_parser("Memory-aware batch size example")
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)

    @find_executable_batch_size(starting_batch_size=args.batch_size)
    def inner_training_loop(batch_size):
        accelerator.free_memory()
        model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args, batch_size=batch_size)
        model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
        metric = None
        for epoch in range(args.num_epochs):
            model.train()
            for batch in train_dl:
                loss = model(**batch).loss
                accelerator.backward(loss)
                optimizer.step()
                scheduler.step()
                optimizer.zero_grad()
            metric = evaluate(accelerator, model, eval_dl)
            accelerator.print(f"epoch {epoch} (batch size {batch_size}):", metric)
        return batch_size, metric

    result = inner_training_loop()
    accelerator.end_training()
    return result


if __name__ == "__main__":
    main()
