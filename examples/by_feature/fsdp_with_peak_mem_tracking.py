"""FSDP (our native FSDP2-style engine) with peak-memory tracking
(reference: examples/by_feature/fsdp_with_peak_mem_tracking.py).

`FullyShardedDataParallelPlugin(fsdp_version=2, ...)` shards every BertLayer's parameters into one flat buffer per
layer; all-gathers and reduce-scatters run on side HIP streams. The example prints the per-epoch peak device memory
(or the process RSS on CPU) next to the metric.
"""

import resource

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

import torch

from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin


def peak_memory_mb(device) -> float:
    if device.type == "cuda":
        return torch.cuda.max_memory_allocated(device) / 2**20
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024


def main(argv=None):
    p = base_parser("FSDP + peak memory example")
    args = p.parse_args(argv)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["BertLayer"])
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, fsdp_plugin=plugin)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    metric = None
    for epoch in range(args.num_epochs):
        if accelerator.device.type == "cuda":
            torch.cuda.reset_peak_memory_stats(accelerator.device)
        model.train()
        for batch in train_dl:
            loss = model(**batch).loss
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
        metric = evaluate(accelerator, model, eval_dl)
        accelerator.print(f"epoch {epoch}: {metric}, peak memory {peak_memory_mb(accelerator.device):.0f} MB")
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
