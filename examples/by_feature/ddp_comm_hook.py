"""DDP communication hooks (reference: examples/by_feature/ddp_comm_hook.py).

`DistributedDataParallelKwargs(comm_hook=...)` selects how our DDP reducer all-reduces each gradient bucket over
RCCL: `no` (fp32), `fp16` / `bf16` (cast the bucket once, all-reduce half the bytes, cast back — averaging folded
in), `power_sgd` / `batched_power_sgd` (rank-r low-rank approximation with error feedback).
"""

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator, DDPCommunicationHookType, DistributedDataParallelKwargs


def main(argv=None):
    p = base_parser("DDP comm hook example")
    p.add_argument("--ddp_comm_hook", type=str, default="bf16", choices=[h.value for h in DDPCommunicationHookType])
    args = p.parse_args(argv)
    kw = DistributedDataParallelKwargs(comm_hook=DDPCommunicationHookType(args.ddp_comm_hook),
                                       comm_state_option={"matrix_approximation_rank": 2, "start_powerSGD_iter": 2})
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, kwargs_handlers=[kw])
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
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
        accelerator.print(f"epoch {epoch}:", metric)
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
