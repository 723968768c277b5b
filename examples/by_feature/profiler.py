"""Profiling with `accelerator.profile(ProfileKwargs(...))` (reference: examples/by_feature/profiler.py).

Each rank writes `profile_<rank>.json` (Chrome trace) into `--output_trace_dir`. On MI355X the `cuda` activity is
served by roctracer through kineto, and the framework's roctx ranges (ACCELERATE_ROCTX=1) label the FSDP / DDP
collectives. For kernel-level counters use `rocprofv3 --kernel-trace --stats` (tools/gpu_steps.sh prof8b).
"""

from _shared import base_parser, build  # noqa: I001  (also puts the repo on sys.path)

import torch

from accelerate_hpc_test_amd import Accelerator, ProfileKwargs


def main(argv=None):
    p = base_parser("Profiler example")
    p.add_argument("--output_trace_dir", type=str, default="profiler_traces")
    p.add_argument("--steps", type=int, default=6)
    args = p.parse_args(argv)
    activities = ["cpu"] if args.cpu or not torch.cuda.is_available() else ["cpu", "cuda"]
    handler = ProfileKwargs(activities=activities, schedule_option={"wait": 1, "warmup": 1, "active": 2, "repeat": 1},
                            record_shapes=True, output_trace_dir=args.output_trace_dir)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, kwargs_handlers=[handler])
    model, optimizer, train_dl, _, scheduler = build(accelerator, args)
    model, optimizer, train_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, scheduler)
    model.train()
    with accelerator.profile() as prof:
        for i, batch in enumerate(train_dl):
            if i >= args.steps:
                break
            loss = model(**batch).loss
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
            prof.step()
    accelerator.print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=10))
    accelerator.end_training()
    return prof


if __name__ == "__main__":
    main()
