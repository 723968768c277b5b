"""Checkpoint / resume with `save_state` / `load_state` (reference: examples/by_feature/checkpointing.py).

`--checkpointing_steps N` saves every N optimizer steps (or `epoch`) under `--output_dir` with the reference layout
(model.safetensors, optimizer.bin, scheduler.bin, sampler/random states, …). `--resume_from_checkpoint DIR` restores
everything and skips the batches that epoch had already consumed (`skip_first_batches`), so a restarted job (e.g.
after the step watchdog killed a hung rank and torchrun relaunched it) continues exactly where it stopped.
"""

import os
import re

from _shared import base_parser, build, evaluate  # noqa: I001  (also puts the repo on sys.path)

from accelerate_hpc_test_amd import Accelerator


def main(argv=None):
    p = base_parser("Checkpointing example")
    p.add_argument("--checkpointing_steps", type=str, default=None, help="an integer N (every N steps) or 'epoch'")
    p.add_argument("--output_dir", type=str, default=".")
    p.add_argument("--resume_from_checkpoint", type=str, default=None)
    args = p.parse_args(argv)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    model, optimizer, train_dl, eval_dl, scheduler = build(accelerator, args)
    model, optimizer, train_dl, eval_dl, scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, scheduler)
    every = int(args.checkpointing_steps) if args.checkpointing_steps and args.checkpointing_steps.isdigit() else None
    overall_step, start_epoch, resume_step = 0, 0, None
    if args.resume_from_checkpoint:
        accelerator.print(f"resumed from checkpoint: {args.resume_from_checkpoint}")
        accelerator.load_state(args.resume_from_checkpoint)
        name = os.path.basename(os.path.normpath(args.resume_from_checkpoint))
        if name.startswith("epoch_"):
            start_epoch = int(re.findall(r"\d+", name)[0]) + 1
        else:
            overall_step = int(re.findall(r"\d+", name)[0])
            start_epoch, resume_step = divmod(overall_step, len(train_dl))
    metric = None
    for epoch in range(start_epoch, args.num_epochs):
        model.train()
        loader = train_dl
        if resume_step is not None and epoch == start_epoch:
            loader = accelerator.skip_first_batches(train_dl, resume_step)
        for batch in loader:
            loss = model(**batch).loss
            accelerator.backward(loss)
            optimizer.step()
            scheduler.step()
            optimizer.zero_grad()
            overall_step += 1
            if every and overall_step % every == 0:
                accelerator.save_state(os.path.join(args.output_dir, f"step_{overall_step}"))
        metric = evaluate(accelerator, model, eval_dl)
        accelerator.print(f"epoch {epoch}:", metric)
        if args.checkpointing_steps == "epoch":
            accelerator.save_state(os.path.join(args.output_dir, f"epoch_{epoch}"))
    accelerator.end_training()
    return metric


if __name__ == "__main__":
    main()
