"""The NLP example with every production feature switched on: checkpointing every N steps or every epoch, resuming
from a checkpoint mid-epoch (`skip_first_batches`), experiment tracking, and a project directory.

Parity: the reference's `examples/complete_nlp_example.py` (same flags: `--checkpointing_steps`,
`--resume_from_checkpoint`, `--with_tracking`, `--output_dir`, `--project_dir`). Data and model come from
`examples/nlp_example.py` (synthetic MRPC-shaped pairs, random-init BERT; offline by construction).

    python examples/complete_nlp_example.py --cpu --tiny --checkpointing_steps 10 --output_dir /tmp/run
    python examples/complete_nlp_example.py --cpu --tiny --resume_from_checkpoint /tmp/run/step_10
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nlp_example import binary_metrics, build_model, get_dataloaders  # noqa: E402

from accelerate_hpc_test_amd import Accelerator  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def training_function(config, args):
    kwargs = {}
    if args.with_tracking:
        kwargs = dict(log_with="all", project_dir=args.project_dir)
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, **kwargs)
    checkpointing_steps = args.checkpointing_steps
    if checkpointing_steps is not None and checkpointing_steps.isdigit():
        checkpointing_steps = int(checkpointing_steps)
    elif checkpointing_steps not in (None, "epoch"):
        raise ValueError(f"--checkpointing_steps must be an integer or 'epoch', got {checkpointing_steps!r}")
    if args.with_tracking:
        accelerator.init_trackers(os.path.splitext(os.path.basename(__file__))[0], config)
    lr, num_epochs, seed, batch_size = config["lr"], int(config["num_epochs"]), int(config["seed"]), int(config["batch_size"])
    set_seed(seed)
    train_dl, eval_dl = get_dataloaders(accelerator, batch_size, n_train=args.n_train, n_eval=args.n_eval)
    model = build_model(args.tiny).to(accelerator.device)
    optimizer = torch.optim.AdamW(params=model.parameters(), lr=lr)
    total = len(train_dl) * num_epochs
    warmup = min(100, max(1, total // 10))
    lr_scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lambda s: min(1.0, (s + 1) / warmup) * max(0.0, 1 - s / max(1, total)))
    model, optimizer, train_dl, eval_dl, lr_scheduler = accelerator.prepare(model, optimizer, train_dl, eval_dl, lr_scheduler)

    overall_step, starting_epoch, resume_step = 0, 0, None
    if args.resume_from_checkpoint:
        accelerator.print(f"Resumed from checkpoint: {args.resume_from_checkpoint}")
        accelerator.load_state(args.resume_from_checkpoint)
        tag = os.path.basename(os.path.normpath(args.resume_from_checkpoint))
        if tag.startswith("epoch_"):
            starting_epoch = int(tag[len("epoch_"):]) + 1
        else:  # step_{N}: N optimizer steps were done; resume inside that epoch
            done = int(tag[len("step_"):])
            starting_epoch, resume_step = divmod(done, len(train_dl))
            overall_step = done
        if resume_step is None:
            overall_step = starting_epoch * len(train_dl)

    metric = None
    for epoch in range(starting_epoch, num_epochs):
        model.train()
        total_loss = 0.0
        active = train_dl
        if resume_step is not None and epoch == starting_epoch:
            active = accelerator.skip_first_batches(train_dl, resume_step)  # continue exactly where the run stopped
        for batch in active:
            outputs = model(**batch)
            loss = outputs.loss
            total_loss += loss.detach().float().item()
            accelerator.backward(loss)
            optimizer.step()
            lr_scheduler.step()
            optimizer.zero_grad()
            overall_step += 1
            if isinstance(checkpointing_steps, int) and overall_step % checkpointing_steps == 0:
                accelerator.save_state(os.path.join(args.output_dir, f"step_{overall_step}"))
        model.eval()
        preds, refs = [], []
        for batch in eval_dl:
            with torch.no_grad():
                logits = model(**batch).logits
            p, r = accelerator.gather_for_metrics((logits.argmax(-1), batch["labels"]))
            preds.append(p.cpu())
            refs.append(r.cpu())
        metric = binary_metrics(torch.cat(preds), torch.cat(refs))
        accelerator.print(f"epoch {epoch}:", metric)
        if args.with_tracking:
            accelerator.log({**metric, "train_loss": total_loss / max(1, len(train_dl)), "epoch": epoch}, step=epoch)
        if checkpointing_steps == "epoch":
            accelerator.save_state(os.path.join(args.output_dir, f"epoch_{epoch}"))
    accelerator.end_training()
    return metric


def main(argv=None):
    parser = argparse.ArgumentParser(description="Complete NLP example: checkpointing, resume, tracking.")
    parser.add_argument("--mixed_precision", type=str, default=None, choices=["no", "fp16", "bf16", "fp8"])
    parser.add_argument("--cpu", action="store_true")
    parser.add_argument("--tiny", action="store_true")
    parser.add_argument("--num_epochs", type=int, default=3)
    parser.add_argument("--n_train", type=int, default=3668)
    parser.add_argument("--n_eval", type=int, default=408)
    parser.add_argument("--checkpointing_steps", type=str, default=None,
                        help="save every N optimizer steps (integer) or at the end of every epoch ('epoch')")
    parser.add_argument("--resume_from_checkpoint", type=str, default=None, help="a step_N or epoch_N directory")
    parser.add_argument("--with_tracking", action="store_true", help="log to every available tracker")
    parser.add_argument("--output_dir", type=str, default=".", help="where checkpoints go")
    parser.add_argument("--project_dir", type=str, default="logs", help="tracker logs")
    args = parser.parse_args(argv)
    config = {"lr": 2e-5 if not args.tiny else 1e-3, "num_epochs": args.num_epochs, "seed": 42, "batch_size": 16}
    return training_function(config, args)


if __name__ == "__main__":
    main()
