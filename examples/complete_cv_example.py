"""The image-classification example with every production feature switched on: step or epoch checkpoints, mid-epoch
resume (`skip_first_batches` on the restored loader position), experiment tracking and a project directory.

Parity: the reference's `examples/complete_cv_example.py` (same flags: `--checkpointing_steps`,
`--resume_from_checkpoint`, `--with_tracking`, `--output_dir`, `--project_dir`). Data and network come from
`examples/cv_example.py` (synthetic pets-shaped images, a small ResNet; offline by construction).

    python examples/complete_cv_example.py --cpu --image_size 32 --n_train 256 --checkpointing_steps epoch --output_dir /tmp/cv
    python examples/complete_cv_example.py --cpu --image_size 32 --n_train 256 --resume_from_checkpoint /tmp/cv/epoch_0
"""

import argparse
import os
import sys

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cv_example import SmallResNet, SyntheticPets  # noqa: E402

from accelerate_hpc_test_amd import Accelerator  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402


def training_function(args):
    kwargs = dict(log_with="all", project_dir=args.project_dir) if args.with_tracking else {}
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision, **kwargs)
    ckpt = args.checkpointing_steps
    if ckpt is not None and ckpt.isdigit():
        ckpt = int(ckpt)
    elif ckpt not in (None, "epoch"):
        raise ValueError(f"--checkpointing_steps must be an integer or 'epoch', got {ckpt!r}")
    if args.with_tracking:
        accelerator.init_trackers("complete_cv_example", vars(args))
    set_seed(args.seed)
    train_dl = DataLoader(SyntheticPets(args.n_train, args.image_size, seed=1), shuffle=True, batch_size=args.batch_size)
    eval_dl = DataLoader(SyntheticPets(args.n_eval, args.image_size, seed=2), shuffle=False, batch_size=args.batch_size)
    model = SmallResNet()
    opt = torch.optim.Adam(model.parameters(), lr=args.lr / 25)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=args.lr, epochs=args.num_epochs, steps_per_epoch=len(train_dl))
    model, opt, train_dl, eval_dl, sched = accelerator.prepare(model, opt, train_dl, eval_dl, sched)

    overall_step, starting_epoch, resume_step = 0, 0, None
    if args.resume_from_checkpoint:
        accelerator.print(f"Resumed from checkpoint: {args.resume_from_checkpoint}")
        accelerator.load_state(args.resume_from_checkpoint)
        tag = os.path.basename(os.path.normpath(args.resume_from_checkpoint))
        if tag.startswith("epoch_"):
            starting_epoch = int(tag[len("epoch_"):]) + 1
            overall_step = starting_epoch * len(train_dl)
        else:  # step_{N}
            overall_step = int(tag[len("step_"):])
            starting_epoch, resume_step = divmod(overall_step, len(train_dl))

    acc = 0.0
    for epoch in range(starting_epoch, args.num_epochs):
        model.train()
        total_loss = 0.0
        active = train_dl
        if resume_step is not None and epoch == starting_epoch:
            active = accelerator.skip_first_batches(train_dl, resume_step)
        for batch in active:
            loss = F.cross_entropy(model(batch["image"]), batch["label"])
            total_loss += loss.detach().float().item()
            accelerator.backward(loss)
            opt.step()
            sched.step()
            opt.zero_grad()
            overall_step += 1
            if isinstance(ckpt, int) and overall_step % ckpt == 0:
                accelerator.save_state(os.path.join(args.output_dir, f"step_{overall_step}"))
        model.eval()
        correct = total = 0
        for batch in eval_dl:
            with torch.no_grad():
                pred = model(batch["image"]).argmax(-1)
            pred, ref = accelerator.gather_for_metrics((pred, batch["label"]))
            correct += (pred == ref).long().sum().item()
            total += ref.numel()
        acc = correct / max(total, 1)
        accelerator.print(f"epoch {epoch}: accuracy {100 * acc:.2f}")
        if args.with_tracking:
            accelerator.log({"accuracy": acc, "train_loss": total_loss / len(train_dl), "epoch": epoch}, step=overall_step)
        if ckpt == "epoch":
            accelerator.save_state(os.path.join(args.output_dir, f"epoch_{epoch}"))
    accelerator.end_training()
    return {"accuracy": acc}


def main(argv=None):
    p = argparse.ArgumentParser(description="Complete image classification example (synthetic pets-shaped data).")
    p.add_argument("--mixed_precision", default=None, choices=["no", "fp16", "bf16", "fp8"])
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--num_epochs", type=int, default=5)
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--lr", type=float, default=3e-2)
    p.add_argument("--image_size", type=int, default=224)
    p.add_argument("--n_train", type=int, default=3680)
    p.add_argument("--n_eval", type=int, default=736)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--checkpointing_steps", default=None, help="an integer N (every N steps) or 'epoch'")
    p.add_argument("--resume_from_checkpoint", default=None)
    p.add_argument("--with_tracking", action="store_true")
    p.add_argument("--output_dir", default=".")
    p.add_argument("--project_dir", default="logs")
    return training_function(p.parse_args(argv))


if __name__ == "__main__":
    main()
