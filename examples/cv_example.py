"""Image classification (Oxford-IIIT-Pets shape: 37 classes) with the Accelerator API.

Same training loop as the reference's `examples/cv_example.py`: normalised image batches, a frozen feature extractor
with a trainable head, OneCycleLR stepped with the optimizer, `gather_for_metrics` evaluation; runnable on CPU
(`--cpu`) or any number of MI355X ranks via `accelerate-amd launch examples/cv_example.py`.

Offline by construction: there is no network for the pets images or timm's pretrained ResNet-50, and neither timm nor
torchvision is installed. The data are synthetic 3-channel images whose class sets a colour / stripe pattern under
noise, and the network is a small residual CNN defined here. `--image_size 64` and `--n_train 512` make a test-sized
run; the defaults (224 px, 3 680 images) match the pets training-set shape.
"""

import argparse
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from accelerate_hpc_test_amd import Accelerator  # noqa: E402
from accelerate_hpc_test_amd.utils import set_seed  # noqa: E402

NUM_CLASSES = 37
MEAN = torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)


class SyntheticPets(Dataset):
    """Class c: a channel mix and a stripe frequency chosen from c, plus noise."""

    def __init__(self, n, image_size, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.labels = torch.randint(0, NUM_CLASSES, (n,), generator=g)
        self.noise_seed = seed
        self.size = image_size
        ys = torch.linspace(0, 1, image_size).view(-1, 1)
        self.grid = ys.expand(image_size, image_size)

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        c = int(self.labels[i])
        g = torch.Generator().manual_seed(self.noise_seed * 100003 + i)
        colour = torch.tensor([(c % 3) / 2, ((c // 3) % 4) / 3, ((c // 12) % 4) / 3]).view(3, 1, 1)
        stripes = 0.5 + 0.5 * torch.sin(self.grid * (2 + c % 5) * 3.14159)
        img = (0.6 * colour * stripes + 0.4 * torch.rand(3, self.size, self.size, generator=g)).clamp(0, 1)
        return {"image": (img - MEAN) / STD, "label": c}


class Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.skip = nn.Sequential() if stride == 1 and cin == cout else nn.Sequential(
            nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + self.skip(x))


class SmallResNet(nn.Module):
    """Feature extractor (`features`) + linear classifier (`classifier`), the split the reference freezes on."""

    def __init__(self, num_classes=NUM_CLASSES, width=32):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, width, 3, 2, 1, bias=False), nn.BatchNorm2d(width), nn.ReLU(),
            Block(width, width, 1), Block(width, 2 * width, 2), Block(2 * width, 4 * width, 2),
            nn.AdaptiveAvgPool2d(1), nn.Flatten())
        self.classifier = nn.Linear(4 * width, num_classes)

    def forward(self, x):
        return self.classifier(self.features(x))


def training_function(args):
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=args.mixed_precision)
    set_seed(args.seed)
    train_ds = SyntheticPets(args.n_train, args.image_size, seed=1)
    eval_ds = SyntheticPets(args.n_eval, args.image_size, seed=2)
    train_dl = DataLoader(train_ds, shuffle=True, batch_size=args.batch_size, num_workers=0)
    eval_dl = DataLoader(eval_ds, shuffle=False, batch_size=args.batch_size, num_workers=0)
    model = SmallResNet()
    if args.freeze_features:  # the reference trains only the head of a pretrained network
        for p in model.features.parameters():
            p.requires_grad = False
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=args.lr / 25)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=args.lr, epochs=args.num_epochs, steps_per_epoch=len(train_dl))
    model, opt, train_dl, eval_dl, sched = accelerator.prepare(model, opt, train_dl, eval_dl, sched)
    acc = 0.0
    for epoch in range(args.num_epochs):
        model.train()
        for batch in train_dl:
            loss = F.cross_entropy(model(batch["image"]), batch["label"])
            accelerator.backward(loss)
            opt.step()
            sched.step()
            opt.zero_grad()
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
    accelerator.end_training()
    return {"accuracy": acc}


def main(argv=None):
    p = argparse.ArgumentParser(description="Image classification example (synthetic pets-shaped data).")
    p.add_argument("--mixed_precision", default=None, choices=["no", "fp16", "bf16", "fp8"])
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--num_epochs", type=int, default=5)
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--lr", type=float, default=3e-2)
    p.add_argument("--image_size", type=int, default=224)
    p.add_argument("--n_train", type=int, default=3680)
    p.add_argument("--n_eval", type=int, default=736)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--freeze_features", action="store_true", help="train only the classifier head")
    return training_function(p.parse_args(argv))


if __name__ == "__main__":
    main()
