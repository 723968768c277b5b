"""Tiny deterministic models/data for tests (parity: reference `test_utils/training.py:21-88`)."""

import numpy as np
import torch
from torch.utils.data import DataLoader


class RegressionDataset:
    def __init__(self, a=2, b=3, length=64, seed=None):
        rng = np.random.default_rng(seed)
        self.length = length
        self.x = rng.normal(size=(length,)).astype(np.float32)
        self.y = a * self.x + b + rng.normal(scale=0.1, size=(length,)).astype(np.float32)

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        return {"x": self.x[i], "y": self.y[i]}


class RegressionModel4XPU(torch.nn.Module):
    def __init__(self, a=0, b=0, double_output=False):
        super().__init__()
        self.a = torch.nn.Parameter(torch.tensor([2, 3]).float())
        self.b = torch.nn.Parameter(torch.tensor([2, 3]).float())
        self.first_batch = True

    def forward(self, x=None):
        if self.first_batch:
            self.first_batch = False
        return x * self.a[0] + self.b[0]


class RegressionModel(torch.nn.Module):
    def __init__(self, a=0, b=0, double_output=False):
        super().__init__()
        self.a = torch.nn.Parameter(torch.tensor(a).float())
        self.b = torch.nn.Parameter(torch.tensor(b).float())
        self.first_batch = True

    def forward(self, x=None):
        if self.first_batch:
            self.first_batch = False
        return x * self.a + self.b


class TinyMLP(torch.nn.Module):
    """Two-layer MLP with a module-list body (exercises FSDP wrapping of repeated blocks)."""

    _no_split_modules = ["Block"]

    def __init__(self, d=16, n=3):
        super().__init__()
        self.inp = torch.nn.Linear(4, d)
        self.blocks = torch.nn.ModuleList([Block(d) for _ in range(n)])
        self.out = torch.nn.Linear(d, 1)

    def forward(self, x):
        h = self.inp(x)
        for b in self.blocks:
            h = b(h)
        return self.out(h).squeeze(-1)


class Block(torch.nn.Module):
    def __init__(self, d):
        super().__init__()
        self.fc1 = torch.nn.Linear(d, 2 * d)
        self.fc2 = torch.nn.Linear(2 * d, d)

    def forward(self, h):
        return h + self.fc2(torch.nn.functional.gelu(self.fc1(h)))


def regression_loader(batch_size=16, length=96, shuffle=False, seed=0):
    return DataLoader(RegressionDataset(length=length, seed=seed), batch_size=batch_size, shuffle=shuffle)
