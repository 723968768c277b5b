"""Minimal script for the templates in this folder:

    accelerate-amd launch --config_file examples/config_yaml_templates/single_accelerator.yaml \
        examples/config_yaml_templates/run_me.py

It builds an Accelerator from the launcher's environment, trains a small regression model for a few steps and prints
the distributed setup it ran with (parity: reference examples/config_yaml_templates/run_me.py).
"""

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from accelerate_hpc_test_amd import Accelerator  # noqa: E402


def main():
    accelerator = Accelerator()
    accelerator.print(f"distributed_type={accelerator.distributed_type} num_processes={accelerator.num_processes} "
                      f"mixed_precision={accelerator.mixed_precision} device={accelerator.device}")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.GELU(), torch.nn.Linear(64, 1))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
    x = torch.randn(256, 16)
    y = x.sum(-1, keepdim=True)
    dl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(x, y), batch_size=32)
    model, opt, dl = accelerator.prepare(model, opt, dl)
    for _ in range(3):
        for xb, yb in dl:
            loss = torch.nn.functional.mse_loss(model(xb).float(), yb.float())
            accelerator.backward(loss)
            opt.step()
            opt.zero_grad()
    accelerator.print(f"final loss {accelerator.reduce(loss.detach(), 'mean').item():.4f}")
    accelerator.end_training()


if __name__ == "__main__":
    main()
