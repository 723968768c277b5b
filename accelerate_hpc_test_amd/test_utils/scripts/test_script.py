"""End-to-end sanity script run by `accelerate-amd test` (and usable under `accelerate-amd launch`).

Parity target: `/root/reference/src/accelerate/test_utils/scripts/test_script.py` — process-state report, RNG
synchronisation, data-loader sharding (no sample lost / duplicated), collectives, and a training-parity check
(the distributed model must match a single-process model trained on the global batch). Runs on whatever the
launch configured: CPU/gloo, one MI355X, or N MI355X over RCCL, DDP or FSDP2.
"""

from __future__ import annotations

import copy

import torch
import torch.nn.functional as F

from accelerate_hpc_test_amd import Accelerator
from accelerate_hpc_test_amd.test_utils.training import TinyMLP
from accelerate_hpc_test_amd.utils import gather, gather_object, set_seed, synchronize_rng_states


def print_main(acc, *msg):
    if acc.is_main_process:
        print(*msg, flush=True)


def rng_sync_check(acc):
    synchronize_rng_states(["torch"])
    v = torch.rand(4)
    allv = gather_object([v.tolist()])
    assert all(x == allv[0] for x in allv), f"torch RNG not synchronized: {allv}"
    print_main(acc, "RNG synchronization: ok")


def dataloader_check(acc):
    n = 37
    dl = torch.utils.data.DataLoader(torch.arange(n), batch_size=4)
    dl = acc.prepare(dl)
    seen = []
    for b in dl:
        seen.append(acc.gather_for_metrics(b).cpu())
    got = torch.cat(seen).tolist()
    assert sorted(got) == list(range(n)), f"data loader lost/duplicated samples: {got}"
    print_main(acc, "DataLoader sharding + gather_for_metrics: ok")


def ops_check(acc):
    t = torch.arange(3.0, device=acc.device) + 3 * acc.process_index
    g = gather(t).cpu()
    assert g.tolist() == [float(i) for i in range(3 * acc.num_processes)]
    r = acc.reduce(torch.ones(1, device=acc.device), reduction="sum").item()
    assert r == acc.num_processes
    print_main(acc, "Collectives (gather/reduce): ok")


def training_check(acc):
    W, rank = acc.num_processes, acc.process_index
    set_seed(0)
    base = TinyMLP().to(acc.device)
    model = copy.deepcopy(base)
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    base_opt = torch.optim.SGD(base.parameters(), lr=0.05)
    model, opt = acc.prepare(model, opt)
    bs = 4
    gen = torch.Generator().manual_seed(1)
    for _ in range(3):
        x = torch.randn(bs * W, 4, generator=gen).to(acc.device)
        y = torch.randn(bs * W, generator=gen).to(acc.device)
        xl, yl = x[rank * bs : (rank + 1) * bs], y[rank * bs : (rank + 1) * bs]
        acc.backward(F.mse_loss(model(xl).float(), yl))
        opt.step()
        opt.zero_grad()
        F.mse_loss(base(x), y).backward()
        base_opt.step()
        base_opt.zero_grad()
    full = acc.get_state_dict(model)
    tol = 1e-4 if acc.mixed_precision == "no" else 5e-2
    if acc.is_main_process:
        for n, q in base.named_parameters():
            assert torch.allclose(full[n].float().cpu(), q.float().cpu(), atol=tol), (n, (full[n].cpu() - q.cpu()).abs().max())
    print_main(acc, f"Training parity vs single process ({acc.distributed_type.value}): ok")


def main():
    acc = Accelerator()
    print_main(acc, "**Initialization**")
    acc.print(acc.state)
    rng_sync_check(acc)
    ops_check(acc)
    dataloader_check(acc)
    training_check(acc)
    acc.wait_for_everyone()
    acc.end_training()


if __name__ == "__main__":
    main()
