"""Communicator pre-flight: a few-second self-test of every process group a multi-GPU run will use, before training.

Why: the first time a job runs on a fresh 8-GPU node, a broken communicator (a rank bound to the wrong device, an IPC
mapping that opens but does not deliver, an xGMI link down) shows up as a hang inside the first FSDP all-gather, long
after the cause. Here each group gets, under a per-call time limit:

  * known-value all-reduce, all-gather and reduce-scatter (every rank checks the exact result);
  * an all-gather and a reduce-scatter of `big_bytes` (default 436 MB = one Llama-3-8B decoder layer in bf16, the FSDP
    unit size), timed: bus bandwidth = (W - 1) / W x bytes / time, the per-link figure to compare with xGMI;
  * for the world group on one node, the HIP-IPC small all-reduce (parallel/small_allreduce.py) with a known value.

A failing check or a call past its limit prints ONE JSON line naming the group and the operation and ends the
process with exit code 3 (no hang until the outer time limit). Parity note: the reference has no such check; it is
this framework's answer to SURVEY §5.8 (transport validation) and §5.3 (failure detection).
"""

from __future__ import annotations

import json
import os
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist

EXIT_CODE = 3


class PreflightError(RuntimeError):
    pass


def _fail(report: dict, group: str, op: str, detail: str, hard_exit: bool):
    rec = {"preflight_error": {"group": group, "op": op, "detail": detail}, "rank": dist.get_rank(), **report}
    print(json.dumps(rec), flush=True)
    if hard_exit:
        os._exit(EXIT_CODE)  # a collective may still be stuck in another thread: do not wait for it
    raise PreflightError(f"{group}/{op}: {detail}")


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _limited(fn, timeout_s: float, on_timeout):
    """Run `fn()`; if it has not returned after `timeout_s`, call `on_timeout()` from a timer thread."""
    timer = threading.Timer(timeout_s, on_timeout)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    finally:
        timer.cancel()


def communicator_preflight(groups: dict, device: torch.device, big_bytes: int = 436 << 20, timeout_s: float = 10.0,
                           iters: int = 3, hard_exit: bool = True, check_ipc: bool = True,
                           init_timeout_s: float = 180.0) -> dict:
    """Self-test `groups` ({name: process group or None for the world}); returns {name: {...bandwidths}} plus
    `ipc_allreduce` and `seconds`. Collective over every rank of every group (call it on all ranks, same order).
    The first call on each group may create its RCCL communicator (topology discovery, connection setup: seconds on a
    cold node), so it gets `init_timeout_s`; every later call gets `timeout_s`."""
    t_all = time.perf_counter()
    report: dict = {}
    for name, group in groups.items():
        W, r = dist.get_world_size(group), dist.get_rank(group)
        entry = {"world": W}
        report[name] = entry

        def run(op, fn, _name=name, limit=None):
            limit = timeout_s if limit is None else limit

            def timed_out():
                _fail({"preflight": report}, _name, op, f"no completion within {limit:.0f}s", True)
            return _limited(lambda: (fn(), _sync(device))[0], limit, timed_out)

        # known values (small): all-reduce, all-gather, reduce-scatter
        x = torch.full((W * 4,), float(r + 1), device=device)
        t0 = time.perf_counter()
        run("all_reduce", lambda: dist.all_reduce(x, group=group), limit=init_timeout_s)
        entry["first_call_s"] = round(time.perf_counter() - t0, 3)
        if not bool((x == W * (W + 1) / 2).all()):
            _fail({"preflight": report}, name, "all_reduce", f"expected {W * (W + 1) / 2}, got {x[:4].tolist()}",
                  hard_exit)
        src = torch.full((4,), float(r), device=device)
        out = torch.empty(W * 4, device=device)
        run("all_gather", lambda: dist.all_gather_into_tensor(out, src, group=group))
        want = torch.arange(W, device=device, dtype=torch.float32).repeat_interleave(4)
        if not torch.equal(out, want):
            _fail({"preflight": report}, name, "all_gather", f"got {out.tolist()[:8]}", hard_exit)
        rs_in = torch.arange(W * 4, device=device, dtype=torch.float32) + r
        rs_out = torch.empty(4, device=device)
        run("reduce_scatter", lambda: dist.reduce_scatter_tensor(rs_out, rs_in, group=group))
        want = (torch.arange(r * 4, r * 4 + 4, device=device, dtype=torch.float32) * W + W * (W - 1) / 2)
        if not torch.equal(rs_out, want):
            _fail({"preflight": report}, name, "reduce_scatter", f"got {rs_out.tolist()}", hard_exit)
        # bandwidth: bf16 all-gather / reduce-scatter of big_bytes (the FSDP unit size)
        n = max(W, (big_bytes // 2) // W * W)
        full = torch.empty(n, dtype=torch.bfloat16, device=device)
        shard = torch.ones(n // W, dtype=torch.bfloat16, device=device)
        for op, fn in (("all_gather_big", lambda: dist.all_gather_into_tensor(full, shard, group=group)),
                       ("reduce_scatter_big", lambda: dist.reduce_scatter_tensor(shard, full, group=group))):
            run(op, fn, limit=max(timeout_s, init_timeout_s / 4))  # warm-up: first use of a size sets up buffers
            t0 = time.perf_counter()
            for _ in range(iters):
                run(op, fn)
            dt = (time.perf_counter() - t0) / iters
            entry[f"{op[:-4]}_busbw_gbs"] = round((W - 1) / W * n * 2 / dt / 1e9, 3) if W > 1 else None
            entry[f"{op[:-4]}_ms"] = round(dt * 1e3, 3)
        del full, shard
        entry["ok"] = True
    if check_ipc and device.type == "cuda":
        from ..parallel import small_allreduce

        c = small_allreduce.get(None)
        ok = None
        if c is not None:
            W, r = dist.get_world_size(), dist.get_rank()
            t = torch.full((16,), float(r + 1), device=device)
            _limited(lambda: (small_allreduce.all_reduce_(t), _sync(device)), timeout_s,
                     lambda: _fail({"preflight": report}, "world", "ipc_all_reduce", "timed out", True))
            ok = bool((t == W * (W + 1) / 2).all())
            if not ok:
                _fail({"preflight": report}, "world", "ipc_all_reduce", f"got {t[:4].tolist()}", hard_exit)
        report["ipc_allreduce"] = ok  # None: path not in use here (RCCL serves small messages)
    report["seconds"] = round(time.perf_counter() - t_all, 2)
    return report


def engine_groups(model) -> tuple:
    """The named process groups a prepared model's engine communicates on: the world, the FSDP engine's all-gather /
    reduce-scatter communicators, the DDP reducer's. Returns ({name: group}, {name: "world"}): the second dict names
    the engine communicators that ARE the world group (gloo engines use it directly), tested once under "world"."""
    groups: dict = {"world": None}
    aliases: dict = {}
    eng = getattr(model, "engine", None)
    if eng is not None:
        for attr, name in (("ag_group", "fsdp_all_gather"), ("rs_group", "fsdp_reduce_scatter"),
                           ("replicate_group", "fsdp_replicate")):
            if not hasattr(eng, attr):
                continue
            g = getattr(eng, attr)
            if g is None or g is dist.group.WORLD:
                if attr != "replicate_group":  # no replicate group = no replication, not the world group
                    aliases[name] = "world"
            elif name not in groups and dist.get_world_size(g) > 1:
                groups[name] = g
    if getattr(model, "comm_group", None) is not None:
        groups["ddp"] = model.comm_group
    return groups, aliases


def preflight_model(model, device: Optional[torch.device] = None, **kw) -> dict:
    device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    groups, aliases = engine_groups(model)
    report = communicator_preflight(groups, device, **kw)
    for name, target in aliases.items():
        report[name] = {"alias_of": target, "ok": report[target]["ok"]}
    return report
