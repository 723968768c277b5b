"""Tracing and throughput observability.

Parity. The reference exposes `torch.profiler` through `ProfileKwargs` / `Accelerator.profile`
(`/root/reference/src/accelerate/utils/dataclasses.py:483-597`, `accelerator.py:4167-4225`) and keeps its throughput
tracker outside the library (`examples/torch_native_parallelism/utils.py:94-190`, whose attention FLOP term drops the
head dimension, `utils.py:109`). Here:

* `trace_range(name)` / `@traced(name)` — roctx ranges (ROCm's torch routes `torch.cuda.nvtx` to roctx), so
  `rocprofv3 --marker-trace --kernel-trace` shows the framework's phases (FSDP unshard / reduce, DDP bucket
  all-reduce, optimizer step) next to the kernels they launch. Off unless `ACCELERATE_ROCTX=1` (each range is a host
  call); when a `torch.profiler` session is active they also become `record_function` regions in its trace.
* `ThroughputTracker` — warm-up-aware tokens/s, steps/s, TFLOP/s per device and peak memory, with the reference
  tracker's `step(batch_tokens, model_flops_per_token)` contract, plus the whole-job token rate.
* `model_flops_per_token(model_or_config, seq_len)` — 6·(matmul params) + causal attention 6·L·S·Hq·D (keeps D).
"""

from __future__ import annotations

import functools
import os
import time
from contextlib import contextmanager
from typing import Optional

import torch


def roctx_enabled() -> bool:
    return os.environ.get("ACCELERATE_ROCTX", "0") == "1"


@contextmanager
def trace_range(name: str):
    """roctx range (when ACCELERATE_ROCTX=1 and a GPU is present) + a profiler region (when one is recording)."""
    use_roctx = roctx_enabled() and torch.cuda.is_available()
    if use_roctx:
        torch.cuda.nvtx.range_push(name)
    rf = None
    if torch.autograd.profiler._is_profiler_enabled:
        rf = torch.autograd.profiler.record_function(name)
        rf.__enter__()
    try:
        yield
    finally:
        if rf is not None:
            rf.__exit__(None, None, None)
        if use_roctx:
            torch.cuda.nvtx.range_pop()


def traced(name: Optional[str] = None):
    """Decorator form of `trace_range`."""

    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **k):
            with trace_range(label):
                return fn(*a, **k)

        return wrapper

    return deco


def _cfg_get(cfg, *names, default=None):
    for n in names:
        v = getattr(cfg, n, None)
        if v is not None:
            return v
    return default


def model_flops_per_token(model_or_config, seq_len: int, causal: bool = True) -> float:
    """Training FLOPs per token of a decoder-only transformer (fwd + bwd = 3 × fwd)."""
    cfg = getattr(model_or_config, "config", model_or_config)
    if hasattr(cfg, "flops_per_token"):  # models/llama.py, models/mixtral.py
        return float(cfg.flops_per_token(seq_len))
    h = _cfg_get(cfg, "hidden_size", "n_embd", "d_model")
    L = _cfg_get(cfg, "num_hidden_layers", "n_layer", "num_layers")
    Hq = _cfg_get(cfg, "num_attention_heads", "n_head")
    Hkv = _cfg_get(cfg, "num_key_value_heads", default=Hq)
    D = _cfg_get(cfg, "head_dim", default=h // Hq)
    inter = _cfg_get(cfg, "intermediate_size", "n_inner", default=4 * h)
    V = _cfg_get(cfg, "vocab_size", default=0)
    gated = 3 if _cfg_get(cfg, "hidden_act", default="silu") in ("silu", "swiglu", "gelu_pytorch_tanh") else 2
    per_layer = h * D * (Hq + 2 * Hkv) + Hq * D * h + gated * h * inter
    attn = 6 * L * seq_len * Hq * D * (0.5 if causal else 1.0) * 2
    return float(6 * (L * per_layer + h * V) + attn)


class ThroughputTracker:
    """Tokens/s, steps/s, TFLOP/s per device and peak memory after `warmup_steps` steps.

    Same contract as the reference's `PerformanceTracker.step(batch_tokens, model_flops_per_token)`: returns
    `{"warmup_completed": True}` on the last warm-up step, `{}` before, metrics after. `batch_tokens` are this rank's
    tokens; `tokens_per_second_whole_job` multiplies by the number of processes (data parallel, equal batches).
    With `sync=True` the device is synchronised before reading the clock so queued kernels are counted.
    """

    def __init__(self, warmup_steps: int = 10, num_processes: Optional[int] = None, sync: bool = True):
        self.warmup_steps = warmup_steps
        if num_processes is None:
            num_processes = torch.distributed.get_world_size() if torch.distributed.is_available() and torch.distributed.is_initialized() else 1
        self.num_processes = num_processes
        self.sync = sync
        self.reset()

    def reset(self):
        self.start_time = None
        self.num_tokens = 0
        self.is_in_warmup = True
        self.step_count = 0

    def _now(self):
        if self.sync and torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        return time.perf_counter()

    def step(self, batch_tokens: int, model_flops_per_token: Optional[float] = None) -> dict:
        self.step_count += 1
        if self.step_count == self.warmup_steps:
            self.start_time = self._now()
            self.num_tokens = 0
            self.is_in_warmup = False
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.reset_peak_memory_stats()
            return {"warmup_completed": True}
        if self.is_in_warmup or self.start_time is None:
            return {}
        self.num_tokens += batch_tokens
        elapsed = self._now() - self.start_time
        steps = self.step_count - self.warmup_steps
        if elapsed <= 0 or steps <= 0:
            return {}
        out = {
            "tokens_per_second": self.num_tokens / elapsed,
            "tokens_per_second_whole_job": self.num_tokens * self.num_processes / elapsed,
            "steps_per_second": steps / elapsed,
            "total_tokens": self.num_tokens,
            "total_time": elapsed,
        }
        if model_flops_per_token is not None:
            out["tflops_per_device"] = model_flops_per_token * self.num_tokens / elapsed / 1e12
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            out["peak_memory_alloc"] = torch.cuda.max_memory_allocated() / 2**30
            out["peak_memory_reserved"] = torch.cuda.max_memory_reserved() / 2**30
            out["peak_memory_active"] = torch.cuda.memory_stats().get("active_bytes.all.peak", 0) / 2**30
        return out

    @staticmethod
    def get_print_message(metrics: dict, with_memory: bool = False) -> str:
        msg = f" | steps/s {metrics['steps_per_second']:.2f} | tokens/s {metrics['tokens_per_second']:.1f}"
        msg += f" (job {metrics['tokens_per_second_whole_job']:.1f})"
        if "tflops_per_device" in metrics:
            msg += f" | TFLOP/s/device {metrics['tflops_per_device']:.1f}"
        if with_memory and "peak_memory_alloc" in metrics:
            msg += (f"\n\tmemory (GiB): active={metrics['peak_memory_active']:.1f}, alloc={metrics['peak_memory_alloc']:.1f}, "
                    f"reserved={metrics['peak_memory_reserved']:.1f}")
        return msg


PerformanceTracker = ThroughputTracker  # the reference example's name
