"""Learning-rate scheduler wrapper.

Parity: `/root/reference/src/accelerate/scheduler.py:25-98`: the scheduler only steps when gradients were
synchronised (not during accumulation), skips when the fp16 scaler skipped the optimizer step, and — when
batches are not split — steps `num_processes` times per call so the schedule is expressed in
per-process optimizer steps like a single-GPU run with the global batch.
"""

from __future__ import annotations

import warnings

from .state import AcceleratorState, GradientState


class AcceleratedScheduler:
    def __init__(self, scheduler, optimizers, step_with_optimizer: bool = True, split_batches: bool = False):
        self.scheduler = scheduler
        self.optimizers = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
        self.split_batches = split_batches
        self.step_with_optimizer = step_with_optimizer
        self.gradient_state = GradientState()

    def step(self, *args, **kwargs):
        if not self.step_with_optimizer:
            self.scheduler.step(*args, **kwargs)
            return
        if not self.gradient_state.sync_gradients:
            if self.gradient_state.adjust_scheduler:
                self.scheduler._step_count += 1
            return
        for opt in self.optimizers:
            if getattr(opt, "step_was_skipped", False):
                return
        if self.split_batches:
            self.scheduler.step(*args, **kwargs)
        else:
            num_processes = AcceleratorState().num_processes
            for _ in range(num_processes):
                if hasattr(self.scheduler, "total_steps"):
                    if self.scheduler._step_count <= self.scheduler.total_steps:
                        self.scheduler.step(*args, **kwargs)
                else:
                    self.scheduler.step(*args, **kwargs)

    def get_last_lr(self):
        return self.scheduler.get_last_lr()

    def state_dict(self):
        return self.scheduler.state_dict()

    def load_state_dict(self, state_dict):
        self.scheduler.load_state_dict(state_dict)

    def get_lr(self):
        return self.scheduler.get_lr()

    def print_lr(self, *args, **kwargs):
        return self.scheduler.print_lr(*args, **kwargs)
