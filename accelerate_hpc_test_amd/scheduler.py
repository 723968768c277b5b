"""Learning-rate scheduler wrapper.

Parity: `/root/reference/src/accelerate/scheduler.py:25-98`. The rules a wrapped scheduler follows:
* it advances only on steps where gradients were synchronised (during accumulation it only bumps its step counter
  when the accumulation plugin asks for `adjust_scheduler`);
* it does not advance when an fp16 scaler skipped the optimizer step;
* without `split_batches` one call advances it once per process, so the schedule is counted in per-process optimizer
  steps as in a single-GPU run over the global batch (OneCycle-style schedulers stop at their `total_steps`).
"""

from __future__ import annotations

from .state import AcceleratorState, GradientState


class AcceleratedScheduler:
    def __init__(self, scheduler, optimizers, step_with_optimizer: bool = True, split_batches: bool = False):
        self.scheduler = scheduler
        self.optimizers = list(optimizers) if isinstance(optimizers, (list, tuple)) else [optimizers]
        self.split_batches = split_batches
        self.step_with_optimizer = step_with_optimizer
        self.gradient_state = GradientState()

    def _advances(self) -> tuple:
        """(scheduler steps this call makes, whether each is bounded by the scheduler's `total_steps`): 0 while
        accumulating or after a skipped optimizer step."""
        if not self.step_with_optimizer:
            return 1, False
        if not self.gradient_state.sync_gradients:
            if self.gradient_state.adjust_scheduler:
                self.scheduler._step_count += 1
            return 0, False
        if any(getattr(opt, "step_was_skipped", False) for opt in self.optimizers):
            return 0, False
        if self.split_batches:
            return 1, False
        return AcceleratorState().num_processes, True

    def step(self, *args, **kwargs):
        count, bounded = self._advances()
        limit = getattr(self.scheduler, "total_steps", None) if bounded else None
        for _ in range(count):
            # bounded schedulers (OneCycleLR) raise past their last step: the per-process repeats stop there
            if limit is None or self.scheduler._step_count <= limit:
                self.scheduler.step(*args, **kwargs)

    # ---- pass-through to the wrapped scheduler
    def __getattr__(self, name):
        if name in ("get_last_lr", "state_dict", "load_state_dict", "get_lr", "print_lr"):
            return getattr(self.__dict__["scheduler"], name)
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")
