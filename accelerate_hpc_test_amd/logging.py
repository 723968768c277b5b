"""Multi-process aware logging.

Parity: `/root/reference/src/accelerate/logging.py:23-126`. `get_logger(name, log_level)` returns an adapter whose
records are emitted by the main process only, unless a call passes `main_process_only=False` (every process logs) or
`in_order=True` without `main_process_only` (every process logs, rank by rank, all ranks meeting at a barrier after
each); `warning_once` deduplicates.
`ACCELERATE_LOG_LEVEL` sets the level when none is given.
"""

from __future__ import annotations

import functools
import logging
import os


def _process_state():
    from .state import PartialState

    if PartialState._shared_state == {}:
        raise RuntimeError(
            "You must initialize the accelerate state by calling either `PartialState()` or `Accelerator()` before "
            "using the logging utility."
        )
    return PartialState()


class MultiProcessAdapter(logging.LoggerAdapter):
    def _emit(self, level, msg, args, kwargs):
        msg, kwargs = self.process(msg, kwargs)
        # one more frame (this helper) between the caller's `stacklevel` and Logger.log
        self.logger.log(level, msg, *args, **{**kwargs, "stacklevel": kwargs.get("stacklevel", 1) + 1})

    def log(self, level, msg, *args, **kwargs):
        state = _process_state()
        explicit_main_only = "main_process_only" in kwargs
        main_only = kwargs.pop("main_process_only", True)
        in_order = kwargs.pop("in_order", False) and not explicit_main_only  # an explicit main_process_only wins
        kwargs.setdefault("stacklevel", 2)
        enabled = self.isEnabledFor(level)
        if in_order and state.num_processes > 1:
            # every rank in turn, ALL ranks joining every barrier (the reference lets the main process log and return
            # while the others wait on barriers it never enters) — also the ranks whose level filters the record out
            # (per-rank levels are common: INFO on main, WARNING elsewhere), or the others would block on them
            for rank in range(state.num_processes):
                if rank == state.process_index and enabled:
                    self._emit(level, msg, args, kwargs)
                state.wait_for_everyone()
            return
        if not enabled:
            return
        if not main_only or state.is_main_process:
            self._emit(level, msg, args, kwargs)

    @functools.lru_cache(None)
    def warning_once(self, *args, **kwargs):
        """`warning`, emitted once per distinct argument tuple."""
        self.warning(*args, **kwargs)


def get_logger(name: str, log_level: str | None = None):
    """A `MultiProcessAdapter` over `logging.getLogger(name)`; `log_level` (or ACCELERATE_LOG_LEVEL) sets its level and
    the root logger's."""
    level = log_level if log_level is not None else os.environ.get("ACCELERATE_LOG_LEVEL")
    logger = logging.getLogger(name)
    if level is not None:
        logger.setLevel(level.upper())
        logger.root.setLevel(level.upper())
    return MultiProcessAdapter(logger, {})
