"""Optimizer wrapper.

Parity: `/root/reference/src/accelerate/optimizer.py:38-213`: state placement on the device, `zero_grad` and
`step` gated by `GradientState.sync_gradients`, fp16 GradScaler stepping with overflow detection
(`step_was_skipped`), picklability.

MI355X-native addition: when the wrapped optimizer is `torch.optim.AdamW`/`Adam` and its parameters live on
the GPU, `step()` runs our HIP multi-tensor AdamW kernel (`ops/adamw.py`: one launch per dtype group over
chunked tensor lists, reading grad/param/m/v once and optionally writing the bf16 shadow copy that the FSDP
engine all-gathers) instead of torch's foreach implementation. The optimizer's `state` keeps torch's layout
(`step`, `exp_avg`, `exp_avg_sq`) so checkpoints are interchangeable. Set `ACCELERATE_FUSED_ADAMW=0` to
disable.
"""

from __future__ import annotations

import contextlib
import inspect
import os

import torch

from .state import AcceleratorState, GradientState
from .utils.dataclasses import DistributedType
from .utils.operations import honor_type


def move_to_device(state, device):
    """Every tensor of a nested optimizer-state structure moved to `device`; containers keep their types."""
    if isinstance(state, torch.Tensor):
        return state.to(device)
    if isinstance(state, dict):
        return type(state)((k, move_to_device(v, device)) for k, v in state.items())
    if isinstance(state, (list, tuple)):
        return honor_type(state, [move_to_device(v, device) for v in state])
    return state


@contextlib.contextmanager
def _record_inner_steps(optimizer):
    """Within the block, calls of `optimizer.step` are counted into the yielded list. A GradScaler skips the inner
    step when it found inf/nan gradients, so an empty list afterwards means the step was skipped. Whatever `step`
    the instance carried before (e.g. an LR scheduler's call counter) is put back afterwards."""
    own = vars(optimizer).get("step")
    inner = optimizer.step
    calls = []

    def counted(*args, **kwargs):
        calls.append(True)
        return inner(*args, **kwargs)

    optimizer.step = counted
    try:
        yield calls
    finally:
        if own is None:
            del optimizer.step
        else:
            optimizer.step = own


def _has_dtensor(optimizer) -> bool:
    try:
        from torch.distributed.tensor import DTensor
    except ImportError:  # pragma: no cover
        return False
    return any(isinstance(p, DTensor) for g in optimizer.param_groups for p in g["params"])


def _fused_adam_eligible(optimizer):
    """"gpu" (HIP multi-tensor kernel), "cpu" (native OpenMP kernel over CPU-offloaded fp32 shards) or None."""
    if os.environ.get("ACCELERATE_FUSED_ADAMW", "1") == "0" or os.environ.get("ACCELERATE_NATIVE_KERNELS", "1") == "0":
        return None
    if type(optimizer) not in (torch.optim.AdamW, torch.optim.Adam):
        return None
    if _has_dtensor(optimizer):  # DTensor wrappers own no storage: torch's DTensor-aware step
        return None
    devs = set()
    for g in optimizer.param_groups:
        if g.get("amsgrad", False) or g.get("maximize", False) or g.get("capturable", False):
            return None
        if g.get("differentiable", False):
            return None
        for p in g["params"]:
            devs.add("gpu" if p.is_cuda else ("cpu" if p.device.type == "cpu" and p.dtype == torch.float32 else "other"))
    if devs == {"gpu"}:
        return "gpu"
    if devs == {"cpu"} and any(hasattr(p, "_acc_bf16_shadow_host") or getattr(p, "_acc_offloaded", False)
                               for g in optimizer.param_groups for p in g["params"]):
        from .ops import _ext

        return "cpu" if _ext.available() else None
    return None


class AcceleratedOptimizer(torch.optim.Optimizer):
    def __init__(self, optimizer, device_placement=True, scaler=None):
        self.optimizer = optimizer
        self.scaler = scaler
        self.accelerator_state = AcceleratorState()
        self.gradient_state = GradientState()
        self.device_placement = device_placement
        self._is_overflow = False
        self._fused_step = None
        if device_placement:
            state_dict = self.optimizer.state_dict()
            state_dict["state"] = move_to_device(state_dict["state"], self.accelerator_state.device)
            self.optimizer.load_state_dict(state_dict)

    # ---- fused HIP AdamW -------------------------------------------------------------------------
    def _maybe_fused(self):
        if self._fused_step is None:
            kind = _fused_adam_eligible(self.optimizer)
            if kind == "gpu":
                from .ops.multi_tensor import FusedAdamStep

                self._fused_step = FusedAdamStep(self.optimizer)
            elif kind == "cpu":
                from .ops.multi_tensor import CpuFusedAdamStep

                self._fused_step = CpuFusedAdamStep(self.optimizer)
            else:
                self._fused_step = False
        return self._fused_step

    @property
    def state(self):
        return self.optimizer.state

    @state.setter
    def state(self, state):
        self.optimizer.state = state

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @param_groups.setter
    def param_groups(self, param_groups):
        self.optimizer.param_groups = param_groups

    @property
    def defaults(self):
        return self.optimizer.defaults

    @defaults.setter
    def defaults(self, defaults):
        self.optimizer.defaults = defaults

    def add_param_group(self, param_group):
        self.optimizer.add_param_group(param_group)
        self._fused_step = None

    def load_state_dict(self, state_dict):
        self.optimizer.load_state_dict(state_dict)
        self._fused_step = None

    def state_dict(self):
        return self.optimizer.state_dict()

    def zero_grad(self, set_to_none=None):
        """Clear gradients at accumulation boundaries only (`set_to_none` defaults to True where supported)."""
        if not self.gradient_state.sync_gradients:
            return
        if "set_to_none" in inspect.signature(self.optimizer.zero_grad).parameters:
            self.optimizer.zero_grad(set_to_none=True if set_to_none is None else set_to_none)
        elif set_to_none is None:
            self.optimizer.zero_grad()
        else:
            raise ValueError(f"{type(self.optimizer).__name__}.zero_grad() takes no `set_to_none` argument")
        hook = getattr(self.optimizer, "_accelerate_post_zero_grad", None)
        if hook is not None:
            hook()

    def train(self):
        if hasattr(self.optimizer, "train") and callable(self.optimizer.train):
            self.optimizer.train()

    def eval(self):
        if hasattr(self.optimizer, "eval") and callable(self.optimizer.eval):
            self.optimizer.eval()

    # ---- optimizer / backward overlap (RcclKwargs.fsdp_optimizer_overlap) ---------------------------------------
    def enable_overlap(self, engine) -> bool:
        """Let the FSDP engine apply this optimizer unit by unit during backward (see
        `FSDPEngine.attach_overlapped_optimizer`). Not with a GradScaler: fp16 overflow is only known at the end."""
        if self.scaler is not None:
            return False
        self._overlap_engine = engine
        engine.attach_overlapped_optimizer(self._step_subset)
        return True

    def _step_subset(self, params):
        ids = {id(p) for p in params}
        fused = self._maybe_fused()
        if fused:
            fused.step(only=ids)
        else:
            _step_filtered(self.optimizer, only=ids)

    def _inner_step(self, closure=None):
        eng = getattr(self, "_overlap_engine", None)
        done = eng.take_overlapped() if eng is not None else set()
        fused = self._maybe_fused()
        if fused and closure is None:
            fused.step(skip=done or None)
            self.optimizer._acc_last_step_fused = True
        else:
            if done:
                _step_filtered(self.optimizer, skip=done)
            else:
                self.optimizer.step(closure)
            self.optimizer._acc_last_step_fused = False

    def step(self, closure=None):
        if not self.gradient_state.sync_gradients:
            return
        if self.scaler is not None:
            with _record_inner_steps(self.optimizer) as calls:
                self.scaler.step(self.optimizer, closure)
            self.scaler.update()
            self._is_overflow = not calls
            self.optimizer._acc_last_step_fused = False
        else:
            self._inner_step(closure)
        post = getattr(self.optimizer, "_accelerate_post_step", None)
        if post is not None:
            post()

    def _switch_parameters(self, parameters_map):
        for param_group in self.optimizer.param_groups:
            param_group["params"] = [parameters_map.get(p, p) for p in param_group["params"]]
        self._fused_step = None

    @property
    def step_was_skipped(self):
        """Whether the last optimizer step was skipped because of fp16 overflow."""
        return self._is_overflow

    _UNPICKLED = frozenset({"_fused_step", "_overlap_engine"})  # rebuilt lazily / re-attached by the engine

    def __getstate__(self):
        return {k: v for k, v in self.__dict__.items() if k not in self._UNPICKLED}

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._fused_step = None


def _step_filtered(optimizer, only=None, skip=None):
    """`optimizer.step()` restricted to the params whose id() is in `only` / not in `skip` (any torch optimizer: the
    param lists are narrowed for the call, per-param state is keyed by the param itself)."""
    saved = [g["params"] for g in optimizer.param_groups]
    try:
        for g in optimizer.param_groups:
            g["params"] = [p for p in g["params"] if (only is None or id(p) in only) and (skip is None or id(p) not in skip)]
        optimizer.step()
    finally:
        for g, ps in zip(optimizer.param_groups, saved):
            g["params"] = ps

