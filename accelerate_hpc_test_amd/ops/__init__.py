"""MI355X HIP kernels exposed as PyTorch ops (see csrc/kernels/*.hip)."""

from ._ext import available as native_available
from .fused import (
    apply_rope,
    attention_reference,
    cross_entropy,
    flash_attention_qkv,
    flash_attn_with_lse,
    rms_norm,
    rope_tables,
    swiglu,
)
from .multi_tensor import FusedAdamStep, clip_grads_by_total_sq, grad_sq_norm
