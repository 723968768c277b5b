"""Llama-family decoder (Llama-2/3/3.1/3.2 shapes) built on the MI355X kernels.

Design choices for CDNA4:
* fused projections: one QKV GEMM (H → (Hq + 2·Hkv)·D) and one gate|up GEMM (H → 2F) — fewer, larger hipBLASLt
  GEMMs; the QKV output is consumed in place by RoPE and flash attention (strided heads, no transposes);
* RMSNorm is fused with the residual add (one pass writes both the normalised activation and the residual);
* SwiGLU, RoPE, flash attention and cross-entropy are HIP kernels (`ops/fused.py`); cross-entropy overwrites the
  logits with their gradient in backward;
* labels are shifted once (not the logits), so no logits-sized copy is made.

`LlamaForCausalLM.from_hf_state_dict` maps HF checkpoints (q/k/v_proj, gate/up_proj) onto the fused layout.
The module exposes `_no_split_modules = ["LlamaDecoderLayer"]` so FSDP transformer wrapping and the big-model
device-map planner treat each decoder layer as one unit, as they do for the reference's HF models.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.fp8 import fp8_tensorwise
from ..ops.fused import apply_rope, cross_entropy, flash_attention_qkv, rms_norm, rope_tables, swiglu


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    initializer_range: float = 0.02
    activation_checkpointing: bool = False

    @property
    def num_params(self) -> int:
        H, F_, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        D, Hq, Hkv = self.head_dim, self.num_attention_heads, self.num_key_value_heads
        per_layer = H * (Hq + 2 * Hkv) * D + Hq * D * H + 3 * H * F_ + 2 * H
        emb = V * H * (1 if self.tie_word_embeddings else 2)
        return L * per_layer + emb + H

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs per token: 6·N (matmuls, fwd+bwd) + causal attention 6·L·S·Hq·D (≈ half of 12·L·S·Hq·D).
        Unlike the reference's helper (examples/torch_native_parallelism/utils.py:94-115) the attention term keeps
        the head dimension."""
        H, L = self.hidden_size, self.num_hidden_layers
        # decoder matmul weights (norm weights excluded) + the lm_head GEMM; the embedding lookup is not a matmul
        n_matmul = self.num_params - self.vocab_size * H * (1 if self.tie_word_embeddings else 2) - H - 2 * H * L
        n_matmul += self.vocab_size * H
        attn = 6 * self.num_hidden_layers * seq_len * self.num_attention_heads * self.head_dim
        return 6 * n_matmul + attn


LLAMA_PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3.1-8b": LlamaConfig(
        rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                      "original_max_position_embeddings": 8192},
        max_position_embeddings=131072,
    ),
    "llama3-70b": LlamaConfig(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64),
    "llama3.2-1b": LlamaConfig(hidden_size=2048, intermediate_size=8192, num_hidden_layers=16, num_attention_heads=32,
                               head_dim=64, tie_word_embeddings=True),
    "llama3.2-3b": LlamaConfig(hidden_size=3072, intermediate_size=8192, num_hidden_layers=28, num_attention_heads=24,
                               tie_word_embeddings=True),
    # small configs for tests / smoke runs (head_dim 128 so the HIP attention path is exercised)
    "llama-tiny": LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                              num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=1024),
    "llama-small": LlamaConfig(vocab_size=32000, hidden_size=1024, intermediate_size=2816, num_hidden_layers=4,
                               num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=4096),
}


class RMSNorm(nn.Module):
    def __init__(self, hidden_size: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.eps = eps

    def forward(self, x, residual=None, amax: bool = False, grad_amax: bool = False):
        # fp32 weights under autocast (DDP mixed precision): the fused kernel runs in the activation dtype.
        w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
        # FSDP: the backward writes dweight straight into the weight's gradient slot (parallel/fsdp.py)
        slot = getattr(self.weight, "_acc_wgrad_slot", None) if w is self.weight else None
        return rms_norm(x, w, self.eps, residual, amax=amax, grad_amax=grad_amax, slot=slot)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.n_q, self.n_kv, self.head_dim = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        self.qkv_proj = nn.Linear(cfg.hidden_size, (self.n_q + 2 * self.n_kv) * self.head_dim, bias=False)
        self.o_proj = nn.Linear(self.n_q * self.head_dim, cfg.hidden_size, bias=False)
        # Optional ring / Ulysses attention installed by parallel/context_parallel.py.
        self.attention_impl = None

    def shard_heads(self, tp_size: int):
        """Called by parallel/tensor_parallel.py after the qkv/o projections were sharded over `tp_size` ranks."""
        if self.n_q % tp_size or self.n_kv % tp_size:
            raise ValueError(f"tp={tp_size} must divide both head counts ({self.n_q} q, {self.n_kv} kv)")
        self.n_q //= tp_size
        self.n_kv //= tp_size

    def forward(self, x, cos, sin, position_ids=None):
        B, S = x.shape[0], x.shape[1]
        qkv = self.qkv_proj(x)
        S = qkv.shape[1]  # sequence-parallel TP gathers the sequence inside qkv_proj
        qkv = qkv.view(B, S, self.n_q + 2 * self.n_kv, self.head_dim)
        qkv = apply_rope(qkv, cos, sin, self.n_q + self.n_kv, position_ids)
        if self.attention_impl is not None:
            o = self.attention_impl(qkv, self.n_q, self.n_kv)
        else:
            o = flash_attention_qkv(qkv, self.n_q, self.n_kv, causal=True)
        return self.o_proj(o.reshape(B, S, self.n_q * self.head_dim))


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_up_proj = nn.Linear(cfg.hidden_size, 2 * cfg.intermediate_size, bias=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x):
        h = swiglu(self.gate_up_proj(x), amax=fp8_tensorwise(self.down_proj), grad_amax=fp8_tensorwise(self.gate_up_proj))
        return self.down_proj(h)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, layer_idx: int = 0):
        super().__init__()
        self.layer_idx = layer_idx
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)

    def forward(self, hidden, residual, cos, sin, position_ids=None):
        # fp8 producer amax: each norm tags its output for the fp8 projection it feeds and its input gradient for the
        # fp8 projection that produced `hidden` (the previous layer's down_proj, this layer's o_proj)
        attn, mlp = self.self_attn, self.mlp
        x, residual = self.input_layernorm(hidden, residual, amax=fp8_tensorwise(attn.qkv_proj),
                                           grad_amax=residual is not None and fp8_tensorwise(mlp.down_proj))
        hidden = attn(x, cos, sin, position_ids)
        x, residual = self.post_attention_layernorm(hidden, residual, amax=fp8_tensorwise(mlp.gate_up_proj),
                                                    grad_amax=fp8_tensorwise(attn.o_proj))
        hidden = mlp(x)
        return hidden, residual


@dataclass
class CausalLMOutput:
    loss: Optional[torch.Tensor] = None
    logits: Optional[torch.Tensor] = None

    def __getitem__(self, k):
        return getattr(self, k) if isinstance(k, str) else (self.loss, self.logits)[k]


class LlamaForCausalLM(nn.Module):
    _no_split_modules = ["LlamaDecoderLayer"]

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.embed_tokens.weight
        self._rope_cache = {}

    # ----- init -----------------------------------------------------------------------------------------
    @torch.no_grad()
    def init_weights(self, module: Optional[nn.Module] = None):
        """HF-style init: N(0, 0.02) for linears/embeddings, ones for norms. Works on any submodule (used by the
        FSDP engine to materialise meta-device units directly on the GPU)."""
        std = self.config.initializer_range
        for m in (module or self).modules():
            if isinstance(m, nn.Linear):
                m.weight.normal_(0.0, std)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.Embedding):
                m.weight.normal_(0.0, std)
            elif isinstance(m, RMSNorm):
                m.weight.fill_(1.0)

    def _rope(self, S, device):
        key = (S, str(device))
        if key not in self._rope_cache:
            n = max(S, self.config.max_position_embeddings if S > self.config.max_position_embeddings else S)
            self._rope_cache[key] = rope_tables(n, self.config.head_dim, self.config.rope_theta, device, self.config.rope_scaling)
        return self._rope_cache[key]

    def forward(self, input_ids, labels=None, position_ids=None, attention_mask=None, return_logits: bool = True,
                shift_labels=None):
        """`labels` are shifted inside (HF convention). Under context/sequence parallelism pass `shift_labels`
        (already shifted on the full sequence, then sharded) instead."""
        B, S = input_ids.shape
        if position_ids is None and getattr(self, "_cp_position_ids", None) is not None:
            position_ids = self._cp_position_ids  # global positions of this rank's context-parallel shard
        rope_len = S
        if position_ids is not None:
            rope_len = max(int(self.config.max_position_embeddings), getattr(self, "_cp_seq_len", None) or 0,
                           S * getattr(self, "_seq_parallel_factor", 1))
        cos, sin = self._rope(rope_len, input_ids.device)
        h = self.embed_tokens(input_ids)
        dt = self.layers[0].self_attn.qkv_proj.weight.dtype if len(self.layers) else h.dtype
        if h.device.type in ("cuda", "cpu") and torch.is_autocast_enabled(h.device.type):
            dt = torch.get_autocast_dtype(h.device.type)  # fp32 master params, bf16 activations (autocast)
        if h.dtype != dt:
            h = h.to(dt)
        residual = None
        for layer in self.layers:
            h, residual = layer(h, residual, cos, sin, position_ids)
        h, _ = self.norm(h, residual, grad_amax=len(self.layers) > 0 and fp8_tensorwise(self.layers[-1].mlp.down_proj))
        logits = self.lm_head(h)
        loss = None
        if shift_labels is None and labels is not None:
            shift_labels = torch.full_like(labels, -100)
            shift_labels[:, :-1] = labels[:, 1:]
        if shift_labels is not None:
            loss = cross_entropy(logits, shift_labels, ignore_index=-100, inplace_backward=not return_logits)
        return CausalLMOutput(loss=loss, logits=logits if return_logits else None)

    # ----- tensor parallelism ---------------------------------------------------------------------------
    def tp_plan(self, sequence_parallel: bool = False) -> dict:
        """Megatron layout for parallel/tensor_parallel.py: fused qkv / gate|up sharded per segment (whole heads,
        matching gate and up rows), o/down row-parallel, lm_head column-parallel with gathered logits."""
        c = self.config
        qkv = [c.num_attention_heads * c.head_dim, c.num_key_value_heads * c.head_dim, c.num_key_value_heads * c.head_dim]
        from ..parallel.tensor_parallel import ColwiseParallel, RowwiseParallel

        plan = {
            "layers.*.self_attn.qkv_proj": ColwiseParallel(segments=qkv),
            "layers.*.self_attn.o_proj": RowwiseParallel(),
            "layers.*.mlp.gate_up_proj": ColwiseParallel(segments=[c.intermediate_size, c.intermediate_size]),
            "layers.*.mlp.down_proj": RowwiseParallel(),
        }
        if not c.tie_word_embeddings:
            plan["lm_head"] = ColwiseParallel(gather_output=True)
        if sequence_parallel:
            plan.update({
                "embed_tokens": "seq_split",
                "layers.*.input_layernorm": "sequence_parallel",
                "layers.*.post_attention_layernorm": "sequence_parallel",
                "norm": "sequence_parallel",
            })
            if c.tie_word_embeddings:
                raise ValueError("sequence-parallel TP needs an untied lm_head")
        return plan

    # ----- HF interop -----------------------------------------------------------------------------------
    @classmethod
    def hf_key_map(cls, cfg: LlamaConfig):
        return {
            "q_proj": "qkv", "k_proj": "qkv", "v_proj": "qkv",
            "gate_proj": "gate_up", "up_proj": "gate_up",
        }

    def load_hf_state_dict(self, sd: dict, strict: bool = True):
        """Load a HF `LlamaForCausalLM` state dict (model.layers.N.self_attn.q_proj.weight, ...)."""
        out = {}
        L = self.config.num_hidden_layers
        get = lambda k: sd[k] if k in sd else sd["model." + k]  # noqa: E731
        out["embed_tokens.weight"] = get("embed_tokens.weight")
        out["norm.weight"] = get("norm.weight")
        if "lm_head.weight" in sd:
            out["lm_head.weight"] = sd["lm_head.weight"]
        elif self.config.tie_word_embeddings:
            out["lm_head.weight"] = out["embed_tokens.weight"]
        for i in range(L):
            p = f"layers.{i}."
            out[p + "self_attn.qkv_proj.weight"] = torch.cat(
                [get(p + "self_attn.q_proj.weight"), get(p + "self_attn.k_proj.weight"), get(p + "self_attn.v_proj.weight")], 0
            )
            out[p + "self_attn.o_proj.weight"] = get(p + "self_attn.o_proj.weight")
            out[p + "mlp.gate_up_proj.weight"] = torch.cat([get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")], 0)
            out[p + "mlp.down_proj.weight"] = get(p + "mlp.down_proj.weight")
            out[p + "input_layernorm.weight"] = get(p + "input_layernorm.weight")
            out[p + "post_attention_layernorm.weight"] = get(p + "post_attention_layernorm.weight")
        return self.load_state_dict(out, strict=strict)


def build_llama(name_or_config, device=None, dtype=None, meta: bool = False) -> LlamaForCausalLM:
    cfg = LLAMA_PRESETS[name_or_config] if isinstance(name_or_config, str) else name_or_config
    if meta:
        with torch.device("meta"):
            return LlamaForCausalLM(cfg)
    model = LlamaForCausalLM(cfg)
    model.init_weights()
    if device is not None or dtype is not None:
        model.to(device=device, dtype=dtype)
    return model
