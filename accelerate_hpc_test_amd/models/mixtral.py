"""Mixtral (sparse MoE decoder) on the MI355X kernels — BASELINE config "Mixtral 8×7B FSDP2 + fp8".

Architecture = Llama attention (fused QKV, RoPE θ=1e6, GQA 32/8, flash attention) + a top-2-of-8 SwiGLU MoE MLP
(`models/moe.py`). `_no_split_modules = ["MixtralDecoderLayer"]` so FSDP wraps one decoder layer per unit (one
all-gather of the layer incl. its 8 experts ≈ 2.8 GB bf16 for 8×7B), like the reference's HF Mixtral under
transformer-based wrapping. HF checkpoints (`block_sparse_moe.experts.N.w1/w2/w3`) map onto the stacked layout via
`load_hf_state_dict`.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from ..ops.fused import cross_entropy, rope_tables
from .llama import CausalLMOutput, LlamaAttention, LlamaConfig, RMSNorm
from .moe import MoEExperts, MoELayer, load_balancing_loss


@dataclass
class MixtralConfig(LlamaConfig):
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    rope_theta: float = 1e6
    max_position_embeddings: int = 32768
    num_local_experts: int = 8
    num_experts_per_tok: int = 2
    router_aux_loss_coef: float = 0.02
    output_router_logits: bool = False

    @property
    def num_params(self) -> int:
        H, F_, L, V, E = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size, self.num_local_experts
        D, Hq, Hkv = self.head_dim, self.num_attention_heads, self.num_key_value_heads
        per_layer = H * (Hq + 2 * Hkv) * D + Hq * D * H + E * 3 * H * F_ + H * E + 2 * H
        return L * per_layer + 2 * V * H + H

    @property
    def active_params(self) -> int:
        H, F_, L, V, E, k = (self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size,
                             self.num_local_experts, self.num_experts_per_tok)
        D, Hq, Hkv = self.head_dim, self.num_attention_heads, self.num_key_value_heads
        per_layer = H * (Hq + 2 * Hkv) * D + Hq * D * H + k * 3 * H * F_ + H * E
        return L * per_layer + V * H  # lm_head GEMM (embedding lookup is free)

    def flops_per_token(self, seq_len: int) -> float:
        return 6 * self.active_params + 6 * self.num_hidden_layers * seq_len * self.num_attention_heads * self.head_dim


MIXTRAL_PRESETS = {
    "mixtral-8x7b": MixtralConfig(),
    "mixtral-8x7b-4l": MixtralConfig(num_hidden_layers=4),  # 1-GPU measurement slice of the full model
    # the deepest slice whose FSDP training state (18 B/param: fp32 master + grad + Adam m, v + bf16 copy, 11.9 B params)
    # plus seq-8192 activations fits one MI355X's 288 GB; the full 46.7 B-param model needs 783 GiB of state on one GPU
    # (98 GiB per GPU at FSDP world size 8), and host offload of it exceeds a 270 GiB host budget as well
    "mixtral-8x7b-8l": MixtralConfig(num_hidden_layers=8),
    "mixtral-tiny": MixtralConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                  num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=1024,
                                  num_local_experts=4),
}


class MixtralDecoderLayer(nn.Module):
    def __init__(self, cfg: MixtralConfig, layer_idx: int = 0):
        super().__init__()
        self.layer_idx = layer_idx
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.block_sparse_moe = MoELayer(cfg.hidden_size, cfg.intermediate_size, cfg.num_local_experts, cfg.num_experts_per_tok)

    def forward(self, hidden, residual, cos, sin, position_ids=None):
        x, residual = self.input_layernorm(hidden, residual)
        hidden = self.self_attn(x, cos, sin, position_ids)
        rec = self.block_sparse_moe.experts.fp8_recipe
        # per-tensor fp8 experts: the norm also produces the abs-max of the routed tokens (no amax pass over them)
        x, residual = self.post_attention_layernorm(hidden, residual, amax=rec is not None and not rec.mx)
        return self.block_sparse_moe(x), residual


class MixtralForCausalLM(nn.Module):
    _no_split_modules = ["MixtralDecoderLayer"]

    def __init__(self, cfg: MixtralConfig):
        super().__init__()
        self.config = cfg
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([MixtralDecoderLayer(cfg, i) for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias=False)
        self._rope_cache = {}

    @torch.no_grad()
    def init_weights(self, module: Optional[nn.Module] = None):
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
            elif isinstance(m, MoEExperts):
                m.w_gate_up.normal_(0.0, std)
                m.w_down.normal_(0.0, std)

    def enable_expert_parallel(self, group, device=None):
        """Shard every layer's experts over `group` onto `device` (see models/moe.py). Returns the expert modules,
        which the FSDP engine must leave alone (they are already sharded)."""
        from ..parallel import comm

        mods, need_init = [], []
        for layer in self.layers:
            if layer.block_sparse_moe.shard_experts(group, device):
                need_init.append(layer.block_sparse_moe.experts)
            mods.append(layer.block_sparse_moe.experts)
        if need_init and device is not None:
            # meta-device model: initialise the local experts directly where they live (per-rank seed)
            state = torch.cuda.get_rng_state(device) if torch.device(device).type == "cuda" else torch.get_rng_state()
            torch.manual_seed(7919 + 104729 * comm.group_rank(group))
            for m in need_init:
                self.init_weights(m)
            if torch.device(device).type == "cuda":
                torch.cuda.set_rng_state(state, device)
            else:
                torch.set_rng_state(state)
        self._ep_group = group
        return mods

    def _rope(self, S, device):
        key = (S, str(device))
        if key not in self._rope_cache:
            self._rope_cache[key] = rope_tables(S, self.config.head_dim, self.config.rope_theta, device, self.config.rope_scaling)
        return self._rope_cache[key]

    def forward(self, input_ids, labels=None, position_ids=None, attention_mask=None, return_logits: bool = True,
                shift_labels=None, output_router_logits: Optional[bool] = None):
        B, S = input_ids.shape
        rope_len = S if position_ids is None else max(S, int(self.config.max_position_embeddings))
        cos, sin = self._rope(rope_len, input_ids.device)
        h = self.embed_tokens(input_ids)
        dt = self.layers[0].self_attn.qkv_proj.weight.dtype if len(self.layers) else h.dtype
        if h.device.type in ("cuda", "cpu") and torch.is_autocast_enabled(h.device.type):
            dt = torch.get_autocast_dtype(h.device.type)
        if h.dtype != dt:
            h = h.to(dt)
        residual = None
        for layer in self.layers:
            h, residual = layer(h, residual, cos, sin, position_ids)
        h, _ = self.norm(h, residual)
        logits = self.lm_head(h)
        loss = None
        if shift_labels is None and labels is not None:
            shift_labels = torch.full_like(labels, -100)
            shift_labels[:, :-1] = labels[:, 1:]
        if shift_labels is not None:
            loss = cross_entropy(logits, shift_labels, ignore_index=-100, inplace_backward=not return_logits)
            want_aux = self.config.output_router_logits if output_router_logits is None else output_router_logits
            if want_aux and self.config.router_aux_loss_coef > 0:
                aux = load_balancing_loss([l.block_sparse_moe.last_router_logits for l in self.layers],
                                          self.config.num_local_experts, self.config.num_experts_per_tok)
                loss = loss + self.config.router_aux_loss_coef * aux.to(loss.dtype)
        for l in self.layers:
            l.block_sparse_moe.last_router_logits = None
        return CausalLMOutput(loss=loss, logits=logits if return_logits else None)

    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict, strict: bool = True):
        """Map HF Mixtral keys (q/k/v_proj, block_sparse_moe.experts.N.w1/w3/w2, gate) onto the fused layout."""
        get = lambda k: sd[k] if k in sd else sd["model." + k]  # noqa: E731
        out = {"embed_tokens.weight": get("embed_tokens.weight"), "norm.weight": get("norm.weight"), "lm_head.weight": sd["lm_head.weight"]}
        E = self.config.num_local_experts
        for i in range(self.config.num_hidden_layers):
            p = f"layers.{i}."
            out[p + "self_attn.qkv_proj.weight"] = torch.cat([get(p + f"self_attn.{n}_proj.weight") for n in "qkv"], 0)
            out[p + "self_attn.o_proj.weight"] = get(p + "self_attn.o_proj.weight")
            out[p + "input_layernorm.weight"] = get(p + "input_layernorm.weight")
            out[p + "post_attention_layernorm.weight"] = get(p + "post_attention_layernorm.weight")
            out[p + "block_sparse_moe.gate.weight"] = get(p + "block_sparse_moe.gate.weight")
            ex = p + "block_sparse_moe.experts."
            out[ex + "w_gate_up"] = torch.stack([torch.cat([get(f"{ex}{e}.w1.weight"), get(f"{ex}{e}.w3.weight")], 0) for e in range(E)])
            out[ex + "w_down"] = torch.stack([get(f"{ex}{e}.w2.weight") for e in range(E)])
        return self.load_state_dict(out, strict=strict)


def build_mixtral(name_or_config, device=None, dtype=None, meta: bool = False) -> MixtralForCausalLM:
    cfg = MIXTRAL_PRESETS[name_or_config] if isinstance(name_or_config, str) else name_or_config
    if meta:
        with torch.device("meta"):
            return MixtralForCausalLM(cfg)
    model = MixtralForCausalLM(cfg)
    model.init_weights()
    if device is not None or dtype is not None:
        model.to(device=device, dtype=dtype)
    return model
