"""Model-family tests on CPU (fp32 reference kernels): MoE routing/grouped experts vs a per-token oracle, Mixtral
forward/backward + HF-checkpoint key mapping, parameter/FLOP accounting."""

import copy

import pytest
import torch

from accelerate_hpc_test_amd.models.mixtral import MIXTRAL_PRESETS, MixtralConfig, MixtralForCausalLM
from accelerate_hpc_test_amd.models.moe import MoELayer, load_balancing_loss


def _naive_moe(layer: MoELayer, x):
    t = x.reshape(-1, x.shape[-1])
    probs = torch.softmax(layer.gate(t).float(), -1)
    w, idx = torch.topk(probs, layer.top_k, -1)
    w = w / w.sum(-1, keepdim=True)
    out = torch.zeros_like(t)
    for i in range(t.shape[0]):
        for j in range(layer.top_k):
            e = idx[i, j]
            h = t[i] @ layer.experts.w_gate_up[e].t()
            g, u = h.chunk(2)
            a = torch.nn.functional.silu(g) * u
            out[i] += w[i, j] * (a @ layer.experts.w_down[e].t())
    return out.view_as(x)


def test_moe_matches_naive_forward_and_backward():
    torch.manual_seed(0)
    layer = MoELayer(hidden=16, intermediate=24, num_experts=4, top_k=2)
    for p in layer.parameters():
        torch.nn.init.normal_(p, std=0.3)
    ref = copy.deepcopy(layer)
    x = torch.randn(2, 5, 16)
    x1, x2 = x.clone().requires_grad_(), x.clone().requires_grad_()
    y = layer(x1)
    y_ref = _naive_moe(ref, x2)
    assert torch.allclose(y, y_ref, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    y_ref.backward(g)
    assert torch.allclose(x1.grad, x2.grad, atol=1e-5)
    for (n, p), q in zip(layer.named_parameters(), ref.parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5), n


def test_moe_unused_expert_gets_zero_grad():
    torch.manual_seed(0)
    layer = MoELayer(hidden=8, intermediate=8, num_experts=4, top_k=1)
    with torch.no_grad():
        layer.gate.weight.zero_()
        layer.gate.weight[0].fill_(10.0)  # everything routes to expert 0 for positive inputs
    torch.nn.init.normal_(layer.experts.w_gate_up)
    torch.nn.init.normal_(layer.experts.w_down)
    x = torch.rand(3, 8) + 0.1
    layer(x).sum().backward()
    assert layer.experts.w_gate_up.grad[1:].abs().sum() == 0
    assert layer.experts.w_gate_up.grad[0].abs().sum() > 0


def test_mixtral_tiny_trains():
    torch.manual_seed(0)
    model = MixtralForCausalLM(MIXTRAL_PRESETS["mixtral-tiny"])
    model.init_weights()
    opt = torch.optim.AdamW(model.parameters(), lr=3e-3)
    ids = torch.randint(0, 512, (2, 32))
    losses = []
    for _ in range(4):
        out = model(ids, labels=ids, output_router_logits=True)
        out.loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(out.loss.item())
    assert losses[-1] < losses[0]


def test_load_balancing_loss_balanced_is_one():
    # every expert receives 1/E of the tokens and 1/E of the probability mass → E · Σ_e (1/E)(1/E) = 1
    probs_even = [torch.log(torch.eye(4).repeat(4, 1) * 0.9 + 0.025)]
    assert abs(load_balancing_loss(probs_even, 4, 1).item() - 1.0) < 1e-4
    # all tokens on one expert with all the mass → E
    skewed = [torch.log(torch.tensor([[0.97, 0.01, 0.01, 0.01]]).repeat(8, 1))]
    assert abs(load_balancing_loss(skewed, 4, 1).item() - 4 * 0.97) < 1e-3


def test_mixtral_param_count_8x7b():
    cfg = MIXTRAL_PRESETS["mixtral-8x7b"]
    assert 46.5e9 < cfg.num_params < 46.9e9
    assert 12.7e9 < cfg.active_params < 13.2e9


def test_mixtral_hf_key_mapping():
    cfg = MixtralConfig(vocab_size=64, hidden_size=32, intermediate_size=48, num_hidden_layers=1, num_attention_heads=2,
                        num_key_value_heads=1, head_dim=16, num_local_experts=2)
    model = MixtralForCausalLM(cfg)
    H, I = 32, 48
    sd = {"model.embed_tokens.weight": torch.randn(64, H), "model.norm.weight": torch.ones(H), "lm_head.weight": torch.randn(64, H)}
    p = "model.layers.0."
    sd[p + "self_attn.q_proj.weight"] = torch.randn(32, H)
    sd[p + "self_attn.k_proj.weight"] = torch.randn(16, H)
    sd[p + "self_attn.v_proj.weight"] = torch.randn(16, H)
    sd[p + "self_attn.o_proj.weight"] = torch.randn(H, 32)
    sd[p + "input_layernorm.weight"] = torch.ones(H)
    sd[p + "post_attention_layernorm.weight"] = torch.ones(H)
    sd[p + "block_sparse_moe.gate.weight"] = torch.randn(2, H)
    for e in range(2):
        sd[p + f"block_sparse_moe.experts.{e}.w1.weight"] = torch.randn(I, H)
        sd[p + f"block_sparse_moe.experts.{e}.w3.weight"] = torch.randn(I, H)
        sd[p + f"block_sparse_moe.experts.{e}.w2.weight"] = torch.randn(H, I)
    model.load_hf_state_dict(sd)
    ex = model.layers[0].block_sparse_moe.experts
    assert torch.equal(ex.w_gate_up[1, :I], sd[p + "block_sparse_moe.experts.1.w1.weight"])
    assert torch.equal(ex.w_gate_up[1, I:], sd[p + "block_sparse_moe.experts.1.w3.weight"])
    assert torch.equal(ex.w_down[0], sd[p + "block_sparse_moe.experts.0.w2.weight"])


def test_llama_fp32_params_under_bf16_autocast():
    """DDP-style mixed precision (fp32 params, Accelerator autocast): bf16 activations, fp32 grads, loss tracks the
    fp32 model."""
    from accelerate_hpc_test_amd import Accelerator
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM

    torch.manual_seed(0)
    model = LlamaForCausalLM(LLAMA_PRESETS["llama-tiny"])
    model.init_weights()
    ids = torch.randint(0, LLAMA_PRESETS["llama-tiny"].vocab_size, (2, 32))
    ref = model(ids, labels=ids).loss.item()
    acc = Accelerator(cpu=True, mixed_precision="bf16")
    pm = acc.prepare(model)
    seen = []
    h = pm.layers[0].self_attn.qkv_proj.register_forward_hook(lambda m, i, o: seen.append((i[0].dtype, o.dtype)))
    loss = pm(ids, labels=ids).loss
    h.remove()
    acc.backward(loss)
    assert seen[0] == (torch.bfloat16, torch.bfloat16)
    assert all(p.grad is not None and p.grad.dtype == torch.float32 for p in model.parameters())
    assert abs(loss.item() - ref) < 0.05 * abs(ref)
