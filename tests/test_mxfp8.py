"""MXFP8 block scaling (TE `MXFP8BlockScaling` parity, reference `utils/transformer_engine.py:165-186`): the PyTorch
reference quantiser / GEMM that the HIP kernels are checked against on the GPU (tests/test_kernels_gpu.py), the grouped
scale layout, the MX linear's autograd on the CPU path, and the recipe plumbing (`use_mxfp8_block_scaling`)."""

import pytest
import torch
import torch.nn as nn

from accelerate_hpc_test_amd.ops import fp8
from accelerate_hpc_test_amd.utils.dataclasses import TERecipeKwargs


def test_grouped_scale_layout_is_a_permutation():
    pos = fp8._mx_pos(64)
    assert sorted(pos.tolist()) == list(range(64))
    # block 8g + 2q + hf sits at byte 8g + 4hf + q: one dword = one fragment lane's scales for four 64-wide K-tiles
    for b in range(64):
        g, q, hf = b // 8, (b % 8) // 2, b % 2
        assert pos[b].item() == 8 * g + 4 * hf + q


@pytest.mark.parametrize("e5m2", [False, True])
def test_reference_quantiser_scale_rounds_up_and_bounds_error(e5m2):
    torch.manual_seed(0)
    x = torch.randn(64, 512) * torch.logspace(-3, 3, 512)  # blocks of very different magnitude
    x[3, 64:96] = 0.0  # an all-zero block
    q, s = fp8._mx_quant_rows(x.to(torch.bfloat16), e5m2)
    fmax = fp8.E5M2_MAX if e5m2 else fp8.E4M3_MAX
    sn = fp8.mx_scales_natural(s).float() - 127.0  # log2 of every block's scale
    amax = x.to(torch.bfloat16).float().reshape(64, 16, 32).abs().amax(-1)
    nz = amax > 0
    # smallest power of two with amax / scale <= fp8_max
    assert torch.all(amax[nz] / torch.exp2(sn[nz]) <= fmax)
    assert torch.all(amax[nz] / torch.exp2(sn[nz] - 1) > fmax * (1 - 1e-6))
    assert s[3, fp8._mx_pos(16)[2]].item() == 0 and torch.all(q[3, 64:96].float() == 0)
    deq = fp8.mx_dequant(q, s)
    ref = x.to(torch.bfloat16).float()
    # per-element error within half an fp8 ulp of the block's scale range
    rel = 2.0 ** (-3 if not e5m2 else -2)
    bound = (torch.exp2(sn) * fmax).repeat_interleave(32, dim=1) * rel
    assert torch.all((deq - ref).abs() <= bound)


def test_reference_quant_colwise_is_quantised_transpose():
    torch.manual_seed(1)
    x = torch.randn(256, 512, dtype=torch.bfloat16)
    q, s, qt, st = fp8.mx_quant(x, False, True)
    assert q.shape == (256, 512) and s.shape == (256, 16) and qt.shape == (512, 256) and st.shape == (512, 8)
    q2, s2 = fp8._mx_quant_rows(x.t().contiguous(), False)
    assert torch.equal(qt.view(torch.uint8), q2.view(torch.uint8)) and torch.equal(st, s2)


def test_reference_mx_gemm_close_to_fp32():
    torch.manual_seed(2)
    a = torch.randn(256, 512, dtype=torch.bfloat16)
    b = torch.randn(256, 512, dtype=torch.bfloat16)
    aq, as_ = fp8.mx_quant(a, False, False)
    bq, bs = fp8.mx_quant(b, False, False)
    bias = torch.randn(256, dtype=torch.bfloat16)
    c = fp8.mx_gemm(aq, bq, as_, bs, bias, torch.float32)
    ref = a.float() @ b.float().t() + bias.float()
    assert ((c - ref).norm() / ref.norm()).item() < 4e-2
    out = torch.ones(256, 256)
    fp8.mx_gemm(aq, bq, as_, bs, bias, out=out, accumulate=True)
    assert torch.allclose(out, c + 1, atol=1e-4)


def test_mx_linear_autograd_cpu_path_matches_bf16():
    torch.manual_seed(3)
    lin = nn.Linear(512, 256, bias=True).to(torch.bfloat16)
    ref = nn.Linear(512, 256, bias=True).to(torch.bfloat16)
    ref.load_state_dict(lin.state_dict())
    lin.__class__ = fp8.Fp8Linear
    lin.fp8_recipe = fp8.Fp8Recipe(mx=True, fmt="HYBRID")
    x = torch.randn(2, 128, 512, dtype=torch.bfloat16, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    y = lin(x)
    y2 = ref(x2)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    (y2.float() * g.float()).sum().backward()
    rel = lambda p, q: ((p.float() - q.float()).norm() / q.float().norm()).item()  # noqa: E731
    assert rel(y, y2) < 5e-2
    assert rel(x.grad, x2.grad) < 1e-1  # e5m2 gradients
    assert rel(lin.weight.grad, ref.weight.grad) < 1e-1
    assert rel(lin.bias.grad, ref.bias.grad) < 1e-2


def test_mx_linear_falls_back_to_bf16_for_untileable_shapes():
    lin = nn.Linear(128, 64).to(torch.bfloat16)
    lin.__class__ = fp8.Fp8Linear
    lin.fp8_recipe = fp8.Fp8Recipe(mx=True)
    x = torch.randn(8, 128, dtype=torch.bfloat16)
    assert torch.equal(lin(x), nn.functional.linear(x, lin.weight, lin.bias))


def _mlp():
    return nn.Sequential(nn.Linear(256, 512), nn.Linear(512, 512), nn.Linear(512, 256), nn.Linear(256, 256))


def test_convert_with_mxfp8_recipe():
    m = _mlp()
    fp8.convert_model_to_fp8(m, recipe=TERecipeKwargs(use_mxfp8_block_scaling=True), backend="TE")
    inner = [x for x in m.modules() if isinstance(x, fp8.Fp8Linear)]
    assert len(inner) == 2 and all(x.fp8_recipe.mx and not x.fp8_recipe.delayed for x in inner)


def test_convert_env_flag_and_rejected_fields(monkeypatch):
    monkeypatch.setenv("ACCELERATE_FP8_USE_MXFP8_BLOCK_SCALING", "1")
    m = _mlp()
    fp8.convert_model_to_fp8(m, recipe=TERecipeKwargs(), backend="TE")
    assert all(x.fp8_recipe.mx for x in m.modules() if isinstance(x, fp8.Fp8Linear))
    for bad in (dict(amax_history_len=16), dict(amax_compute_algo="max")):
        with pytest.raises(ValueError, match="not supported for MXFP8"):
            fp8.convert_model_to_fp8(_mlp(), recipe=TERecipeKwargs(**bad), backend="TE")
