"""Non-blocking checkpoint writes (utils/async_checkpoint.py, csrc/runtime/d2h_writer.cpp): the safetensors layout the
writer produces is read back by `safetensors` itself (CPU), and on an MI355X the native writer's snapshot semantics:
the live tensors may change right after `save_file` returns, the file holds the values of the save."""
import os

import pytest
import torch
from safetensors.torch import load_file

from accelerate_hpc_test_amd.utils import async_checkpoint as ac


def test_safetensors_layout_cpu(tmp_path):
    torch.manual_seed(0)
    ts = {"a": torch.randn(3, 5), "b": torch.randn(7).to(torch.bfloat16), "c": torch.randint(0, 9, (4,)),
          "d": torch.randn(6).to(torch.float8_e4m3fn), "e": torch.zeros(0), "f|exp_avg": torch.randn(2, 2).half()}
    path = str(tmp_path / "x.safetensors")
    assert ac.writer().save_file(ts, path, metadata={"format": "pt"}) is False  # CPU: written synchronously
    back = load_file(path)
    assert list(back) == list(ts) or set(back) == set(ts)
    for k, v in ts.items():
        assert back[k].dtype == v.dtype and back[k].shape == v.shape
        assert torch.equal(back[k].view(torch.uint8) if v.dtype == torch.float8_e4m3fn else back[k],
                           v.view(torch.uint8) if v.dtype == torch.float8_e4m3fn else v), k


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_native_writer_snapshot_and_roundtrip(tmp_path):
    torch.manual_seed(0)
    dev = "cuda"
    ts = {"big": torch.randn(40 << 20, device=dev),  # 160 MB: several 64 MB pieces
          "bf": torch.randn(1000, 333, device=dev).to(torch.bfloat16),
          "f8": torch.randn(4097, device=dev).to(torch.float8_e5m2),
          "empty": torch.zeros(0, device=dev), "i": torch.arange(17, device=dev)}
    want = {k: v.cpu().clone() for k, v in ts.items()}
    path = str(tmp_path / "s.safetensors")
    pending = ac.writer().save_file(ts, path)
    assert pending, "a few hundred MB must fit as a device snapshot"
    for v in ts.values():  # the next optimizer step overwriting the live state
        if v.numel():
            v.zero_() if v.dtype != torch.float8_e5m2 else v.copy_(torch.zeros_like(v))
    ac.wait_pending_saves()
    back = load_file(path)
    for k, v in want.items():
        a = back[k].view(torch.uint8) if v.dtype == torch.float8_e5m2 else back[k]
        b = v.view(torch.uint8) if v.dtype == torch.float8_e5m2 else v
        assert torch.equal(a, b), k
    assert os.path.getsize(path) >= (40 << 20) * 4
