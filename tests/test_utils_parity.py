"""Reference tests/test_utils.py and tests/test_kwargs_handlers.py topics, pinned against the upstream accelerate
installed in the image (skipped without it): pure helpers give the same results, kwargs handlers emit the same
non-default kwargs, and environment helpers behave the same."""

import collections
import os
from datetime import timedelta

import pytest
import torch

import accelerate_hpc_test_amd.utils as ours

up = pytest.importorskip("accelerate.utils")

Point = collections.namedtuple("Point", "x y")


def test_tensor_structure_helpers_match_upstream():
    nested = {"a": torch.arange(6).view(3, 2), "b": [torch.ones(3), (torch.zeros(3, 1), Point(torch.arange(3), torch.arange(3.0)))]}
    for fn in ("listify", "find_batch_size"):
        assert getattr(ours, fn)(nested) == getattr(up, fn)(nested), fn
    a, b = ours.slice_tensors(nested, slice(0, 2)), up.slice_tensors(nested, slice(0, 2))
    assert ours.listify(a) == up.listify(b)
    assert isinstance(a["b"][1][1], Point)
    parts = [{"x": torch.ones(2, 3), "y": [torch.zeros(2)]}, {"x": torch.zeros(1, 3), "y": [torch.ones(1)]}]
    assert ours.listify(ours.concatenate(parts)) == up.listify(up.concatenate(parts))
    assert type(ours.honor_type(Point(1, 2), iter([3, 4]))) is Point
    assert ours.honor_type(Point(1, 2), iter([3, 4])) == up.honor_type(Point(1, 2), iter([3, 4]))
    assert ours.is_namedtuple(Point(1, 2)) and not ours.is_namedtuple((1, 2))


def test_misc_helpers_match_upstream():
    d1 = {"a": {"b": 1, "c": {"d": 2}}, "e": 3}
    d2 = {"a": {"c": {"f": 4}}, "g": 5}
    assert ours.merge_dicts(dict(d2), {k: (dict(v) if isinstance(v, dict) else v) for k, v in d1.items()}) == \
        up.merge_dicts(dict(d2), {k: (dict(v) if isinstance(v, dict) else v) for k, v in d1.items()})
    for n in (0, 1023, 1024, 5 * 2**20, 3 * 2**30 + 7):
        assert ours.convert_bytes(n) == up.convert_bytes(n), n
    m = torch.nn.Sequential(torch.nn.Linear(2, 2))
    assert ours.recursive_getattr(m, "0.weight") is up.recursive_getattr(m, "0.weight")
    for obj in (m, torch.nn.Linear, 3):
        assert ours.get_pretty_name(obj) == up.get_pretty_name(obj)


def test_extract_model_from_parallel_compiled_module():
    m = torch.nn.Linear(3, 3)
    comp = torch.compile(m, backend="eager")
    for keep in (True, False):  # upstream default keeps the compiled wrapper
        want = up.extract_model_from_parallel(comp, keep_torch_compile=keep)
        assert ours.extract_model_from_parallel(comp, keep_torch_compile=keep) is want
    assert ours.extract_model_from_parallel(comp, keep_torch_compile=False) is m


@pytest.mark.parametrize("name,kw", [
    ("AutocastKwargs", {"enabled": False}),
    ("AutocastKwargs", {"cache_enabled": True}),
    ("GradScalerKwargs", {"init_scale": 1024, "growth_interval": 10}),
    ("InitProcessGroupKwargs", {"timeout": timedelta(seconds=42)}),
    ("DistributedDataParallelKwargs", {"find_unused_parameters": True, "bucket_cap_mb": 15}),
])
def test_kwargs_handlers_emit_the_same_non_default_kwargs(name, kw):
    assert getattr(ours, name)(**kw).to_kwargs() == getattr(up, name)(**kw).to_kwargs()


def test_environment_helpers():
    with ours.clear_environment():
        assert "PATH" not in os.environ
    assert "PATH" in os.environ
    with ours.patch_environment(acc_test_var="1"):
        assert os.environ["ACC_TEST_VAR"] == "1"
    assert "ACC_TEST_VAR" not in os.environ
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        port = s.getsockname()[1]
        assert ours.is_port_in_use(port)
    a, b = torch.ones(3), torch.ones(3)
    a, b = ours.release_memory(a, b)
    assert a is None and b is None
