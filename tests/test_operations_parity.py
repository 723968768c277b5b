"""Operations whose exact output is API (sizes of padded batches) against the upstream `accelerate` installed in the
image; skipped when it is absent."""

import pytest
import torch

from accelerate_hpc_test_amd.utils import operations as ours

up = pytest.importorskip("accelerate.utils.operations")


@pytest.mark.parametrize("num_processes", range(1, 9))
def test_pad_input_tensors_matches_upstream(num_processes):
    for batch in range(1, 40):
        t = torch.arange(batch * 3, dtype=torch.float32).view(batch, 3)
        nested = {"x": t, "y": [t[:, :1].long()]}
        a = up.pad_input_tensors(nested, batch, num_processes)
        b = ours.pad_input_tensors(nested, batch, num_processes)
        assert torch.equal(a["x"], b["x"]) and torch.equal(a["y"][0], b["y"][0]), (batch, num_processes)


def test_pad_across_processes_single_process_is_identity():
    from accelerate_hpc_test_amd.state import PartialState

    PartialState(cpu=True)
    t = torch.randn(3, 5)
    assert ours.pad_across_processes(t, dim=1) is t
    assert ours.pad_across_processes(t, dim=7) is t  # out-of-range dim: unchanged
