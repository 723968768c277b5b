"""Accelerator.free_memory (reference accelerator.py:3867-3912) + dropping the user's references must release the
wrapped model's engine and buffers. Hooks that the engines register on parameters live in C++ autograd metadata the
Python cycle collector cannot see through, so a strong engine reference there leaked every shard (33 GiB measured on
an 8-layer Llama-3-8B-width model on MI355X, tests/test_memory_gpu.py); they hold the engine weakly."""

import gc
import weakref

import torch

from accelerate_hpc_test_amd import debug_launcher


def test_fsdp_engine_is_collected_after_free_memory():
    from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState

    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(fsdp_plugin=plugin, cpu=True)
    with torch.device("meta"):
        model = LlamaForCausalLM(LLAMA_PRESETS["llama-tiny"])
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    model, opt = acc.prepare(model, opt)
    ids = torch.randint(0, 512, (1, 128))
    out = model(ids, labels=ids)
    acc.backward(out.loss)
    opt.step()
    opt.zero_grad()
    eng = weakref.ref(model.engine)
    master = weakref.ref(model.engine.units[1].master)
    acc.free_memory()
    del model, opt, out, acc
    gc.collect()
    assert eng() is None and master() is None


def _ddp_release():
    from accelerate_hpc_test_amd import Accelerator
    from accelerate_hpc_test_amd.test_utils.training import TinyMLP

    acc = Accelerator(cpu=True)
    model = TinyMLP()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = acc.prepare(model, opt)
    acc.backward(model(torch.randn(4, 4)).sum())
    opt.step()
    ref = weakref.ref(model)
    acc.free_memory()
    del model, opt, acc
    gc.collect()
    assert ref() is None, "DDP reducer still alive after free_memory"


def test_ddp_reducer_is_collected_after_free_memory():
    debug_launcher(_ddp_release, num_processes=2)


def _ddp_reprepare():
    """Advisor r3 (high): the fused weight-gradient install converts the user's nn.Linear modules in place; preparing the
    same model again (after free_memory, in a new Accelerator) must re-bind them to the new reducer, so that after
    `zero_grad(set_to_none=True)` every Linear weight still gets its (all-reduced) gradient."""
    import torch.distributed as dist

    from accelerate_hpc_test_amd import Accelerator
    from accelerate_hpc_test_amd.parallel.ddp import _DDPFusedLinear
    from accelerate_hpc_test_amd.state import AcceleratorState, GradientState

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    x = torch.randn(6, 8) * (dist.get_rank() + 1)

    def grads(m):
        return [p.grad.clone() if p.grad is not None else None for p in m.parameters()]

    acc = Accelerator(cpu=True)
    m1, opt = acc.prepare(model, torch.optim.SGD(model.parameters(), lr=0.0))
    assert any(type(m) is _DDPFusedLinear for m in model.modules())
    acc.backward(m1(x).square().sum())
    g1 = grads(model)
    opt.zero_grad(set_to_none=True)
    acc.free_memory()
    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    for keep_old_alive in (False, True):
        acc2 = Accelerator(cpu=True)
        m2, opt2 = acc2.prepare(model, torch.optim.SGD(model.parameters(), lr=0.0))
        opt2.zero_grad(set_to_none=True)
        acc2.backward(m2(x).square().sum())
        g2 = grads(model)
        for a, b in zip(g1, g2):
            assert b is not None and torch.count_nonzero(b) > 0
            torch.testing.assert_close(a, b)
        opt2.zero_grad(set_to_none=True)
        if not keep_old_alive:
            del m1  # first pass: the first reducer is gone; second pass: the previous one (m2) is still referenced
            gc.collect()
        m1 = m2
        acc2.free_memory()
        AcceleratorState._reset_state(True)
        GradientState._reset_state()


def test_ddp_reprepare_same_model_keeps_weight_grads():
    debug_launcher(_ddp_reprepare, num_processes=2)
