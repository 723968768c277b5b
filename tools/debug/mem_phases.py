"""Allocated HBM after each phase of a training step, world-size-1 shortcut vs forced-sharded FSDP (diagnostic)."""
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin  # noqa: E402
from accelerate_hpc_test_amd.models.llama import LlamaConfig, LlamaForCausalLM  # noqa: E402
from accelerate_hpc_test_amd.state import AcceleratorState, GradientState  # noqa: E402
from accelerate_hpc_test_amd.utils import RcclKwargs  # noqa: E402

G = 2**30
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29561", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for force in (False, True):
    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    torch.cuda.empty_cache()
    cfg = LlamaConfig(num_hidden_layers=int(sys.argv[1]) if len(sys.argv) > 1 else 8)
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"])
    acc = Accelerator(mixed_precision="bf16", fsdp_plugin=plugin, kwargs_handlers=[RcclKwargs(fsdp_force_sharded=force)])
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5)
    model, opt = acc.prepare(model, opt)
    ids = torch.randint(0, cfg.vocab_size, (1, 4096)).cuda()
    rec = []
    for step in range(3):
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        a0 = torch.cuda.memory_allocated()
        out = model(ids, labels=ids, return_logits=False)
        torch.cuda.synchronize()
        a1, p1 = torch.cuda.memory_allocated(), torch.cuda.max_memory_allocated()
        acc.backward(out.loss)
        torch.cuda.synchronize()
        a2, p2 = torch.cuda.memory_allocated(), torch.cuda.max_memory_allocated()
        opt.step()
        torch.cuda.synchronize()
        a3, p3 = torch.cuda.memory_allocated(), torch.cuda.max_memory_allocated()
        opt.zero_grad()
        a4 = torch.cuda.memory_allocated()
        rec.append([round(x / G, 2) for x in (a0, a1, p1, a2, p2, a3, p3, a4)])
    print(f"force={force} [start, after fwd, fwd peak, after bwd, bwd peak, after step, step peak, after zero_grad] GiB:")
    for r in rec:
        print("   ", r)
    del model, opt, acc, out
