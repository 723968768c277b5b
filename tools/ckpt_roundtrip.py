"""Sharded checkpoint round trip of Llama-3-8B on the FSDP engine's multi-rank code path at one rank (forced sharded,
one-rank RCCL group): a few AdamW steps (timed), `save_state` (SHARDED_STATE_DICT: model shard as safetensors + JSON,
optimizer shard as safetensors + JSON) through the non-blocking writer (utils/async_checkpoint.py: device snapshot,
native D2H file writer), training steps while the files are written (timed against the steps before), the wait for
the writer, perturb, `load_state`, compare with the state at save time. Prints wall times, checkpoint bytes, the
process's peak host RSS and the RSS growth across save and load, as one JSON line.

    python tools/ckpt_roundtrip.py [--model llama3-8b] [--dir /tmp/ckpt8b] [--seq 2048]"""
import argparse
import json
import os
import resource
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rss_gib():
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 2**20
    return 0.0


def dir_bytes(d):
    return sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(d) for f in fs)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--dir", default=None)
    p.add_argument("--seq", type=int, default=2048)
    args = p.parse_args()
    from accelerate_hpc_test_amd import Accelerator, FullyShardedDataParallelPlugin
    from accelerate_hpc_test_amd.models.llama import LLAMA_PRESETS, LlamaForCausalLM
    from accelerate_hpc_test_amd.utils import RcclKwargs, fsdp_utils

    ckpt = args.dir
    if ckpt is None:  # the filesystem with the most room: the checkpoint is ~64 GB for 8B (fp32 master + bf16 moments)
        cands = [d for d in ("/tmp", os.getcwd(), "/dev/shm") if os.path.isdir(d)]
        best = max(cands, key=lambda d: shutil.disk_usage(d).free)
        ckpt = os.path.join(best, "acc_ckpt_roundtrip")
    free = shutil.disk_usage(os.path.dirname(ckpt)).free
    print(json.dumps({"ckpt_dir": ckpt, "free_gib": round(free / 2**30, 1)}), flush=True)
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl", init_method="tcp://127.0.0.1:29547", rank=0, world_size=1,
                                         device_id=torch.device("cuda", 0))
    plugin = FullyShardedDataParallelPlugin(fsdp_version=2, auto_wrap_policy="transformer_based_wrap",
                                            transformer_cls_names_to_wrap=["LlamaDecoderLayer"],
                                            state_dict_type="SHARDED_STATE_DICT")
    acc = Accelerator(mixed_precision="bf16", fsdp_plugin=plugin, kwargs_handlers=[RcclKwargs(fsdp_force_sharded=True)])
    cfg = LLAMA_PRESETS[args.model]
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-5)
    model, opt = acc.prepare(model, opt)
    assert model.engine.sharded
    ids = torch.randint(0, cfg.vocab_size, (1, args.seq), device=acc.device)

    def step():
        t0 = time.time()
        acc.backward(model(ids, labels=ids).loss)
        opt.step()
        opt.zero_grad()
        torch.cuda.synchronize()
        return time.time() - t0

    normal = [step() for _ in range(4)][1:]
    def snapshot():
        eng = model.engine
        m = torch.stack([u.master.double().sum() for u in eng.units]).cpu()
        st = opt.optimizer.state if hasattr(opt, "optimizer") else opt.state
        s = torch.stack([t.double().sum() for v in st.values() for t in v.values() if torch.is_tensor(t) and t.dim() > 0]).cpu()
        return m, s

    before = snapshot()
    rss0 = rss_gib()
    shutil.rmtree(ckpt, ignore_errors=True)
    from accelerate_hpc_test_amd.utils.async_checkpoint import wait_pending_saves, writer

    t = time.time()
    acc.save_state(ckpt)
    torch.cuda.synchronize()
    t_save = time.time() - t  # what the training loop is blocked for
    during = [step() for _ in range(3)]  # the writer streams the snapshot to disk meanwhile
    t = time.time()
    wait_pending_saves()
    t_wait = time.time() - t
    t_total = t_save + sum(during) + t_wait
    nbytes = dir_bytes(ckpt)
    rss_after_save = rss_gib()
    with torch.no_grad():
        for u in model.engine.units:
            u.master.add_(1.0)
    fsdp_utils.IO_STATS["bytes_read"] = 0
    rss_before_load = rss_gib()
    t = time.time()
    acc.load_state(ckpt)
    torch.cuda.synchronize()
    t_load = time.time() - t
    after = snapshot()
    ok = bool(torch.equal(before[0], after[0]) and torch.equal(before[1], after[1]))
    res = {"model": args.model, "world": 1, "path": "fsdp-forced-sharded", "ckpt_gib": round(nbytes / 2**30, 2),
           "save_blocking_s": round(t_save, 3), "async_snapshot_gib": round(writer().last_snapshot_bytes / 2**30, 2),
           "step_s_before_save": [round(x, 3) for x in normal], "step_s_while_writing": [round(x, 3) for x in during],
           "wait_after_steps_s": round(t_wait, 2), "save_to_disk_s": round(t_total, 1), "load_s": round(t_load, 1),
           "save_gbps_end_to_end": round(nbytes / t_total / 1e9, 2), "load_gbps": round(nbytes / t_load / 1e9, 2),
           "tensor_bytes_read_gib": round(fsdp_utils.IO_STATS["bytes_read"] / 2**30, 2),
           "rss_gib": {"before_save": round(rss0, 1), "after_save": round(rss_after_save, 1),
                       "before_load": round(rss_before_load, 1), "after_load": round(rss_gib(), 1),
                       "peak": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 1)},
           "roundtrip_exact": ok}
    print(json.dumps(res), flush=True)
    shutil.rmtree(ckpt, ignore_errors=True)
    acc.end_training()
    assert ok, "state differs after the round trip"


if __name__ == "__main__":
    main()
