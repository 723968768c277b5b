"""BASELINE config #4 in the reference's own terms: big-model load time and per-token generation time
(reference `benchmarks/big_model_inference/big_model_inference.py`, numbers P8a-P8g in BASELINE.md).

The reference loads a Hub checkpoint with `from_pretrained(device_map="auto")` and times `model.generate` on six short
prompts. Offline here, so the same steps run on a synthetic checkpoint of the same architecture:

1. the transformers model class is built from its config on the meta device (no weights);
2. random weights (N(0, 0.02), norms = 1) are written once as a sharded safetensors checkpoint (`--ckpt-dir`, reused
   when present) — 5 GB shards with the standard `model.safetensors.index.json`;
3. **load** = `load_checkpoint_and_dispatch(meta_model, ckpt, device_map="auto", max_memory=..., dtype=...)` of this
   framework (device-map planner, streaming safetensors reader, pinned H2D engine, host / disk offload hooks), timed
   to the last byte on the GPU. The checkpoint was just written, so its shards are in the page cache (the reference's
   timings read from its Hub cache the same way; dropping the cache needs root);
4. **generate** = `model.generate` (greedy) on six prompts of the reference's token lengths (random ids, no tokenizer
   offline), `--new-tokens` each; per-token time = wall time / new tokens, reported with and without the first prompt
   as the reference does.

    python tools/bench_generate.py --model gpt-neox-20b                       # all on one GPU
    python tools/bench_generate.py --model opt-30b --gpu-mem 40GiB            # forced host offload
    python tools/bench_generate.py --model gpt-neox-20b --gpu-mem 20GiB --cpu-mem 10GiB --disk-offload
    python tools/bench_generate.py --model tiny --cpu                         # CPU plumbing check (tests)
Prints one JSON line.
"""

import argparse
import json
import os
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PROMPT_LENGTHS = [5, 9, 9, 8, 5, 9]  # token counts of the reference's six PROMPTS under the GPT-J tokenizer


def make_config(name: str):
    import transformers as tf

    if name == "gpt-j-6b":
        return tf.GPTJConfig(n_embd=4096, n_layer=28, n_head=16, rotary_dim=64, vocab_size=50400, n_positions=2048)
    if name == "gpt-neox-20b":
        return tf.GPTNeoXConfig(vocab_size=50432, hidden_size=6144, num_hidden_layers=44, num_attention_heads=64,
                                intermediate_size=24576, rotary_pct=0.25, max_position_embeddings=2048)
    if name == "opt-30b":
        return tf.OPTConfig(vocab_size=50272, hidden_size=7168, num_hidden_layers=48, ffn_dim=28672,
                            num_attention_heads=56, word_embed_proj_dim=7168, max_position_embeddings=2048)
    if name == "llama3-70b":
        return tf.LlamaConfig(vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                              num_attention_heads=64, num_key_value_heads=8, rope_theta=500000.0,
                              max_position_embeddings=8192)
    if name == "tiny":
        return tf.GPTNeoXConfig(vocab_size=512, hidden_size=64, num_hidden_layers=4, num_attention_heads=4,
                                intermediate_size=128, max_position_embeddings=256)
    raise ValueError(f"unknown model {name}")


def build_meta(config, dtype):
    import transformers as tf

    from accelerate_hpc_test_amd import init_empty_weights

    with init_empty_weights():
        model = tf.AutoModelForCausalLM.from_config(config, torch_dtype=dtype)
    model.eval()
    return model


def write_checkpoint(model, path: str, dtype, device: str, shard_bytes: int = 5 << 30):
    """Random-init sharded safetensors checkpoint of `model`'s state dict (tied names written once per name)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    shard, size, n, weight_map, total = {}, 0, 0, {}, 0

    def flush():
        nonlocal shard, size, n
        if shard:
            fname = f"model-{n:05d}.safetensors"
            save_file(shard, os.path.join(path, fname), metadata={"format": "pt"})
            for k in shard:
                weight_map[k] = fname
            n += 1
            shard, size = {}, 0

    g = torch.Generator(device=device).manual_seed(0)
    for name, t in model.state_dict().items():
        x = torch.empty(t.shape, dtype=dtype if t.is_floating_point() else t.dtype, device=device)
        if not t.is_floating_point():
            x.zero_()
        elif name.endswith(("norm.weight", "layernorm.weight", "ln_f.weight", "ln_1.weight", "layer_norm.weight")):
            x.fill_(1.0)
        elif name.endswith("bias"):
            x.zero_()
        else:
            x.normal_(0.0, 0.02, generator=g)
        shard[name] = x.cpu()
        size += x.numel() * x.element_size()
        total += x.numel() * x.element_size()
        if size >= shard_bytes:
            flush()
    flush()
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, f)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gpt-j-6b")
    p.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    p.add_argument("--gpu-mem", default=None, help="per-GPU budget for the device map (forces host offload)")
    p.add_argument("--cpu-mem", default="200GiB")
    p.add_argument("--disk-offload", action="store_true", help="blocks beyond --cpu-mem go to an offload folder")
    p.add_argument("--ckpt-dir", default=None)
    p.add_argument("--new-tokens", type=int, default=16)
    p.add_argument("--keep-ckpt", action="store_true")
    p.add_argument("--cpu", action="store_true")
    args = p.parse_args()
    dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    dev = "cpu" if args.cpu else "cuda"
    sync = (lambda: None) if args.cpu else torch.cuda.synchronize

    from accelerate_hpc_test_amd import load_checkpoint_and_dispatch
    from accelerate_hpc_test_amd.utils import compute_module_sizes

    config = make_config(args.model)
    ckpt = args.ckpt_dir or os.path.join(os.environ.get("TMPDIR", "/tmp"), f"acc_ckpt_{args.model}_{args.dtype}")
    t0 = time.time()
    if not os.path.isfile(os.path.join(ckpt, "model.safetensors.index.json")):
        write_checkpoint(build_meta(config, dtype), ckpt, dtype, device=dev)
    t_write = time.time() - t0

    model = build_meta(config, dtype)
    n_gpu = 0 if args.cpu else torch.cuda.device_count()
    max_memory = {i: (args.gpu_mem or "270GiB") for i in range(n_gpu)}
    max_memory["cpu"] = args.cpu_mem
    if args.cpu:
        max_memory = {"cpu": args.cpu_mem}
    offload_folder = os.path.join(os.environ.get("TMPDIR", "/tmp"), "acc_offload") if args.disk_offload else None
    if offload_folder:
        shutil.rmtree(offload_folder, ignore_errors=True)
    sync()
    t0 = time.perf_counter()
    model = load_checkpoint_and_dispatch(model, ckpt, device_map="auto", max_memory=max_memory, dtype=dtype,
                                         no_split_module_classes=model._no_split_modules, offload_folder=offload_folder)
    sync()
    t_load = time.perf_counter() - t0

    sizes = compute_module_sizes(model, dtype=dtype)
    per_device = {}
    for module, d in model.hf_device_map.items():
        per_device[str(d)] = per_device.get(str(d), 0) + sizes[module]

    main = "cpu" if args.cpu else "cuda:0"
    g = torch.Generator().manual_seed(1)
    times, toks, checksum = [], [], 0
    with torch.no_grad():
        for n in PROMPT_LENGTHS:
            ids = torch.randint(100, config.vocab_size - 100, (1, n), generator=g).to(main)
            sync()
            t0 = time.perf_counter()
            out = model.generate(ids, attention_mask=torch.ones_like(ids), max_new_tokens=args.new_tokens,
                                 min_new_tokens=args.new_tokens, do_sample=False, pad_token_id=0)
            sync()
            times.append(time.perf_counter() - t0)
            toks.append(out.shape[1] - n)
            checksum = (checksum * 1000003 + int(out[0, n:].long().sum().item())) % (1 << 61)
    per_tok = [t / k for t, k in zip(times, toks)]
    total_bytes = sum(per_device.values())
    host_bytes = sum(v for k, v in per_device.items() if k in ("cpu", "disk"))
    gen_s = sum(times[1:])
    rec = {
        "metric": "big-model load s / generation s per token (reference benchmarks/big_model_inference)",
        "model": args.model,
        "dtype": args.dtype,
        "load_s": round(t_load, 2),
        "s_per_token": round(sum(per_tok) / len(per_tok), 4),
        "s_per_token_first": round(per_tok[0], 4),
        "s_per_token_excl_first": round(sum(per_tok[1:]) / (len(per_tok) - 1), 4),
        "new_tokens": args.new_tokens,
        "generated_checksum": checksum,  # greedy decoding: equal across placements of the same checkpoint
        "params_b": round(sum(v for k, v in sizes.items() if k == "") / (torch.finfo(dtype).bits // 8) / 1e9, 2),
        "placement_gib": {k: round(v / 2**30, 1) for k, v in per_device.items()},
        # load: checkpoint bytes / load time (page-cache safetensors -> pinned staging -> HBM, or -> host offload store)
        "load_gbs": round(total_bytes / t_load / 1e9, 1),
        # generation with offload: the offloaded blocks stream back once per forward (one forward per new token)
        "offload_stream_gbs": round(host_bytes * sum(toks[1:]) / gen_s / 1e9, 1) if host_bytes and gen_s > 0 else None,
        "n_gpus": n_gpu,
        "checkpoint_write_s": round(t_write, 1),
        "data": "synthetic checkpoint (random-init weights, reference architecture), random prompt ids of the "
                "reference prompts' lengths; checkpoint in page cache",
    }
    print(json.dumps(rec), flush=True)
    if not args.keep_ckpt and args.ckpt_dir is None:
        shutil.rmtree(ckpt, ignore_errors=True)
    if offload_folder:
        shutil.rmtree(offload_folder, ignore_errors=True)


if __name__ == "__main__":
    main()
