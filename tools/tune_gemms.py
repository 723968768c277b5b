"""Offline hipBLASLt solution search for the linear-layer GEMMs of a model step (see ops/gemm_tuning.py).

Each linear (out, in) at T tokens produces three GEMMs — forward x·Wᵀ (TunableOp "TN"), dgrad dy·W ("NN") and
wgrad dyᵀ·x ("NT"). We reproduce exactly those calls with one nn.Linear fwd+bwd per shape so the TunableOp keys
match the training step, print progress per shape and rewrite the table after each one (a long search never goes
silent, partial results survive a time-out).

    python tools/tune_gemms.py --model llama3-8b --tokens 8192 --out gpurun_out/tunableop_gfx950.csv \
        [--seed-table accelerate_hpc_test_amd/ops/tuned/tunableop_gfx950.csv]
"""

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def linear_shapes(model: str):
    from accelerate_hpc_test_amd.models import LLAMA_PRESETS, MIXTRAL_PRESETS

    if model in LLAMA_PRESETS:
        c = LLAMA_PRESETS[model]
        qkv = (c.num_attention_heads + 2 * c.num_key_value_heads) * c.head_dim
        return [(qkv, c.hidden_size), (c.hidden_size, c.num_attention_heads * c.head_dim),
                (2 * c.intermediate_size, c.hidden_size), (c.hidden_size, c.intermediate_size), (c.vocab_size, c.hidden_size)]
    c = MIXTRAL_PRESETS[model]
    qkv = (c.num_attention_heads + 2 * c.num_key_value_heads) * c.head_dim
    return [(qkv, c.hidden_size), (c.hidden_size, c.num_attention_heads * c.head_dim), (c.vocab_size, c.hidden_size)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--tokens", type=int, default=8192)
    p.add_argument("--out", default="gpurun_out/tunableop_gfx950.csv")
    p.add_argument("--seed-table", default=None)
    p.add_argument("--max-duration-ms", type=int, default=10)
    p.add_argument("--max-iterations", type=int, default=30)
    args = p.parse_args()
    import torch.cuda.tunable as tunable

    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(args.out, insert_device_ordinal=False)
    tunable.set_max_tuning_duration(args.max_duration_ms)
    tunable.set_max_tuning_iterations(args.max_iterations)
    if args.seed_table and os.path.isfile(args.seed_table):
        tunable.read_file(args.seed_table)
        print(f"seeded with {len(tunable.get_results())} results from {args.seed_table}", flush=True)
    dev = torch.device("cuda")
    for out_f, in_f in linear_shapes(args.model):
        t0 = time.time()
        lin = torch.nn.Linear(in_f, out_f, bias=False, device=dev, dtype=torch.bfloat16)
        x = torch.randn(args.tokens, in_f, device=dev, dtype=torch.bfloat16, requires_grad=True)
        y = lin(x)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        print(f"tuned linear out={out_f} in={in_f}: {time.time() - t0:.1f}s ({len(tunable.get_results())} results)", flush=True)
        del lin, x, y
        torch.cuda.empty_cache()
    # NOTE: TunableOp persists only the results found in THIS process (also at exit, from C++); fold the seed table
    # back in afterwards, from another process: `python tools/tune_gemms.py --merge OUT SEED`.
    print("done", flush=True)


def merge_tables(out_path, *others):
    lines = []
    for p in (out_path,) + others:
        if os.path.isfile(p):
            lines += open(p).read().splitlines()
    seen, out = set(), []
    for ln in lines:
        key = ",".join(ln.split(",")[:2])
        if ln.strip() and key not in seen:
            seen.add(key)
            out.append(ln)
    open(out_path, "w").write("\n".join(out) + "\n")
    print(f"merged -> {out_path}: {sum(1 for l in out if not l.startswith('Validator'))} GEMM entries")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--merge":
        merge_tables(*sys.argv[2:])
    else:
        main()
