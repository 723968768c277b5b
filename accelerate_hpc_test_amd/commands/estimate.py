"""`accelerate-amd estimate-memory`: how much memory a model needs to load / train.

Parity target: `/root/reference/src/accelerate/commands/estimate.py:187-318` (same table: dtype, largest layer,
total size, training with Adam). There is no network on an MI355X training node, so the model is resolved from
(a) a built-in preset of `models/` (`llama3-8b`, `llama3-70b`, ...), (b) a local directory with a `config.json`,
or (c) a name already in the local Hugging Face cache — always instantiated on the meta device.

MI355X addition: `--num_gpus N` adds the per-GPU footprint of this framework's FSDP2 layout (fp32 master shard
+ fp32 grad shard + bf16 all-gather shard + 2 fp32 Adam moments, all 1/N) plus the largest unsharded bf16 unit,
which is what decides whether a model fits in 288 GB of HBM3E per GPU.
"""

from __future__ import annotations

import argparse
import os
from typing import Optional

import torch

from ..big_modeling import init_empty_weights
from ..utils.other import convert_bytes
from ..utils.device_map import calculate_maximum_sizes

MI355X_HBM_BYTES = 288 * 10**9


def create_empty_model(model_name: str, library_name: Optional[str] = None, trust_remote_code: bool = False):
    """Instantiate `model_name` with no storage (meta device)."""
    from ..models.llama import LLAMA_PRESETS, LlamaForCausalLM

    if model_name in LLAMA_PRESETS:
        with init_empty_weights():
            return LlamaForCausalLM(LLAMA_PRESETS[model_name])
    try:
        from ..models import MODEL_PRESETS  # other families register here
    except ImportError:
        MODEL_PRESETS = {}
    if model_name in MODEL_PRESETS:
        builder = MODEL_PRESETS[model_name]
        with init_empty_weights():
            return builder()
    if library_name not in (None, "transformers"):
        raise ValueError(f"Only `transformers` models (or built-in presets) can be estimated offline, got `{library_name}`.")
    try:
        import transformers
    except ImportError as e:
        raise RuntimeError(f"`{model_name}` is not a built-in preset and `transformers` is not importable.") from e
    os.environ.setdefault("HF_HUB_OFFLINE", "1")
    try:
        config = transformers.AutoConfig.from_pretrained(model_name, trust_remote_code=trust_remote_code)
    except OSError as e:
        raise RuntimeError(
            f"Could not resolve `{model_name}` offline: pass a built-in preset name, a local directory containing "
            "config.json, or a model already present in the local Hugging Face cache."
        ) from e
    with init_empty_weights():
        cls = transformers.AutoModelForCausalLM if getattr(config, "architectures", None) else transformers.AutoModel
        try:
            return cls.from_config(config, trust_remote_code=trust_remote_code)
        except ValueError:
            return transformers.AutoModel.from_config(config, trust_remote_code=trust_remote_code)


def estimate_training_usage(bytes: int, mixed_precision: str, msamp_config: Optional[str] = None) -> dict:
    """Training memory (batch 1, activations excluded) for a model of `bytes` fp32 bytes with Adam."""
    fp32 = bytes
    half = bytes // 2
    sizes = {"model": -1, "optimizer": -1, "gradients": -1, "step": -1}
    if mixed_precision == "float32":
        sizes.update(model=fp32, gradients=fp32, optimizer=2 * fp32, step=4 * fp32)
    elif mixed_precision in ("float16", "bfloat16") or (mixed_precision == "fp8" and msamp_config is None):
        sizes.update(model=fp32, gradients=fp32 + half, optimizer=2 * fp32, step=2 * fp32)
    return sizes


def fsdp_per_gpu_bytes(num_params: int, largest_layer_params: int, num_gpus: int) -> int:
    """Per-GPU steady-state bytes of this framework's FSDP2 engine (activations excluded)."""
    sharded = num_params * (4 + 4 + 2 + 8) / num_gpus  # master, grad, bf16 shard, exp_avg + exp_avg_sq
    unsharded = 2 * largest_layer_params * 2  # current + prefetched bf16 unit
    return int(sharded + unsharded)


def gather_data(args):
    model = create_empty_model(args.model_name, library_name=args.library_name, trust_remote_code=args.trust_remote_code)
    total_size, largest_layer = calculate_maximum_sizes(model)
    num_params = sum(p.numel() for p in model.parameters())
    bytes_per_param = total_size / max(num_params, 1)
    rows = []
    divisor = {"float32": 1, "float16": 2, "bfloat16": 2, "int8": 4, "int4": 8}
    for dtype in args.dtypes:
        training = estimate_training_usage(total_size, dtype)
        d = divisor.get(dtype, 1)
        row = [dtype, largest_layer[0] / d, total_size / d, training]
        rows.append(row)
    fsdp = None
    if getattr(args, "num_gpus", None):
        largest_params = int(largest_layer[0] / bytes_per_param)
        fsdp = fsdp_per_gpu_bytes(num_params, largest_params, args.num_gpus)
    return rows, fsdp


def create_ascii_table(headers: list, rows: list, title: str) -> str:
    cols = list(zip(*([headers] + rows)))
    widths = [max(len(str(c)) for c in col) + 2 for col in cols]
    total = sum(widths) + len(widths) - 1
    bar = lambda l, m, r: l + m.join("─" * w for w in widths) + r  # noqa: E731
    fmt = lambda cells: "│" + "│".join(str(c).center(w) for c, w in zip(cells, widths)) + "│"  # noqa: E731
    out = ["┌" + "─" * total + "┐", "│" + title.center(total) + "│", bar("├", "┬", "┤"), fmt(headers), bar("├", "┼", "┤")]
    out += [fmt(r) for r in rows]
    out.append(bar("└", "┴", "┘"))
    return "\n".join(out)


def estimate_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("estimate-memory")
    else:
        parser = argparse.ArgumentParser(description="Model size estimator for fitting a model onto MI355X memory.")
    parser.add_argument("model_name", type=str, help="Built-in preset, local model directory, or cached hub name.")
    parser.add_argument("--library_name", type=str, choices=["timm", "transformers"], help="Model library (offline).")
    parser.add_argument(
        "--dtypes", type=str, nargs="+", default=["float32", "float16", "int8", "int4"],
        choices=["float32", "float16", "bfloat16", "int8", "int4"], help="dtypes to report.",
    )
    parser.add_argument("--trust_remote_code", action="store_true", default=False)
    parser.add_argument("--num_gpus", type=int, default=None, help="Also report the per-GPU FSDP2 footprint on N MI355X.")
    if subparsers is not None:
        parser.set_defaults(func=estimate_command)
    return parser


def estimate_command(args):
    rows, fsdp = gather_data(args)
    printable = []
    for dtype, largest, total, training in rows:
        peak = max(training.values())
        printable.append([dtype, convert_bytes(largest), convert_bytes(total), convert_bytes(peak) if peak != -1 else "N/A"])
    table = create_ascii_table(["dtype", "Largest Layer", "Total Size", "Training using Adam"], printable, f"Memory Usage for loading `{args.model_name}`")
    print(table)
    if fsdp is not None:
        fits = "fits" if fsdp < MI355X_HBM_BYTES * 0.9 else "does NOT fit"
        print(f"FSDP2 bf16 on {args.num_gpus}x MI355X: {convert_bytes(fsdp)} per GPU before activations ({fits} in 288 GB HBM3E)")
    return rows


def main():
    parser = estimate_command_parser()
    args = parser.parse_args()
    estimate_command(args)


if __name__ == "__main__":
    main()
