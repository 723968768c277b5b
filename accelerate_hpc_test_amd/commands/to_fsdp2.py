"""`accelerate-amd to-fsdp2`: rewrite an FSDP1 config file into FSDP2 form.

Parity target: `/root/reference/src/accelerate/commands/to_fsdp2.py:71-172`: the same key renames / removals and
the sharding-strategy → `fsdp_reshard_after_forward` value mapping. Rules live in one table below.
"""

import argparse
import logging
from pathlib import Path

import yaml

logger = logging.getLogger(__name__)

description = "Convert an FSDP1 `accelerate` config file to FSDP2."

_KEEP = "keep"
_DROP = "drop"
_LATER = "not-yet"

# FSDP1 key → (action, FSDP2 key)
_RULES = {
    "fsdp_version": (_KEEP, "fsdp_version"),
    "fsdp_reshard_after_forward": (_KEEP, "fsdp_reshard_after_forward"),
    "fsdp_auto_wrap_policy": (_KEEP, "fsdp_auto_wrap_policy"),
    "fsdp_backward_prefetch": (_DROP, None),
    "fsdp_forward_prefetch": (_LATER, None),
    "fsdp_cpu_ram_efficient_loading": (_KEEP, "fsdp_cpu_ram_efficient_loading"),
    "fsdp_offload_params": (_KEEP, "fsdp_offload_params"),
    "fsdp_sharding_strategy": (_KEEP, "fsdp_reshard_after_forward"),
    "fsdp_state_dict_type": (_KEEP, "fsdp_state_dict_type"),
    "fsdp_sync_module_states": (_DROP, None),
    "fsdp_transformer_layer_cls_to_wrap": (_KEEP, "fsdp_transformer_layer_cls_to_wrap"),
    "fsdp_min_num_params": (_KEEP, "fsdp_min_num_params"),
    "fsdp_use_orig_params": (_DROP, None),
    "fsdp_activation_checkpointing": (_KEEP, "fsdp_activation_checkpointing"),
}

_RESHARD = {"FULL_SHARD": True, "SHARD_GRAD_OP": False, "HYBRID_SHARD": True, "HYBRID_SHARD_ZERO2": False, "NO_SHARD": False}
_VALUE_MAPS = {"fsdp_sharding_strategy": _RESHARD, "fsdp_reshard_after_forward": _RESHARD}


def convert_config_to_fsdp2(config: dict) -> dict:
    section = config.get("fsdp_config") or {}
    if not section:
        logger.info("No FSDP config found in the config file, skipping conversion...")
        return config
    if section.get("fsdp_version", 1) == 2:
        logger.warning("Config already specifies FSDP2, skipping conversion (set `fsdp_version: 1` to force it).")
        return config
    converted = {}
    for key, value in section.items():
        action, new_key = _RULES.get(key, (_KEEP, key))
        if action == _DROP:
            logger.warning(f"Argument {key} has been removed in FSDP2, skipping this key...")
            continue
        if action == _LATER:
            logger.warning(f"Argument {key} is not yet implemented in FSDP2, skipping this key...")
            continue
        converted[new_key] = _VALUE_MAPS.get(key, {}).get(value, value) if isinstance(value, str) else value
    converted["fsdp_version"] = 2
    config["fsdp_config"] = converted
    return config


def load_config(config_file: str) -> dict:
    config = yaml.safe_load(Path(config_file).read_text())
    if not config:
        raise ValueError("Config file is empty")
    return config


def _validate_to_fsdp2_args(args):
    if not Path(args.config_file).exists():
        raise FileNotFoundError(f"Config file {args.config_file} not found")
    if not args.overwrite and args.output_file is None:
        raise ValueError("If --overwrite is not set, --output_file must be provided")
    if not args.overwrite and Path(args.output_file).exists():
        raise FileExistsError(f"Output file {args.output_file} already exists and --overwrite is not set")


def to_fsdp2_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("to-fsdp2", description=description)
    else:
        parser = argparse.ArgumentParser(description=description)
    parser.add_argument("--config_file", type=str, required=True, help="The config file to convert to FSDP2.")
    parser.add_argument("--overwrite", action="store_true", default=False, help="Overwrite the input file.")
    parser.add_argument("--output_file", type=str, default=None, help="Where to write the converted config.")
    if subparsers is not None:
        parser.set_defaults(func=to_fsdp2_command)
    return parser


def to_fsdp2_command(args):
    _validate_to_fsdp2_args(args)
    config = load_config(args.config_file)
    out = args.output_file or args.config_file
    Path(out).write_text(yaml.safe_dump(convert_config_to_fsdp2(config)))


def main():
    parser = to_fsdp2_command_parser()
    to_fsdp2_command(parser.parse_args())


if __name__ == "__main__":
    main()
