"""`accelerate-amd config default` / `write_basic_config`: non-interactive config for the local machine.

Parity: `/root/reference/src/accelerate/commands/config/default.py:36-163`. Detects the MI355X GPUs of the node
(one process per GPU, MULTI_GPU over RCCL) and falls back to a CPU config.
"""

from pathlib import Path

import torch

from .config_args import ClusterConfig, default_json_config_file

description = "Create a default config file for Accelerate with only a few flags set."


def write_basic_config(mixed_precision="no", save_location: str = default_json_config_file):
    """Write a basic config (all local GPUs, one process each) to `save_location`; returns the path or False if a
    config already exists there."""
    path = Path(save_location)
    path.parent.mkdir(parents=True, exist_ok=True)
    if path.exists():
        print(f"Configuration already exists at {save_location}, will not override. Run `accelerate-amd config` manually or pass a different `save_location`.")
        return False
    mixed_precision = mixed_precision.lower()
    if mixed_precision not in ["no", "fp16", "bf16", "fp8"]:
        raise ValueError(f"`mixed_precision` should be one of 'no', 'fp16', 'bf16', or 'fp8'. Received {mixed_precision}")
    config = {
        "compute_environment": "LOCAL_MACHINE",
        "mixed_precision": mixed_precision,
    }
    num_gpus = torch.cuda.device_count()
    config["num_processes"] = num_gpus if num_gpus > 0 else 1
    config["use_cpu"] = num_gpus == 0
    if num_gpus > 1:
        config["distributed_type"] = "MULTI_GPU"
    else:
        config["distributed_type"] = "NO"
    config["debug"] = False
    config["enable_cpu_affinity"] = False
    config = ClusterConfig(**config)
    config.to_json_file(path)
    return path


def default_command_parser(parser, parents):
    from ..utils import SubcommandHelpFormatter

    parser = parser.add_parser("default", parents=parents, help=description, formatter_class=SubcommandHelpFormatter)
    parser.add_argument(
        "--config_file",
        default=default_json_config_file,
        help="The path to use to store the config file.",
        dest="save_location",
    )
    parser.add_argument(
        "--mixed_precision",
        choices=["no", "fp16", "bf16", "fp8"],
        type=str,
        help="Whether or not to use mixed precision training.",
        default="no",
    )
    parser.set_defaults(func=default_config_command)
    return parser


def default_config_command(args):
    config_file = write_basic_config(args.mixed_precision, args.save_location)
    if config_file:
        print(f"accelerate configuration saved at {config_file}")
