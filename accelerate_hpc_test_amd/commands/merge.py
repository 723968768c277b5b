"""`accelerate-amd merge-weights`: merge a SHARDED FSDP checkpoint into one file (parity: reference
commands/merge.py:26-69 → utils/fsdp_utils.merge_fsdp_weights)."""

import argparse

from ..utils.fsdp_utils import merge_fsdp_weights

description = "Merge the shards of a sharded FSDP checkpoint (saved by `save_state`/`save_model`) into one safetensors/bin file."


def merge_command(args):
    merge_fsdp_weights(args.checkpoint_directory, args.output_path, not args.unsafe_serialization, args.remove_checkpoint_dir)


def merge_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("merge-weights", description=description)
    else:
        parser = argparse.ArgumentParser(description=description)
    parser.add_argument("checkpoint_directory", type=str, help="Directory with the sharded weights saved by FSDP.")
    parser.add_argument("output_path", type=str, help="Directory the merged weights are written to.")
    parser.add_argument("--unsafe_serialization", action="store_true", default=False, help="Write a torch .bin instead of safetensors.")
    parser.add_argument("--remove_checkpoint_dir", action="store_true", default=False, help="Delete the sharded input afterwards.")
    if subparsers is not None:
        parser.set_defaults(func=merge_command)
    return parser


def main():
    parser = merge_command_parser()
    args = parser.parse_args()
    merge_command(args)


if __name__ == "__main__":
    main()
