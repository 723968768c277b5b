"""`accelerate-amd` root CLI (parity: reference commands/accelerate_cli.py): config, env, estimate-memory,
launch, merge-weights, test, to-fsdp2, aliases (opt-in upstream-style command names)."""

from argparse import ArgumentParser

from .aliases import aliases_command_parser
from .config import get_config_parser
from .env import env_command_parser
from .estimate import estimate_command_parser
from .launch import launch_command_parser
from .merge import merge_command_parser
from .test import test_command_parser
from .to_fsdp2 import to_fsdp2_command_parser


def build_parser() -> ArgumentParser:
    parser = ArgumentParser("accelerate-amd CLI tool", usage="accelerate-amd <command> [<args>]", allow_abbrev=False)
    subparsers = parser.add_subparsers(help="accelerate-amd command helpers")
    get_config_parser(subparsers=subparsers)
    estimate_command_parser(subparsers=subparsers)
    env_command_parser(subparsers=subparsers)
    launch_command_parser(subparsers=subparsers)
    merge_command_parser(subparsers=subparsers)
    test_command_parser(subparsers=subparsers)
    to_fsdp2_command_parser(subparsers=subparsers)
    aliases_command_parser(subparsers=subparsers)
    return parser


def main(argv=None):
    parser = build_parser()
    args = parser.parse_args(argv)
    if not hasattr(args, "func"):
        parser.print_help()
        raise SystemExit(1)
    rc = args.func(args)
    if isinstance(rc, int) and not isinstance(rc, bool) and rc != 0:
        raise SystemExit(rc)
    return rc


if __name__ == "__main__":
    main()
