"""`accelerate-amd config`: run the questionnaire and save the answers (parity: reference commands/config/config.py)."""

import argparse
import os

from .cluster import get_cluster_input
from .config_args import default_config_file, default_yaml_config_file

description = (
    "Launches a series of prompts to create and save a `default_config.yaml` configuration file for your training "
    "system. Should always be ran first on your machine."
)


def get_user_input(answers=None):
    return get_cluster_input(answers)


def config_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("config", description=description)
    else:
        parser = argparse.ArgumentParser("accelerate-amd config command", description=description)
    parser.add_argument(
        "--config_file",
        default=None,
        help=f"The path to use to store the config file. Will default to {default_config_file}.",
    )
    if subparsers is not None:
        parser.set_defaults(func=config_command)
    return parser


def config_command(args, answers=None):
    config = get_user_input(answers)
    config_file = args.config_file if args.config_file is not None else default_yaml_config_file
    os.makedirs(os.path.dirname(os.path.abspath(config_file)), exist_ok=True)
    config.save(config_file)
    print(f"accelerate configuration saved at {config_file}")
    return config_file


def main():
    parser = config_command_parser()
    args = parser.parse_args()
    config_command(args)


if __name__ == "__main__":
    main()
