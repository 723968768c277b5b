"""`accelerate-amd config update`: re-save an existing config so new fields get their defaults and legacy keys
are migrated (parity: reference commands/config/update.py)."""

from pathlib import Path

from .config_args import default_config_file, load_config_from_file

description = "Update an existing config file with the latest defaults while maintaining the old configuration."


def update_config(args):
    config_file = args.config_file
    if config_file is None and Path(default_config_file).exists():
        config_file = default_config_file
    elif not Path(config_file or "").exists():
        raise ValueError(f"The passed config file located at {config_file} doesn't exist.")
    config = load_config_from_file(config_file)
    config.save(config_file)
    return config_file


def update_command_parser(parser, parents):
    from ..utils import SubcommandHelpFormatter

    parser = parser.add_parser("update", parents=parents, help=description, formatter_class=SubcommandHelpFormatter)
    parser.add_argument("--config_file", default=None, help="The path to the config file to update.")
    parser.set_defaults(func=update_config_command)
    return parser


def update_config_command(args):
    config_file = update_config(args)
    print(f"Successfully updated the configuration file at {config_file}.")
