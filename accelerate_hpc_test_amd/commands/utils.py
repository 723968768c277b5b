"""Small argparse helpers shared by the CLI sub-commands (parity: reference commands/utils.py)."""

import argparse


class SubcommandHelpFormatter(argparse.RawDescriptionHelpFormatter):
    """Drops the redundant `{a,b,c}` choice list that argparse prints for sub-parsers."""

    def _format_usage(self, usage, actions, groups, prefix):
        text = super()._format_usage(usage, actions, groups, prefix)
        return text.replace("<command> [<args>] ", "")


def add_bool(group, flag: str, help: str, default=None):
    """`--flag` / `--flag true|false` style boolean option (accepts both, like the reference's config flags)."""
    from ..utils.environment import str_to_bool

    def conv(v):
        return bool(str_to_bool(v))

    group.add_argument(flag, nargs="?", const=True, default=default, type=conv, help=help)
