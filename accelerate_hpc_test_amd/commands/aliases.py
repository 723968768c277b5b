"""`accelerate-amd aliases install|remove|list`: opt-in drop-in command names.

The reference ships `accelerate`, `accelerate-launch`, `accelerate-config`, `accelerate-estimate-memory` and
`accelerate-merge-weights` (`/root/reference/setup.py:70-78`). This package installs them as `accelerate-amd*` so it
never shadows an installed upstream `accelerate`; a user switching over can opt in to the upstream names either at
install time (`ACCELERATE_AMD_INSTALL_ALIASES=1 pip install .`, see setup.py) or afterwards with this command, which
writes small launcher scripts into a directory of their choice (default: the directory of the running interpreter's
scripts) that run this package's CLI with the same interpreter.
"""

from __future__ import annotations

import os
import stat
import sys
import sysconfig
from argparse import ArgumentParser

# alias -> argv prefix handed to accelerate_hpc_test_amd.commands.accelerate_cli.main
ALIASES = {
    "accelerate": [],
    "accelerate-launch": ["launch"],
    "accelerate-config": ["config"],
    "accelerate-estimate-memory": ["estimate-memory"],
    "accelerate-merge-weights": ["merge-weights"],
}
_MARK = "# accelerate-amd alias"

description = "Install / remove / list the opt-in upstream-style command names (accelerate, accelerate-launch, ...)."


def _script(prefix: list) -> str:
    # the package's parent directory is a fallback import root (for in-tree / editable use without installation)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return (f"#!{sys.executable}\n{_MARK}\nimport sys\n"
            f"try:\n    from accelerate_hpc_test_amd.commands.accelerate_cli import main\n"
            f"except ModuleNotFoundError:\n    sys.path.insert(0, {root!r})\n"
            f"    from accelerate_hpc_test_amd.commands.accelerate_cli import main\n"
            f"rc = main({prefix!r} + sys.argv[1:])\n"
            f"sys.exit(rc if isinstance(rc, int) and not isinstance(rc, bool) else 0)\n")


def _default_dir() -> str:
    return sysconfig.get_path("scripts")


def install(directory: str, force: bool = False) -> list:
    os.makedirs(directory, exist_ok=True)
    if not force:  # check every target before writing any, so a refusal leaves no partial install behind
        foreign = [n for n, st in listed(directory).items() if st == "other"]
        if foreign:
            raise FileExistsError(f"{', '.join(os.path.join(directory, n) for n in foreign)} exist(s) and are not "
                                  "accelerate-amd aliases (use --force to replace)")
    written = []
    for name, prefix in ALIASES.items():
        path = os.path.join(directory, name)
        with open(path, "w") as f:
            f.write(_script(prefix))
        os.chmod(path, os.stat(path).st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
        written.append(path)
    return written


def remove(directory: str) -> list:
    gone = []
    for name in ALIASES:
        path = os.path.join(directory, name)
        if os.path.exists(path):
            with open(path, errors="replace") as f:
                if _MARK in f.read(4096):
                    os.remove(path)
                    gone.append(path)
    return gone


def listed(directory: str) -> dict:
    out = {}
    for name in ALIASES:
        path = os.path.join(directory, name)
        ours = False
        if os.path.exists(path):
            with open(path, errors="replace") as f:
                ours = _MARK in f.read(4096)
        out[name] = "installed" if ours else ("other" if os.path.exists(path) else "absent")
    return out


def aliases_command(args):
    d = args.dir or _default_dir()
    if args.action == "install":
        for p in install(d, force=args.force):
            print(f"wrote {p}")
    elif args.action == "remove":
        for p in remove(d):
            print(f"removed {p}")
    else:
        for name, st in listed(d).items():
            print(f"{name:28s} {st}")
    return 0


def aliases_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("aliases", description=description)
    else:
        parser = ArgumentParser("accelerate-amd aliases", description=description)
    parser.add_argument("action", choices=["install", "remove", "list"])
    parser.add_argument("--dir", default=None, help="Target directory (default: this interpreter's scripts directory).")
    parser.add_argument("--force", action="store_true", help="Replace existing files that are not our aliases.")
    if subparsers is not None:
        parser.set_defaults(func=aliases_command)
    return parser
