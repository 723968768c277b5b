"""`accelerate-amd test`: run the bundled end-to-end sanity script through `launch` with the user's config
(parity: reference commands/test.py:22-65 → test_utils/scripts/test_script.py)."""

import argparse
import os
import sys

from ..utils.launch import run_child


def test_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("test")
    else:
        parser = argparse.ArgumentParser("accelerate-amd test command")
    parser.add_argument("--config_file", default=None, help="Config file to launch the sanity script with.")
    if subparsers is not None:
        parser.set_defaults(func=test_command)
    return parser


def test_command(args):
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "test_utils", "scripts", "test_script.py")
    cmd = [sys.executable, "-m", "accelerate_hpc_test_amd.commands.launch"]
    if args.config_file is not None:
        cmd += ["--config_file", args.config_file]
    cmd.append(script)
    rc = run_child(cmd, os.environ.copy())
    if rc == 0:
        print("Test is a success! You are ready for your distributed training!")
    else:
        print(f"Test failed (exit code {rc}).")
    return rc


def main():
    parser = test_command_parser()
    args = parser.parse_args()
    raise SystemExit(test_command(args))


if __name__ == "__main__":
    main()
