"""`accelerate-amd env`: print the environment facts useful in bug reports (parity: reference commands/env.py:32-123).

Reports the ROCm/HIP/RCCL stack, the MI355X devices (gfx arch, HBM), the xGMI topology summary and the default
config file content.
"""

import argparse
import os
import platform
import subprocess

import numpy as np
import psutil
import torch

from .. import __version__ as version
from ..utils.environment import env_summary, get_xgmi_topology
from .config.config_args import default_config_file, load_config_from_file


def env_command_parser(subparsers=None):
    if subparsers is not None:
        parser = subparsers.add_parser("env")
    else:
        parser = argparse.ArgumentParser("accelerate-amd env command")
    parser.add_argument("--config_file", default=None, help="The config file to use for the default values in the launching script.")
    parser.add_argument("--topology", action="store_true", help="Also print the xGMI link matrix (rocm-smi --showtopo).")
    if subparsers is not None:
        parser.set_defaults(func=env_command)
    return parser


def env_command(args):
    s = env_summary()
    info = {
        "`accelerate_hpc_test_amd` version": version,
        "Platform": platform.platform(),
        "`accelerate` bash location": _which("accelerate-amd"),
        "Python version": platform.python_version(),
        "Numpy version": np.__version__,
        "PyTorch version": f"{torch.__version__} (HIP {s['hip']})",
        "RCCL version": s["rccl"],
        "System RAM": f"{psutil.virtual_memory().total / 1024**3:.2f} GB",
        "GPU count": s["gpus"],
        "GPU type": ", ".join(sorted(set(s["gpu_names"]))) if s["gpu_names"] else "none",
        "GPU arch": s["arch"],
        "HBM per device (GiB)": s["hbm_per_device_gb"],
        "HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES", "unset"),
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "unset"),
    }
    config_file = getattr(args, "config_file", None)
    cfg = None
    if config_file is not None or os.path.isfile(default_config_file):
        try:
            cfg = load_config_from_file(config_file).to_dict()
        except Exception as e:  # a broken config file is itself useful information
            cfg = f"unreadable ({e})"
    lines = ["", "Copy-and-paste the text below in your GitHub issue", ""]
    lines += [f"- {k}: {v}" for k, v in info.items()]
    lines.append("- Default config:")
    if isinstance(cfg, dict):
        lines += [f"\t- {k}: {v}" for k, v in cfg.items()]
    else:
        lines.append(f"\t{cfg if cfg else 'Not found'}")
    if getattr(args, "topology", False):
        from ..parallel.topology import environment_problems, link_problems, parse_link_types

        text = get_xgmi_topology()
        lines.append("- xGMI topology:")
        lines.append(text or "\tunavailable")
        types = parse_link_types(text)
        gpus = sorted({i for i, _ in types})
        problems = environment_problems() + link_problems(gpus, types)
        lines.append("- Communication checks: " + ("ok" if not problems else "; ".join(problems)))
    print("\n".join(lines))
    info["Default config"] = cfg
    return info


def _which(name):
    try:
        return subprocess.run(["which", name], capture_output=True, text=True, check=False).stdout.strip() or "not on PATH"
    except Exception:
        return "unknown"


def main() -> int:
    parser = env_command_parser()
    args = parser.parse_args()
    env_command(args)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
