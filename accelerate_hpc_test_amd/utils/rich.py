"""Opt-in rich tracebacks (parity: reference utils/rich.py): installed when `ACCELERATE_ENABLE_RICH=1`."""

from .environment import parse_flag_from_env
from .imports import is_rich_available

if is_rich_available() and parse_flag_from_env("ACCELERATE_ENABLE_RICH"):
    from rich.traceback import install

    install(show_locals=False)
elif parse_flag_from_env("ACCELERATE_ENABLE_RICH"):
    raise ModuleNotFoundError("To use the rich extension, install rich with `pip install rich`")
