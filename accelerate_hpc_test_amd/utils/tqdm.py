"""Progress bar that only renders on the main process (parity: reference utils/tqdm.py)."""

from .imports import is_tqdm_available


def tqdm(*args, main_process_only: bool = True, **kwargs):
    """`tqdm.auto.tqdm` wrapper; on non-main local processes the bar is disabled (`main_process_only=True`)."""
    if not is_tqdm_available():
        raise ImportError("`tqdm` is not installed.")
    if len(args) > 0 and isinstance(args[0], bool):
        raise ValueError("Passing `True` or `False` as the first argument is not supported; use `main_process_only=`.")
    from tqdm.auto import tqdm as _tqdm

    if main_process_only:
        from .other import PartialState

        kwargs["disable"] = kwargs.get("disable", False) or PartialState().local_process_index != 0
    return _tqdm(*args, **kwargs)
