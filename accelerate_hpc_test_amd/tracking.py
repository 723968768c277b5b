"""Experiment trackers.

Parity: `/root/reference/src/accelerate/tracking.py:45-1317` — `GeneralTracker` API (`name`, `requires_logging_directory`,
`store_init_configuration`, `log`, `finish`, `tracker`), `on_main_process` gating, `filter_trackers`, and adapters
for TensorBoard, WandB, Trackio, CometML, Aim, MLflow, ClearML, DVCLive, SwanLab (each imported lazily; only the
ones installed can be selected). `JSONLTracker` is an always-available file tracker (one JSON line per `log`),
used by the MI355X throughput benchmark and tests.
"""

from __future__ import annotations

import json
import os
import time
from functools import wraps
from typing import Any, Optional, Union

from .logging import get_logger
from .state import PartialState
from .utils.dataclasses import LoggerType
from .utils.imports import (
    is_aim_available,
    is_clearml_available,
    is_comet_ml_available,
    is_dvclive_available,
    is_mlflow_available,
    is_swanlab_available,
    is_tensorboard_available,
    is_trackio_available,
    is_wandb_available,
)

logger = get_logger(__name__)


def on_main_process(function):
    """Run a tracker method only on the main process (when `main_process_only` is set on the tracker)."""

    @wraps(function)
    def execute_on_main_process(self, *args, **kwargs):
        if getattr(self, "main_process_only", False):
            return PartialState().on_main_process(function)(self, *args, **kwargs)
        return function(self, *args, **kwargs)

    return execute_on_main_process


def get_available_trackers():
    return _available_trackers


class GeneralTracker:
    """Base class for trackers. Subclasses set `name`, `requires_logging_directory`, and implement `tracker`,
    `store_init_configuration`, `log` (and optionally `finish`)."""

    main_process_only = True

    _REQUIRED = ("name", "requires_logging_directory", "tracker")

    def __init__(self, _blank=False):
        missing = [] if _blank else [f"`{a}`" for a in self._REQUIRED if not hasattr(type(self), a) and not hasattr(self, a)]
        if missing:
            raise NotImplementedError(
                "The implementation for this tracker class is missing the following required attributes. Please "
                f"define them in the class definition: {', '.join(missing)}")

    def start(self):
        pass

    def store_init_configuration(self, values: dict):
        pass

    def log(self, values: dict, step: Optional[int], **kwargs):
        pass

    def finish(self):
        pass


class JSONLTracker(GeneralTracker):
    """Native tracker: appends `{"step": ..., "time": ..., **values}` lines to `<logging_dir>/<run_name>/metrics.jsonl`."""

    name = "jsonl"
    requires_logging_directory = True

    @on_main_process
    def __init__(self, run_name: str, logging_dir: Union[str, os.PathLike] = ".", **kwargs):
        super().__init__()
        self.run_name = run_name
        self.dir = os.path.join(str(logging_dir), run_name)
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, "metrics.jsonl")
        self._f = None

    @property
    def tracker(self):
        return self.path

    @on_main_process
    def start(self):
        self._f = open(self.path, "a")

    @on_main_process
    def store_init_configuration(self, values: dict):
        with open(os.path.join(self.dir, "config.json"), "w") as f:
            json.dump({k: (v if isinstance(v, (int, float, str, bool, type(None), list, dict)) else str(v)) for k, v in values.items()}, f, indent=2)

    @on_main_process
    def log(self, values: dict, step: Optional[int] = None, **kwargs):
        if self._f is None:
            self.start()
        rec = {"step": step, "time": time.time()}
        for k, v in values.items():
            if hasattr(v, "item"):
                v = v.item()
            rec[k] = v
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    @on_main_process
    def finish(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class TensorBoardTracker(GeneralTracker):
    name = "tensorboard"
    requires_logging_directory = True

    @on_main_process
    def __init__(self, run_name: str, logging_dir: Union[str, os.PathLike], **kwargs):
        super().__init__()
        self.run_name = run_name
        self.logging_dir = os.path.join(logging_dir, run_name)
        self.init_kwargs = kwargs

    @on_main_process
    def start(self):
        try:
            from torch.utils import tensorboard
        except ModuleNotFoundError:
            import tensorboardX as tensorboard
        self.writer = tensorboard.SummaryWriter(self.logging_dir, **self.init_kwargs)

    @property
    def tracker(self):
        return self.writer

    @on_main_process
    def store_init_configuration(self, values: dict):
        self.writer.add_hparams(values, metric_dict={})
        self.writer.flush()
        project_run_name = time.time()
        dir_name = os.path.join(self.logging_dir, str(project_run_name))
        os.makedirs(dir_name, exist_ok=True)
        import yaml

        with open(os.path.join(dir_name, "hparams.yml"), "w") as outfile:
            yaml.safe_dump({k: (v if isinstance(v, (int, float, str, bool)) else str(v)) for k, v in values.items()}, outfile)

    @on_main_process
    def log(self, values: dict, step: Optional[int] = None, **kwargs):
        for k, v in _scalars(values).items():
            if isinstance(v, (int, float)):
                self.writer.add_scalar(k, v, global_step=step, **kwargs)
            elif isinstance(v, str):
                self.writer.add_text(k, v, global_step=step, **kwargs)
            elif isinstance(v, dict):
                self.writer.add_scalars(k, v, global_step=step, **kwargs)
        self.writer.flush()

    @on_main_process
    def log_images(self, values: dict, step: Optional[int] = None, **kwargs):
        """`values`: {tag: stacked images [N, C, H, W] (array or tensor)}."""
        for k, v in values.items():
            self.writer.add_images(k, v, global_step=step, **kwargs)
        self.writer.flush()

    @on_main_process
    def finish(self):
        self.writer.close()


def _scalars(values: dict) -> dict:
    """0-d tensors / numpy scalars -> Python numbers (tracker libraries reject tensors)."""
    out = {}
    for k, v in values.items():
        if hasattr(v, "item") and getattr(v, "ndim", 0) == 0:
            v = v.item()
        out[k] = v
    return out


class _LazyTracker(GeneralTracker):
    """Adapter for a tracker library with an init/log/finish API, imported only when selected."""

    module_name = ""
    requires_logging_directory = False

    @on_main_process
    def __init__(self, run_name: str, /, **kwargs):
        # positional-only: a library's own `run_name` option (MLflow, ...) can travel in **kwargs
        super().__init__()
        self.run_name = run_name  # the project / experiment name the Accelerator passes
        self.init_kwargs = kwargs
        self.run = None

    @property
    def tracker(self):
        return self.run


class WandBTracker(_LazyTracker):
    name = "wandb"
    main_process_only = False

    @on_main_process
    def start(self):
        import wandb

        self.run = wandb.init(project=self.run_name, **self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values: dict):
        import wandb

        wandb.config.update(values, allow_val_change=True)

    @on_main_process
    def log(self, values: dict, step: Optional[int] = None, **kwargs):
        self.run.log(_scalars(values), step=step, **kwargs)

    @on_main_process
    def log_images(self, values: dict, step: Optional[int] = None, **kwargs):
        """`values`: {key: list of images (arrays / PIL)} -> wandb.Image panels."""
        import wandb

        self.log({k: [wandb.Image(img) for img in imgs] for k, imgs in values.items()}, step=step, **kwargs)

    @on_main_process
    def log_table(self, table_name: str, columns: Optional[list] = None, data: Optional[list] = None, dataframe=None,
                  step: Optional[int] = None, **kwargs):
        """One wandb.Table from `columns` + `data` rows, or from a pandas `dataframe`."""
        import wandb

        self.log({table_name: wandb.Table(columns=columns, data=data, dataframe=dataframe)}, step=step, **kwargs)

    @on_main_process
    def finish(self):
        self.run.finish()


class TrackioTracker(_LazyTracker):
    name = "trackio"

    @on_main_process
    def start(self):
        import trackio

        self.run = trackio.init(project=self.run_name, **self.init_kwargs)

    @on_main_process
    def log(self, values, step=None, **kwargs):
        self.run.log(_scalars(values), **kwargs)

    @on_main_process
    def finish(self):
        self.run.finish()


class CometMLTracker(_LazyTracker):
    name = "comet_ml"

    @on_main_process
    def start(self):
        import comet_ml

        self.run = comet_ml.start(project_name=self.run_name, **self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values):
        self.run.log_parameters(values)

    @on_main_process
    def log(self, values, step=None, **kwargs):
        if step is not None:
            self.run.set_step(step)
        for k, v in _scalars(values).items():
            if isinstance(v, (int, float)):
                self.run.log_metric(k, v, step=step, **kwargs)
            elif isinstance(v, str):
                self.run.log_other(k, v, **kwargs)
            elif isinstance(v, dict):
                self.run.log_metrics(v, step=step, **kwargs)

    @on_main_process
    def finish(self):
        self.run.end()


class AimTracker(_LazyTracker):
    name = "aim"
    requires_logging_directory = True

    @on_main_process
    def __init__(self, run_name: str, /, logging_dir=".", **kwargs):
        super().__init__(run_name, **kwargs)
        self.aim_repo_path = logging_dir

    @on_main_process
    def start(self):
        from aim import Run

        self.run = Run(repo=self.aim_repo_path, **self.init_kwargs)
        self.run.name = self.run_name

    @on_main_process
    def store_init_configuration(self, values):
        self.run["hparams"] = values

    @on_main_process
    def log(self, values, step=None, **kwargs):
        for key, value in _scalars(values).items():
            self.run.track(value, name=key, step=step, **kwargs)

    @on_main_process
    def log_images(self, values: dict, step: Optional[int] = None, kwargs: Optional[dict] = None):
        """`values`: {name: image or (image, caption)}; `kwargs` = {"aim_image": {...}, "track": {...}}."""
        import aim

        kwargs = kwargs or {}
        for name, val in values.items():
            img, caption = val if isinstance(val, tuple) else (val, "")
            self.run.track(aim.Image(img, caption=caption, **kwargs.get("aim_image", {})), name=name, step=step,
                           **kwargs.get("track", {}))

    @on_main_process
    def finish(self):
        self.run.close()


class MLflowTracker(_LazyTracker):
    name = "mlflow"
    requires_logging_directory = False

    @on_main_process
    def start(self):
        import mlflow

        exp = mlflow.set_experiment(self.run_name)
        self.run = mlflow.start_run(experiment_id=exp.experiment_id, **self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values):
        import mlflow

        mlflow.log_params({k: str(v)[:250] for k, v in values.items()})

    @on_main_process
    def log(self, values, step=None, **kwargs):
        import mlflow

        vals = _scalars(values)
        skipped = [k for k, v in vals.items() if not isinstance(v, (int, float))]
        if skipped:
            logger.warning_once(f"MLflow logs numbers only; not logged: {skipped}")
        mlflow.log_metrics({k: v for k, v in vals.items() if isinstance(v, (int, float))}, step=step)

    @on_main_process
    def log_figure(self, figure, artifact_file: str, **kwargs):
        import mlflow

        mlflow.log_figure(figure=figure, artifact_file=artifact_file, **kwargs)

    @on_main_process
    def log_artifact(self, local_path: str, artifact_path: Optional[str] = None):
        import mlflow

        mlflow.log_artifact(local_path=local_path, artifact_path=artifact_path)

    @on_main_process
    def log_artifacts(self, local_dir: str, artifact_path: Optional[str] = None):
        import mlflow

        mlflow.log_artifacts(local_dir=local_dir, artifact_path=artifact_path)

    @on_main_process
    def finish(self):
        import mlflow

        mlflow.end_run()


class ClearMLTracker(_LazyTracker):
    name = "clearml"

    @on_main_process
    def start(self):
        from clearml import Task

        self.run = Task.init(project_name=self.run_name, **self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values):
        self.run.connect_configuration(values)

    @staticmethod
    def _title_series(key: str):
        """"eval_loss" -> ("loss", "eval"); keys without a split prefix -> (key, "train")."""
        for prefix in ("eval", "test", "train"):
            if key.startswith(prefix + "_"):
                return key[len(prefix) + 1 :], prefix
        return key, "train"

    @on_main_process
    def log(self, values, step=None, **kwargs):
        clearml_logger = self.run.get_logger()
        for k, v in _scalars(values).items():
            if not isinstance(v, (int, float)):
                logger.warning_once(f"ClearML logs numbers only; not logged: {k}")
                continue
            if step is None:
                clearml_logger.report_single_value(name=k, value=v, **kwargs)
            else:
                title, series = self._title_series(k)
                clearml_logger.report_scalar(title=title, series=series, value=v, iteration=step, **kwargs)

    @on_main_process
    def log_images(self, values: dict, step: Optional[int] = None, **kwargs):
        clearml_logger = self.run.get_logger()
        for k, v in values.items():
            title, series = self._title_series(k)
            clearml_logger.report_image(title=title, series=series, iteration=step, image=v, **kwargs)

    @on_main_process
    def log_table(self, table_name: str, columns: Optional[list] = None, data: Optional[list] = None, dataframe=None,
                  step: Optional[int] = None, **kwargs):
        """A table from `columns` + `data` rows (header row first) or a pandas `dataframe`."""
        table = dataframe
        if table is None:
            if data is None:
                raise ValueError("`ClearMLTracker.log_table` needs `data` or `dataframe`.")
            table = ([list(columns)] if columns is not None else []) + [list(r) for r in data]
        title, series = self._title_series(table_name)
        self.run.get_logger().report_table(title=title, series=series, table_plot=table, iteration=step, **kwargs)

    @on_main_process
    def finish(self):
        self.run.close()


class DVCLiveTracker(_LazyTracker):
    name = "dvclive"

    @on_main_process
    def start(self):
        from dvclive import Live

        self.run = Live(**self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values):
        self.run.log_params(values)

    @on_main_process
    def log(self, values, step=None, **kwargs):
        if step is not None:
            self.run.step = step
        for k, v in _scalars(values).items():
            self.run.log_metric(k, v, **kwargs)
        self.run.next_step()

    @on_main_process
    def finish(self):
        self.run.end()


class SwanLabTracker(_LazyTracker):
    name = "swanlab"

    @on_main_process
    def start(self):
        import swanlab

        self.run = swanlab.init(project=self.run_name, **self.init_kwargs)

    @on_main_process
    def store_init_configuration(self, values):
        import swanlab

        swanlab.config.update(values, allow_val_change=True)

    @on_main_process
    def log(self, values, step=None, **kwargs):
        self.run.log(_scalars(values), step=step, **kwargs)

    @on_main_process
    def log_images(self, values: dict, step: Optional[int] = None, **kwargs):
        import swanlab

        self.log({k: [swanlab.Image(img) for img in imgs] for k, imgs in values.items()}, step=step, **kwargs)

    @on_main_process
    def finish(self):
        self.run.finish()


LOGGER_TYPE_TO_CLASS = {
    "aim": AimTracker,
    "comet_ml": CometMLTracker,
    "mlflow": MLflowTracker,
    "tensorboard": TensorBoardTracker,
    "wandb": WandBTracker,
    "clearml": ClearMLTracker,
    "dvclive": DVCLiveTracker,
    "swanlab": SwanLabTracker,
    "trackio": TrackioTracker,
    "jsonl": JSONLTracker,
}

_available_trackers = ["jsonl"]
for _name, _check in (
    ("tensorboard", is_tensorboard_available),
    ("wandb", is_wandb_available),
    ("comet_ml", is_comet_ml_available),
    ("aim", is_aim_available),
    ("mlflow", is_mlflow_available),
    ("clearml", is_clearml_available),
    ("dvclive", is_dvclive_available),
    ("swanlab", is_swanlab_available),
    ("trackio", is_trackio_available),
):
    if _check():
        _available_trackers.append(_name)


def _resolve_tracker(entry, logging_dir):
    """One `log_with` entry -> a GeneralTracker instance, a usable LoggerType, or None (package not installed)."""
    if isinstance(entry, GeneralTracker):
        return entry
    try:
        kind = LoggerType(entry)
    except ValueError:
        raise ValueError(f"Unsupported logging capability: {entry}. Choose between {LoggerType.list()}") from None
    name = str(kind)
    if name not in get_available_trackers():
        logger.debug(f"Tracker `{name}` requested but its package is not installed; skipping it.")
        return None
    if LOGGER_TYPE_TO_CLASS[name].requires_logging_directory and logging_dir is None:
        raise ValueError(f"Logging with `{name}` requires a `logging_dir` to be passed in.")
    return kind


def filter_trackers(log_with: Optional[list[Union[str, LoggerType, GeneralTracker]]] = None, logging_dir: Union[str, os.PathLike] = None):
    """Resolve `log_with` to the list of usable trackers: custom tracker objects pass through, names / LoggerTypes
    are kept when their package is installed (checking the logging-directory requirement), "all" expands to every
    installed tracker. Behaviour: reference tracking.py:1262-1317."""
    if log_with is None:
        return []
    entries = list(log_with) if isinstance(log_with, (list, tuple)) else [log_with]
    custom = [e for e in entries if isinstance(e, GeneralTracker)]
    if any(e == "all" or e == LoggerType.ALL for e in entries if not isinstance(e, GeneralTracker)):
        return custom + get_available_trackers()
    resolved = []
    for entry in entries:
        t = _resolve_tracker(entry, logging_dir)
        if t is not None and (isinstance(t, GeneralTracker) or t not in resolved):
            resolved.append(t)
    return resolved
