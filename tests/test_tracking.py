"""Tracker adapters against fake tracker libraries injected into `sys.modules` (none of them is installed here): what
each adapter calls on init / config / log / images / tables / finish, deferred initialisation (nothing is imported
or started in `__init__`), tensor scalars converted, and the Accelerator round trip (`init_trackers` -> `log` ->
`end_training`) with library trackers, the native JSONL tracker and a custom `GeneralTracker`. Reference behaviour:
`/root/reference/tests/test_tracking.py` (TensorBoard :89, WandB :158, MLflow :223, CometML :327, ClearML :388,
SwanLab :530, custom :689, DVCLive :736, deferred init :779)."""

import json
import os
import sys
import types
from unittest import mock

import numpy as np
import pytest
import torch

from accelerate_hpc_test_amd import tracking
from accelerate_hpc_test_amd.state import AcceleratorState, GradientState
from accelerate_hpc_test_amd.tracking import (
    AimTracker,
    ClearMLTracker,
    CometMLTracker,
    DVCLiveTracker,
    GeneralTracker,
    JSONLTracker,
    MLflowTracker,
    SwanLabTracker,
    TensorBoardTracker,
    TrackioTracker,
    WandBTracker,
)


@pytest.fixture(autouse=True)
def _reset():
    AcceleratorState._reset_state(True)
    GradientState._reset_state()
    yield
    AcceleratorState._reset_state(True)


def _fake(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    return m


def test_deferred_initialisation_imports_nothing():
    """Constructing any adapter must not import or start its library (reference TrackerDeferredInitializationTest)."""
    poison = {n: None for n in ("wandb", "trackio", "comet_ml", "aim", "mlflow", "clearml", "dvclive", "swanlab", "tensorboardX")}
    with mock.patch.dict(sys.modules, poison):  # a None entry makes `import x` raise
        for cls in (WandBTracker, TrackioTracker, CometMLTracker, MLflowTracker, ClearMLTracker, DVCLiveTracker, SwanLabTracker):
            t = cls("run")
            assert t.tracker is None
        AimTracker("run", logging_dir="x")
        TensorBoardTracker("run", "logs")


def test_wandb_adapter_calls():
    run = mock.MagicMock()
    wb = _fake("wandb", init=mock.MagicMock(return_value=run), config=mock.MagicMock(), Image=mock.MagicMock(side_effect=lambda x: ("img", x)),
               Table=mock.MagicMock(side_effect=lambda **kw: ("table", kw)))
    with mock.patch.dict(sys.modules, {"wandb": wb}):
        t = WandBTracker("proj", entity="team")
        t.start()
        wb.init.assert_called_once_with(project="proj", entity="team")
        assert t.tracker is run
        t.store_init_configuration({"lr": 1e-3})
        wb.config.update.assert_called_once_with({"lr": 1e-3}, allow_val_change=True)
        t.log({"loss": torch.tensor(2.5), "acc": 0.5}, step=7)
        run.log.assert_called_with({"loss": 2.5, "acc": 0.5}, step=7)
        t.log_images({"samples": [np.zeros((2, 2)), np.ones((2, 2))]}, step=8)
        args, kw = run.log.call_args
        assert [a[0] for a in args[0]["samples"]] == ["img", "img"] and kw == {"step": 8}
        t.log_table("preds", columns=["a", "b"], data=[[1, 2]], step=9)
        args, kw = run.log.call_args
        assert args[0]["preds"] == ("table", {"columns": ["a", "b"], "data": [[1, 2]], "dataframe": None}) and kw == {"step": 9}
        t.finish()
        run.finish.assert_called_once()


def test_tensorboard_adapter_calls(tmp_path):
    writer = mock.MagicMock()
    tbx = _fake("tensorboardX", SummaryWriter=mock.MagicMock(return_value=writer))
    # torch.utils.tensorboard needs the tensorboard package (absent) -> the adapter falls back to tensorboardX
    with mock.patch.dict(sys.modules, {"tensorboardX": tbx, "torch.utils.tensorboard": None}):
        t = TensorBoardTracker("run", str(tmp_path), flush_secs=5)
        t.start()
        tbx.SummaryWriter.assert_called_once_with(os.path.join(str(tmp_path), "run"), flush_secs=5)
        t.store_init_configuration({"lr": 0.1, "obj": object()})
        writer.add_hparams.assert_called_once()
        hp = [p for p in (tmp_path / "run").rglob("hparams.yml")]
        assert len(hp) == 1 and "lr: 0.1" in hp[0].read_text()
        t.log({"loss": torch.tensor(1.0), "note": "hi", "multi": {"a": 1.0}}, step=3)
        writer.add_scalar.assert_called_once_with("loss", 1.0, global_step=3)
        writer.add_text.assert_called_once_with("note", "hi", global_step=3)
        writer.add_scalars.assert_called_once_with("multi", {"a": 1.0}, global_step=3)
        imgs = np.zeros((2, 3, 4, 4))
        t.log_images({"grid": imgs}, step=4)
        writer.add_images.assert_called_once_with("grid", imgs, global_step=4)
        t.finish()
        writer.close.assert_called_once()


def test_mlflow_adapter_calls():
    ml = _fake("mlflow", set_experiment=mock.MagicMock(return_value=types.SimpleNamespace(experiment_id="e1")),
               start_run=mock.MagicMock(return_value="RUN"), log_params=mock.MagicMock(), log_metrics=mock.MagicMock(),
               log_figure=mock.MagicMock(), log_artifact=mock.MagicMock(), log_artifacts=mock.MagicMock(), end_run=mock.MagicMock())
    with mock.patch.dict(sys.modules, {"mlflow": ml}):
        t = MLflowTracker("exp", run_name="r")
        t.start()
        ml.set_experiment.assert_called_once_with("exp")
        ml.start_run.assert_called_once_with(experiment_id="e1", run_name="r")
        t.store_init_configuration({"lr": 0.1, "long": "x" * 400})
        params = ml.log_params.call_args[0][0]
        assert params["lr"] == "0.1" and len(params["long"]) == 250
        t.log({"loss": torch.tensor(0.5), "text": "skip me"}, step=2)
        ml.log_metrics.assert_called_once_with({"loss": 0.5}, step=2)
        t.log_figure("FIG", "plots/f.png")
        ml.log_figure.assert_called_once_with(figure="FIG", artifact_file="plots/f.png")
        t.log_artifact("a.txt", "dir")
        ml.log_artifact.assert_called_once_with(local_path="a.txt", artifact_path="dir")
        t.log_artifacts("outdir")
        ml.log_artifacts.assert_called_once_with(local_dir="outdir", artifact_path=None)
        t.finish()
        ml.end_run.assert_called_once()


def test_comet_adapter_calls():
    exp = mock.MagicMock()
    cm = _fake("comet_ml", start=mock.MagicMock(return_value=exp))
    with mock.patch.dict(sys.modules, {"comet_ml": cm}):
        t = CometMLTracker("proj", workspace="w")
        t.start()
        cm.start.assert_called_once_with(project_name="proj", workspace="w")
        t.store_init_configuration({"lr": 1})
        exp.log_parameters.assert_called_once_with({"lr": 1})
        t.log({"loss": torch.tensor(3.0), "tag": "x", "grp": {"a": 1}}, step=5)
        exp.set_step.assert_called_once_with(5)
        exp.log_metric.assert_called_once_with("loss", 3.0, step=5)
        exp.log_other.assert_called_once_with("tag", "x")
        exp.log_metrics.assert_called_once_with({"a": 1}, step=5)
        t.finish()
        exp.end.assert_called_once()


def test_clearml_adapter_calls():
    task = mock.MagicMock()
    lg = task.get_logger.return_value
    cl = _fake("clearml", Task=types.SimpleNamespace(init=mock.MagicMock(return_value=task)))
    with mock.patch.dict(sys.modules, {"clearml": cl}):
        t = ClearMLTracker("proj", task_name="t")
        t.start()
        cl.Task.init.assert_called_once_with(project_name="proj", task_name="t")
        t.store_init_configuration({"lr": 1})
        task.connect_configuration.assert_called_once_with({"lr": 1})
        t.log({"eval_loss": 1.0, "train_acc": 0.5, "loss": 2.0}, step=3)
        calls = sorted((c.kwargs["title"], c.kwargs["series"], c.kwargs["value"]) for c in lg.report_scalar.call_args_list)
        assert calls == [("acc", "train", 0.5), ("loss", "eval", 1.0), ("loss", "train", 2.0)]
        t.log({"final_bleu": 31.0})
        lg.report_single_value.assert_called_once_with(name="final_bleu", value=31.0)
        t.log_images({"test_img": np.zeros((4, 4))}, step=1)
        assert lg.report_image.call_args.kwargs["title"] == "img" and lg.report_image.call_args.kwargs["series"] == "test"
        t.log_table("eval_tbl", columns=["a", "b"], data=[[1, 2], [3, 4]], step=2)
        assert lg.report_table.call_args.kwargs["table_plot"] == [["a", "b"], [1, 2], [3, 4]]
        with pytest.raises(ValueError):
            t.log_table("x")
        t.finish()
        task.close.assert_called_once()


def test_aim_dvclive_swanlab_trackio_adapters(tmp_path):
    aim_run = mock.MagicMock()
    aim = _fake("aim", Run=mock.MagicMock(return_value=aim_run), Image=mock.MagicMock(side_effect=lambda img, caption="": ("IMG", caption)))
    live = mock.MagicMock()
    dvc = _fake("dvclive", Live=mock.MagicMock(return_value=live))
    sl_run = mock.MagicMock()
    sl = _fake("swanlab", init=mock.MagicMock(return_value=sl_run), config=mock.MagicMock(), Image=mock.MagicMock(side_effect=lambda x: "SIMG"))
    tr_run = mock.MagicMock()
    tr = _fake("trackio", init=mock.MagicMock(return_value=tr_run))
    with mock.patch.dict(sys.modules, {"aim": aim, "dvclive": dvc, "swanlab": sl, "trackio": tr}):
        a = AimTracker("run", logging_dir=str(tmp_path))
        a.start()
        aim.Run.assert_called_once_with(repo=str(tmp_path))
        assert aim_run.name == "run"
        a.store_init_configuration({"lr": 1})
        aim_run.__setitem__.assert_called_once_with("hparams", {"lr": 1})
        a.log({"loss": torch.tensor(1.0)}, step=2)
        aim_run.track.assert_called_with(1.0, name="loss", step=2)
        a.log_images({"pic": (np.zeros(2), "cap")}, step=3)
        assert aim_run.track.call_args.args[0] == ("IMG", "cap")
        a.finish()
        aim_run.close.assert_called_once()

        d = DVCLiveTracker("run", dir="x")
        d.start()
        dvc.Live.assert_called_once_with(dir="x")
        d.store_init_configuration({"lr": 1})
        live.log_params.assert_called_once_with({"lr": 1})
        d.log({"loss": torch.tensor(1.0), "acc": 0.5}, step=4)
        assert live.step == 4 and [c.args for c in live.log_metric.call_args_list] == [("loss", 1.0), ("acc", 0.5)]
        live.next_step.assert_called_once()
        d.finish()
        live.end.assert_called_once()

        s = SwanLabTracker("proj")
        s.start()
        sl.init.assert_called_once_with(project="proj")
        s.store_init_configuration({"lr": 1})
        sl.config.update.assert_called_once_with({"lr": 1}, allow_val_change=True)
        s.log({"loss": torch.tensor(1.0)}, step=1)
        sl_run.log.assert_called_with({"loss": 1.0}, step=1)
        s.log_images({"i": [np.zeros(2)]}, step=2)
        sl_run.log.assert_called_with({"i": ["SIMG"]}, step=2)
        s.finish()
        sl_run.finish.assert_called_once()

        k = TrackioTracker("proj")
        k.start()
        tr.init.assert_called_once_with(project="proj")
        k.log({"loss": torch.tensor(1.0)}, step=1)
        tr_run.log.assert_called_once_with({"loss": 1.0})
        k.finish()
        tr_run.finish.assert_called_once()


def test_accelerator_round_trip_with_library_jsonl_and_custom_trackers(tmp_path):
    from accelerate_hpc_test_amd import Accelerator

    class Custom(GeneralTracker):
        name = "custom"
        requires_logging_directory = False

        def __init__(self):
            super().__init__()
            self.events = []

        @property
        def tracker(self):
            return self.events

        def start(self):
            self.events.append("start")

        def store_init_configuration(self, values):
            self.events.append(("config", values))

        def log(self, values, step=None, **kwargs):
            self.events.append(("log", values, step, kwargs))

        def finish(self):
            self.events.append("finish")

    run = mock.MagicMock()
    wb = _fake("wandb", init=mock.MagicMock(return_value=run), config=mock.MagicMock())
    custom = Custom()
    with mock.patch.dict(sys.modules, {"wandb": wb}), mock.patch.object(tracking, "_available_trackers", ["jsonl", "wandb"]):
        acc = Accelerator(cpu=True, log_with=["wandb", "jsonl", custom], project_dir=str(tmp_path))
        acc.init_trackers("proj", config={"lr": 0.5}, init_kwargs={"wandb": {"tags": ["a"]}})
        wb.init.assert_called_once_with(project="proj", tags=["a"])
        acc.log({"loss": 1.25}, step=1, log_kwargs={"custom": {"commit": True}})
        run.log.assert_called_once_with({"loss": 1.25}, step=1)
        assert acc.get_tracker("custom", unwrap=True) is custom.events
        assert isinstance(acc.get_tracker("jsonl"), JSONLTracker)
        with pytest.raises(ValueError):
            acc.get_tracker("mlflow")
        acc.end_training()
    run.finish.assert_called_once()
    assert custom.events == ["start", ("config", {"lr": 0.5}), ("log", {"loss": 1.25}, 1, {"commit": True}), "finish"]
    lines = (tmp_path / "proj" / "metrics.jsonl").read_text().splitlines()
    assert [json.loads(l)["loss"] for l in lines] == [1.25]
    assert json.loads((tmp_path / "proj" / "config.json").read_text()) == {"lr": 0.5}


def test_filter_trackers_rules(tmp_path):
    from accelerate_hpc_test_amd.state import PartialState

    PartialState(cpu=True)  # the multi-process logger needs the state (as inside Accelerator.__init__)
    with mock.patch.object(tracking, "_available_trackers", ["jsonl", "wandb"]):
        assert [str(t) for t in tracking.filter_trackers(["wandb", "mlflow"])] == ["wandb"]  # mlflow unavailable: dropped
        assert sorted(str(t) for t in tracking.filter_trackers("all", logging_dir=str(tmp_path))) == ["jsonl", "wandb"]
        with pytest.raises(ValueError, match="logging_dir"):
            tracking.filter_trackers(["jsonl"])
        with pytest.raises(ValueError, match="Unsupported"):
            tracking.filter_trackers(["not-a-tracker"])
