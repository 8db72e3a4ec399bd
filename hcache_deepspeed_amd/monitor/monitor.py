"""Monitoring fan-out (reference: monitor/monitor.py MonitorMaster :30-59, csv_monitor, tensorboard, wandb, comet).

Events are ``(name, value, step)`` tuples with the reference names (``Train/Samples/train_loss``,
``Train/Samples/lr``, ``Train/Samples/loss_scale``). Backends whose python packages are absent
(tensorboard / wandb / comet are not installed in this image) are skipped with a warning.
"""
import csv
import os

from ..utils.logging import warning_once


class Monitor:

    def __init__(self, cfg):
        self.enabled = bool(cfg.get("enabled", False))

    def write_events(self, events):
        raise NotImplementedError


class CSVMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        self.output_path = cfg.get("output_path", "") or "."
        self.job_name = cfg.get("job_name", "DeepSpeedJobName")
        self.filenames = {}

    def write_events(self, events):
        if not self.enabled:
            return
        d = os.path.join(self.output_path, self.job_name)
        os.makedirs(d, exist_ok=True)
        for name, value, step in events:
            fn = os.path.join(d, name.replace("/", "_") + ".csv")
            new = not os.path.exists(fn)
            with open(fn, "a", newline="") as f:
                w = csv.writer(f)
                if new:
                    w.writerow(["step", name])
                w.writerow([step, value])


class TensorBoardMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        self.writer = None
        if self.enabled:
            try:
                from torch.utils.tensorboard import SummaryWriter
                path = os.path.join(cfg.get("output_path", "") or ".", cfg.get("job_name", "DeepSpeedJobName"))
                self.writer = SummaryWriter(log_dir=path)
            except Exception:  # tensorboard not installed
                warning_once("tensorboard monitor requested but tensorboard is not importable; disabled")
                self.enabled = False

    def write_events(self, events):
        if self.writer is None:
            return
        for name, value, step in events:
            self.writer.add_scalar(name, value, step)
        self.writer.flush()


class WandbMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        self.wandb = None
        if self.enabled:
            try:
                import wandb
                wandb.init(project=cfg.get("project", "deepspeed"), group=cfg.get("group"), entity=cfg.get("team"))
                self.wandb = wandb
            except Exception:
                warning_once("wandb monitor requested but wandb is not importable; disabled")
                self.enabled = False

    def write_events(self, events):
        if self.wandb is None:
            return
        for name, value, step in events:
            self.wandb.log({name: value}, step=step)


class CometMonitor(Monitor):
    """Comet ML experiment logging (reference monitor/comet.py); gated on ``comet_ml`` being importable."""

    def __init__(self, cfg):
        super().__init__(cfg)
        self.experiment = None
        self.samples_log_interval = int(cfg.get("samples_log_interval", 100))
        if self.enabled:
            try:
                import comet_ml
                kw = {k: cfg.get(k) for k in ("api_key", "project", "workspace", "experiment_key", "mode", "online")
                      if cfg.get(k) is not None}
                self.experiment = comet_ml.start(**kw)
                if cfg.get("experiment_name"):
                    self.experiment.set_name(cfg["experiment_name"])
            except Exception:
                warning_once("comet monitor requested but comet_ml is not importable; disabled")
                self.enabled = False

    def write_events(self, events):
        if self.experiment is None:
            return
        for name, value, step in events:
            if step % self.samples_log_interval == 0:
                self.experiment.log_metric(name, value, step=step)


class MonitorMaster:

    def __init__(self, monitor_config):
        monitor_config = monitor_config or {}
        self.monitors = []
        if (monitor_config.get("csv_monitor") or {}).get("enabled"):
            self.monitors.append(CSVMonitor(monitor_config["csv_monitor"]))
        if (monitor_config.get("tensorboard") or {}).get("enabled"):
            self.monitors.append(TensorBoardMonitor(monitor_config["tensorboard"]))
        if (monitor_config.get("wandb") or {}).get("enabled"):
            self.monitors.append(WandbMonitor(monitor_config["wandb"]))
        if (monitor_config.get("comet") or {}).get("enabled"):
            self.monitors.append(CometMonitor(monitor_config["comet"]))
        self.enabled = any(m.enabled for m in self.monitors)

    def write_events(self, events):
        for m in self.monitors:
            if m.enabled:
                m.write_events(events)
