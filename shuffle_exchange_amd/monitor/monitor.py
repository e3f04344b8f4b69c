"""Training monitors (parity: reference monitor/monitor.py:30 MonitorMaster, csv_monitor.py:12,
tensorboard.py:13, wandb.py:12, comet.py:23). CSV is always available; TensorBoard / W&B / Comet are
used only if their packages import (none is required)."""
import csv
import os


class Monitor:
    enabled = False

    def write_events(self, events):
        raise NotImplementedError


class CSVMonitor(Monitor):
    def __init__(self, cfg):
        self.enabled = cfg.enabled
        self.dir = os.path.join(cfg.output_path or "./csv_monitor", cfg.job_name)
        self._files = {}

    def write_events(self, events):
        if not self.enabled:
            return
        os.makedirs(self.dir, exist_ok=True)
        for name, value, step in events:
            fn = os.path.join(self.dir, name.replace("/", "_") + ".csv")
            new = not os.path.exists(fn)
            with open(fn, "a", newline="") as f:
                w = csv.writer(f)
                if new:
                    w.writerow(["step", name])
                w.writerow([step, value])


class TensorBoardMonitor(Monitor):
    def __init__(self, cfg):
        self.enabled = False
        if not cfg.enabled:
            return
        try:
            from torch.utils.tensorboard import SummaryWriter
            self.writer = SummaryWriter(log_dir=os.path.join(cfg.output_path or "./runs", cfg.job_name))
            self.enabled = True
        except Exception:
            self.enabled = False

    def write_events(self, events):
        if self.enabled:
            for name, value, step in events:
                self.writer.add_scalar(name, value, step)
            self.writer.flush()


class WandbMonitor(Monitor):
    """Weights & Biases (reference monitor/wandb.py:12); active only if ``wandb`` imports."""

    def __init__(self, cfg):
        self.enabled = False
        if not getattr(cfg, "enabled", False):
            return
        try:
            import wandb
            wandb.init(project=getattr(cfg, "project", None) or "sxe", group=getattr(cfg, "group", None),
                       entity=getattr(cfg, "team", None))
            self._wandb = wandb
            self.enabled = True
        except Exception:
            self.enabled = False

    def write_events(self, events):
        if self.enabled:
            for name, value, step in events:
                self._wandb.log({name: value}, step=step)


class CometMonitor(Monitor):
    """Comet ML (reference monitor/comet.py:23); active only if ``comet_ml`` imports."""

    def __init__(self, cfg):
        self.enabled = False
        if not getattr(cfg, "enabled", False):
            return
        try:
            import comet_ml
            self._exp = comet_ml.Experiment(project_name=getattr(cfg, "project", None),
                                            workspace=getattr(cfg, "workspace", None))
            name = getattr(cfg, "experiment_name", None)
            if name:
                self._exp.set_name(name)
            self.enabled = True
        except Exception:
            self.enabled = False

    def write_events(self, events):
        if self.enabled:
            for name, value, step in events:
                self._exp.log_metric(name, value, step=step)


class MonitorMaster(Monitor):
    def __init__(self, model_cfg):
        self.monitors = [CSVMonitor(model_cfg.csv_monitor), TensorBoardMonitor(model_cfg.tensorboard),
                         WandbMonitor(model_cfg.wandb), CometMonitor(model_cfg.comet)]
        self.enabled = any(m.enabled for m in self.monitors)

    def write_events(self, events):
        for m in self.monitors:
            if m.enabled:
                m.write_events(events)
