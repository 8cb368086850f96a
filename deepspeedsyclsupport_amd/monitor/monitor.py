"""Metric fan-out to TensorBoard / W&B / CSV (reference `deepspeed/monitor/*`). Backends are optional imports."""
import csv
import os

from .. import comm as dist


class Monitor:

    def __init__(self, cfg):
        self.enabled = cfg.enabled

    def write_events(self, event_list):
        raise NotImplementedError


class TensorBoardMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        self.summary_writer = None
        if self.enabled and dist.get_rank() == 0:
            try:
                from torch.utils.tensorboard import SummaryWriter
                self.summary_writer = SummaryWriter(log_dir=os.path.join(cfg.output_path or "runs", cfg.job_name))
            except Exception:
                self.enabled = False

    def write_events(self, event_list, flush=True):
        if self.summary_writer is None:
            return
        for name, value, step in event_list:
            self.summary_writer.add_scalar(name, value, step)
        if flush:
            self.summary_writer.flush()


class WandbMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        if self.enabled and dist.get_rank() == 0:
            try:
                import wandb
                wandb.init(project=cfg.project, group=cfg.group, entity=cfg.team)
                self._wandb = wandb
            except Exception:
                self.enabled = False

    def write_events(self, event_list):
        if self.enabled and dist.get_rank() == 0:
            for name, value, step in event_list:
                self._wandb.log({name: value}, step=step)


class csvMonitor(Monitor):

    def __init__(self, cfg):
        super().__init__(cfg)
        self.log_dir = os.path.join(cfg.output_path or "csv_logs", cfg.job_name)
        if self.enabled and dist.get_rank() == 0:
            os.makedirs(self.log_dir, exist_ok=True)

    def write_events(self, event_list):
        if not (self.enabled and dist.get_rank() == 0):
            return
        for name, value, step in event_list:
            fname = os.path.join(self.log_dir, name.replace("/", "_") + ".csv")
            new = not os.path.exists(fname)
            with open(fname, "a", newline="") as f:
                w = csv.writer(f)
                if new:
                    w.writerow(["step", name])
                w.writerow([step, value])


class MonitorMaster(Monitor):

    def __init__(self, monitor_config):
        self.enabled = monitor_config.enabled
        self.monitors = []
        if monitor_config.tensorboard.enabled:
            self.monitors.append(TensorBoardMonitor(monitor_config.tensorboard))
        if monitor_config.wandb.enabled:
            self.monitors.append(WandbMonitor(monitor_config.wandb))
        if monitor_config.csv_monitor.enabled:
            self.monitors.append(csvMonitor(monitor_config.csv_monitor))

    def write_events(self, event_list):
        for m in self.monitors:
            m.write_events(event_list)


def check_tb_availability():
    """Raise ImportError unless a TensorBoard writer can be created."""
    try:
        from torch.utils.tensorboard import SummaryWriter  # noqa: F401
    except ImportError:
        print("If you want to use tensorboard logging, please `pip install tensorboard`")
        raise


def check_wandb_availability():
    try:
        import wandb  # noqa: F401
    except ImportError:
        print('If you want to use wandb logging, please `pip install wandb` and follow the instructions at '
              'https://docs.wandb.ai/quickstart')
        raise

