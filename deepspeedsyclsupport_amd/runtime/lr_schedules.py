"""LR schedules with the reference's names, params and state-dict shape (`runtime/lr_schedules.py:267-878`):
LRRangeTest, OneCycle, WarmupLR, WarmupDecayLR, WarmupCosineLR."""
import math

from torch.optim import Optimizer

LR_SCHEDULE = "lr_schedule"
LR_RANGE_TEST = "LRRangeTest"
ONE_CYCLE = "OneCycle"
WARMUP_LR = "WarmupLR"
WARMUP_DECAY_LR = "WarmupDecayLR"
WARMUP_COSINE_LR = "WarmupCosineLR"
VALID_LR_SCHEDULES = [LR_RANGE_TEST, ONE_CYCLE, WARMUP_LR, WARMUP_DECAY_LR, WARMUP_COSINE_LR]
WARMUP_LOG_RATE = "log"
WARMUP_LINEAR_RATE = "linear"


def _opt(optimizer):
    # ZeRO wrappers expose the inner torch optimizer's param_groups
    return optimizer if hasattr(optimizer, "param_groups") else optimizer.optimizer


def _as_list(x, n):
    return list(x) if isinstance(x, (list, tuple)) else [x] * n


class _Sched:

    def __init__(self, optimizer, last_batch_iteration=-1):
        self.optimizer = _opt(optimizer)
        self.last_batch_iteration = last_batch_iteration

    def get_last_lr(self):
        assert getattr(self, "_last_lr", None) is not None, "need to call step() first"
        return self._last_lr

    def step(self, last_batch_iteration=None):
        if last_batch_iteration is None:
            last_batch_iteration = self.last_batch_iteration + 1
        self.last_batch_iteration = last_batch_iteration
        for pg, lr in zip(self.optimizer.param_groups, self.get_lr()):
            pg["lr"] = lr
        self._last_lr = [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"last_batch_iteration": self.last_batch_iteration}

    def load_state_dict(self, sd):
        self.last_batch_iteration = sd["last_batch_iteration"]


class LRRangeTest(_Sched):

    def __init__(self, optimizer, lr_range_test_min_lr=1e-3, lr_range_test_step_size=2000,
                 lr_range_test_step_rate=1.0, lr_range_test_staircase=False, last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        n = len(self.optimizer.param_groups)
        self.min_lr = _as_list(lr_range_test_min_lr, n)
        self.step_size = lr_range_test_step_size
        self.step_rate = lr_range_test_step_rate
        self.staircase = lr_range_test_staircase
        if last_batch_iteration == -1:
            for pg, lr in zip(self.optimizer.param_groups, self.min_lr):
                pg["lr"] = lr
            self._last_lr = list(self.min_lr)

    def get_lr(self):
        it = self.last_batch_iteration + 1
        interval = it // self.step_size if self.staircase else it / self.step_size
        return [m * (1 + self.step_rate * interval) for m in self.min_lr]


class OneCycle(_Sched):

    def __init__(self, optimizer, cycle_min_lr, cycle_max_lr, decay_lr_rate=0.0, cycle_first_step_size=2000,
                 cycle_second_step_size=None, cycle_first_stair_count=0, cycle_second_stair_count=None,
                 decay_step_size=0, cycle_momentum=True, cycle_min_mom=0.8, cycle_max_mom=0.9, decay_mom_rate=0.0,
                 last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        n = len(self.optimizer.param_groups)
        self.min_lrs = _as_list(cycle_min_lr, n)
        self.max_lrs = _as_list(cycle_max_lr, n)
        self.first = float(cycle_first_step_size)
        self.second = float(cycle_second_step_size if cycle_second_step_size is not None else cycle_first_step_size)
        self.total = self.first + self.second
        self.step_ratio = self.first / self.total
        self.first_stair = cycle_first_stair_count
        self.second_stair = cycle_first_stair_count if cycle_second_stair_count is None else cycle_second_stair_count
        self.decay_lr_rate = decay_lr_rate
        self.decay_step_size = decay_step_size
        self.cycle_momentum = cycle_momentum
        self.min_moms = [(cycle_min_mom, 0.99)] * n
        self.max_moms = [(cycle_max_mom, 0.99)] * n
        self.decay_mom_rate = decay_mom_rate
        if last_batch_iteration == -1:
            for pg, lr in zip(self.optimizer.param_groups, self.min_lrs):
                pg["lr"] = lr
            self._last_lr = list(self.min_lrs)

    def _scale(self):
        it = self.last_batch_iteration + 1
        cycle = math.floor(1 + it / self.total)
        x = 1.0 + it / self.total - cycle
        return x / self.step_ratio if x <= self.step_ratio else (x - 1) / (self.step_ratio - 1)

    def get_lr(self):
        it = self.last_batch_iteration + 1
        if it < self.total:
            s = self._scale()
            lrs = [lo + (hi - lo) * s for lo, hi in zip(self.min_lrs, self.max_lrs)]
            if self.cycle_momentum:
                for pg, lo, hi in zip(self.optimizer.param_groups, self.min_moms, self.max_moms):
                    mom = hi[0] - (hi[0] - lo[0]) * s
                    if "betas" in pg:
                        pg["betas"] = (mom, pg["betas"][1])
            return lrs
        decay_it = it - self.total
        interval = decay_it / self.decay_step_size if self.decay_step_size else 0
        if self.cycle_momentum:  # after the cycle momentum returns to (and decays from) its max
            for pg, hi in zip(self.optimizer.param_groups, self.max_moms):
                if "betas" in pg:
                    pg["betas"] = (hi[0] * (1 + self.decay_mom_rate * interval), pg["betas"][1])
        return [lo / (1 + self.decay_lr_rate * interval) for lo in self.min_lrs]


    def get_mom(self):
        """Momentum (beta1 / momentum) per parameter group at the current step, [(mom, beta2)] for Adam-style
        groups; None when momentum is not cycled."""
        if not self.cycle_momentum:
            return None
        it = self.last_batch_iteration + 1
        out = []
        if it < self.total:
            s = self._scale()
            for lo, hi in zip(self.min_moms, self.max_moms):
                out.append((hi[0] - (hi[0] - lo[0]) * s, hi[1]))
            return out
        interval = (it - self.total) / self.decay_step_size if self.decay_step_size else 0
        return [(hi[0] * (1 + self.decay_mom_rate * interval), hi[1]) for hi in self.max_moms]


class WarmupLR(_Sched):

    def __init__(self, optimizer: Optimizer, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        n = len(self.optimizer.param_groups)
        self.min_lrs = _as_list(warmup_min_lr, n)
        self.max_lrs = _as_list(warmup_max_lr, n)
        self.delta_lrs = [b - a for a, b in zip(self.min_lrs, self.max_lrs)]
        self.warmup_num_steps = max(2, warmup_num_steps)
        if warmup_type not in (WARMUP_LOG_RATE, WARMUP_LINEAR_RATE):
            warmup_type = WARMUP_LOG_RATE
        self.warmup_type = warmup_type
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)
        if last_batch_iteration == -1:
            self._last_lr = list(self.min_lrs)

    def _gamma(self):
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            if self.warmup_type == WARMUP_LOG_RATE:
                return self.inverse_log_warm_up * math.log(it + 1)
            return it / self.warmup_num_steps
        return 1.0

    def get_lr(self):
        if self.last_batch_iteration < 0:
            return list(self.min_lrs)
        g = self._gamma()
        return [a + d * g for a, d in zip(self.min_lrs, self.delta_lrs)]


class WarmupDecayLR(WarmupLR):

    def __init__(self, optimizer, total_num_steps, warmup_min_lr=0.0, warmup_max_lr=0.001, warmup_num_steps=1000,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        self.total_num_steps = total_num_steps
        super().__init__(optimizer, warmup_min_lr, warmup_max_lr, warmup_num_steps, warmup_type,
                         last_batch_iteration)

    def _gamma(self):
        it = self.last_batch_iteration
        if it < self.warmup_num_steps:
            return super()._gamma()
        return max(0.0, float(self.total_num_steps - it) /
                   float(max(1.0, self.total_num_steps - self.warmup_num_steps)))


class WarmupCosineLR(_Sched):

    def __init__(self, optimizer, total_num_steps, warmup_min_ratio=0.0, warmup_num_steps=1000, cos_min_ratio=0.0001,
                 warmup_type=WARMUP_LOG_RATE, last_batch_iteration=-1):
        super().__init__(optimizer, last_batch_iteration)
        self.total_num_steps = total_num_steps
        self.warmup_min_ratio = warmup_min_ratio
        self.warmup_num_steps = max(2, warmup_num_steps)
        self.cos_min_ratio = cos_min_ratio
        self.warmup_type = warmup_type
        self.org_lrs = [g["lr"] for g in self.optimizer.param_groups]
        self.inverse_log_warm_up = 1.0 / math.log(self.warmup_num_steps)
        if last_batch_iteration == -1:
            self._last_lr = [lr * warmup_min_ratio for lr in self.org_lrs]

    def get_lr_ratio(self):
        it = self.last_batch_iteration
        if it < 0:
            return 0.0
        if it < self.warmup_num_steps:
            if self.warmup_type == WARMUP_LOG_RATE:
                r = self.inverse_log_warm_up * math.log(it + 1)
            else:
                r = it / self.warmup_num_steps
            return self.warmup_min_ratio + (1.0 - self.warmup_min_ratio) * r
        real = it - self.warmup_num_steps + 1
        total = self.total_num_steps - self.warmup_num_steps
        ratio_delta = 1.0 - self.cos_min_ratio
        return self.cos_min_ratio + ratio_delta * 0.5 * (1 + math.cos(math.pi * min(real / max(total, 1), 1.0)))

    def get_lr(self):
        r = self.get_lr_ratio()
        return [lr * r for lr in self.org_lrs]


SCHEDULERS = {
    LR_RANGE_TEST: LRRangeTest,
    ONE_CYCLE: OneCycle,
    WARMUP_LR: WarmupLR,
    WARMUP_DECAY_LR: WarmupDecayLR,
    WARMUP_COSINE_LR: WarmupCosineLR
}


def add_tuning_arguments(parser):
    group = parser.add_argument_group("Convergence Tuning", "Convergence tuning configurations")
    group.add_argument("--lr_schedule", type=str, default=None, help="LR schedule for training.")
    group.add_argument("--warmup_min_lr", type=float, default=0)
    group.add_argument("--warmup_max_lr", type=float, default=0.001)
    group.add_argument("--warmup_num_steps", type=int, default=1000)
    group.add_argument("--warmup_type", type=str, default=WARMUP_LOG_RATE)
    return parser


# ------------------------------------------------------------------------------------------------ command-line glue
_CLI_KEYS = {
    LR_RANGE_TEST: ("lr_range_test_min_lr", "lr_range_test_step_rate", "lr_range_test_step_size",
                    "lr_range_test_staircase"),
    ONE_CYCLE: ("cycle_first_step_size", "cycle_first_stair_count", "cycle_second_step_size",
                "cycle_second_stair_count", "decay_step_size", "cycle_min_lr", "cycle_max_lr", "decay_lr_rate",
                "cycle_min_mom", "cycle_max_mom", "decay_mom_rate"),
    WARMUP_LR: ("warmup_min_lr", "warmup_max_lr", "warmup_num_steps", "warmup_type"),
    WARMUP_DECAY_LR: ("warmup_min_lr", "warmup_max_lr", "warmup_num_steps", "warmup_type", "total_num_steps"),
    WARMUP_COSINE_LR: ("warmup_min_ratio", "warmup_num_steps", "warmup_type", "total_num_steps", "cos_min_ratio"),
}


def parse_arguments():
    """Parser with the convergence-tuning flags; returns (known args, remaining argv)."""
    import argparse
    parser = add_tuning_arguments(argparse.ArgumentParser())
    return parser.parse_known_args()


def override_params(args, params):
    """Copy every schedule flag that `args` carries (and is not None) into the schedule's parameter dict."""
    for keys in _CLI_KEYS.values():
        for k in keys:
            v = getattr(args, k, None)
            if v is not None:
                params[k] = v


def override_lr_range_test_params(args, params):
    for k in _CLI_KEYS[LR_RANGE_TEST]:
        if getattr(args, k, None) is not None:
            params[k] = getattr(args, k)


def override_1cycle_params(args, params):
    for k in _CLI_KEYS[ONE_CYCLE]:
        if getattr(args, k, None) is not None:
            params[k] = getattr(args, k)


def override_warmupLR_params(args, params):
    for k in _CLI_KEYS[WARMUP_LR]:
        if getattr(args, k, None) is not None:
            params[k] = getattr(args, k)


def get_config_from_args(args):
    """({"type": schedule, "params": {...}}, None) from command-line flags, or (None, reason)."""
    name = getattr(args, "lr_schedule", None)
    if name is None:
        return None, "--lr_schedule not specified on command line"
    if name not in VALID_LR_SCHEDULES:
        return None, f"{name} is not supported LR schedule"
    params = {}
    for k in _CLI_KEYS[name]:
        if getattr(args, k, None) is not None:
            params[k] = getattr(args, k)
    return {"type": name, "params": params}, None


def get_lr_from_config(config):
    """(starting learning rate, "") of a schedule config, or (None, reason)."""
    if "type" not in config:
        return None, "LR schedule type not defined in config"
    if "params" not in config:
        return None, "LR schedule params not defined in config"
    name, params = config["type"], config["params"]
    if name not in VALID_LR_SCHEDULES:
        return None, f"{name} is not a valid LR schedule"
    if name == LR_RANGE_TEST:
        return params.get("lr_range_test_min_lr", 1e-3), ""
    if name == ONE_CYCLE:
        return params.get("cycle_max_lr", 0.1), ""
    return params.get("warmup_max_lr", 0.001), ""


def get_torch_optimizer(optimizer):
    """The torch optimizer behind an optimizer wrapper (ZeRO / fp16 wrappers keep it as `.optimizer`)."""
    import torch
    if isinstance(optimizer, torch.optim.Optimizer):
        return optimizer
    inner = getattr(optimizer, "optimizer", None)
    if isinstance(inner, torch.optim.Optimizer):
        return inner
    raise TypeError(f"{type(optimizer).__name__} is not a subclass of torch.optim.Optimizer")

