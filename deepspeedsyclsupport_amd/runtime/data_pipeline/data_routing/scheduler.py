"""Random-LTD token-budget schedule (reference `runtime/data_pipeline/data_routing/scheduler.py`): the number of
tokens each middle layer keeps grows from `min_value` to `max_value` over `schedule_config.require_steps`, in
multiples of `seq_per_step` (fixed_linear)."""
import math


class RandomLTDScheduler:

    def __init__(self, config):
        self.config = config
        sch = config["random_ltd_schedule"]
        self.min_value, self.max_value = sch["min_value"], sch["max_value"]
        self.schedule_type = sch.get("schedule_type", "fixed_linear")
        sc = sch["schedule_config"]
        self.require_steps = sc["require_steps"]
        self.seq_per_step = sc.get("seq_per_step", 16)
        self.total_layer_num = config.get("total_layer_num", 0)
        self.random_ltd_layer_num = config.get("random_ltd_layer_num", 0)
        self.state = {"current_seq": self.min_value, "consumed_layer_tokens": 0, "step": 0}

    def get_current_seq(self):
        return self.state["current_seq"]

    def set_current_seq(self, seq):
        self.state["current_seq"] = seq

    def update_seq(self, global_steps):
        if self.state["current_seq"] < self.max_value:
            frac = min(float(global_steps) / self.require_steps, 1.0)
            seq = self.min_value + (self.max_value - self.min_value) * frac
            seq = int(math.floor(seq / self.seq_per_step) * self.seq_per_step)
            self.state["current_seq"] = min(max(seq, self.min_value), self.max_value)
        self.state["step"] = global_steps
        return self.state["current_seq"]

    def get_total_layer_tokens(self, train_iters):
        total = 0
        for s in range(train_iters):
            frac = min(float(s) / self.require_steps, 1.0)
            total += self.min_value + (self.max_value - self.min_value) * frac
        return total

    def state_dict(self):
        return dict(self.state)

    def load_state_dict(self, sd):
        self.state.update(sd)
