"""Curriculum difficulty schedule (reference `runtime/data_pipeline/curriculum_scheduler.py:13-170`; same config keys:
min_difficulty, max_difficulty, schedule_type in {fixed_discrete, fixed_root, fixed_linear, custom},
schedule_config {difficulty, max_step | total_curriculum_step, difficulty_step, root_degree})."""
import math


class CurriculumScheduler:

    def __init__(self, config):
        for k in ("min_difficulty", "max_difficulty", "schedule_type"):
            assert k in config, f"curriculum learning requires '{k}'"
        self.state = dict(min_difficulty=config["min_difficulty"], max_difficulty=config["max_difficulty"],
                          current_difficulty=config["min_difficulty"], schedule_type=config["schedule_type"],
                          schedule_config=config.get("schedule_config", {}))
        t, sc = config["schedule_type"], self.state["schedule_config"]
        if t == "fixed_discrete":
            assert sc.get("difficulty") and sc.get("max_step") is not None
            assert len(sc["difficulty"]) == len(sc["max_step"]) + 1, "need one more difficulty than max_step"
        elif t in ("fixed_root", "fixed_linear"):
            assert "total_curriculum_step" in sc and "difficulty_step" in sc
            if t == "fixed_root":
                assert "root_degree" in sc
        elif t != "custom":
            raise ValueError(f"unsupported curriculum schedule type {t}")
        self.custom_get_difficulty = None

    def get_current_difficulty(self):
        return self.state["current_difficulty"]

    def set_current_difficulty(self, d):
        self.state["current_difficulty"] = d

    def set_custom_get_difficulty(self, fn):
        self.custom_get_difficulty = fn

    def get_state(self):
        return self.state

    def set_state(self, state):
        self.state = state

    def _root(self, step, degree):
        sc = self.state["schedule_config"]
        lo, hi = self.state["min_difficulty"], self.state["max_difficulty"]
        frac = (float(step) / sc["total_curriculum_step"])**(1.0 / degree)
        d = math.floor(frac * (hi - lo) + lo)
        d -= d % sc["difficulty_step"]
        return min(d, hi)

    def get_difficulty(self, global_steps):
        t, sc = self.state["schedule_type"], self.state["schedule_config"]
        if t == "fixed_discrete":
            for diff, mx in zip(sc["difficulty"], sc["max_step"]):
                if global_steps <= mx:
                    return diff
            return sc["difficulty"][-1]
        if t == "fixed_linear":
            return self._root(global_steps, 1)
        if t == "fixed_root":
            return self._root(global_steps, sc["root_degree"])
        return self.custom_get_difficulty(global_steps)

    def update_difficulty(self, global_steps):
        if self.state["current_difficulty"] < self.state["max_difficulty"]:
            self.state["current_difficulty"] = self.get_difficulty(global_steps)
        return self.state["current_difficulty"]
