"""Curriculum learning difficulty schedules (parity: reference
runtime/data_pipeline/curriculum_scheduler.py ``CurriculumScheduler``: fixed_discrete /
fixed_root / fixed_linear / custom, difficulty_step rounding, state dict)."""
import math


class CurriculumScheduler:
    def __init__(self, config):
        c = dict(config)
        self.state = {
            "min_difficulty": c["min_difficulty"],
            "max_difficulty": c["max_difficulty"],
            "current_difficulty": c["min_difficulty"],
            "schedule_type": c["schedule_type"],
            "schedule_config": dict(c.get("schedule_config", {})),
        }
        self.custom_get_difficulty = None
        st, sc = self.state["schedule_type"], self.state["schedule_config"]
        if st == "fixed_discrete":
            assert len(sc["difficulty"]) == len(sc["max_step"]) + 1, "fixed_discrete: len(difficulty) = len(max_step)+1"
        elif st in ("fixed_root", "fixed_linear"):
            assert "total_curriculum_step" in sc and "difficulty_step" in sc
            if st == "fixed_root":
                assert "root_degree" in sc
        elif st != "custom":
            raise ValueError(f"unknown curriculum schedule {st}")

    def get_current_difficulty(self):
        return self.state["current_difficulty"]

    def set_current_difficulty(self, d):
        self.state["current_difficulty"] = d

    def set_custom_get_difficulty(self, fn):
        self.custom_get_difficulty = fn

    def get_state(self):
        return dict(self.state)

    def set_state(self, state):
        self.state = dict(state)

    def _fixed_root(self, global_step, degree):
        sc = self.state["schedule_config"]
        lo, hi = self.state["min_difficulty"], self.state["max_difficulty"]
        frac = (float(global_step) / sc["total_curriculum_step"]) ** (1.0 / degree)
        d = math.floor(frac * (hi - lo) + lo)
        d -= d % sc["difficulty_step"]
        return min(max(d, lo), hi)

    def get_difficulty(self, global_step):
        st, sc = self.state["schedule_type"], self.state["schedule_config"]
        if st == "fixed_discrete":
            for d, s in zip(sc["difficulty"], sc["max_step"]):
                if global_step <= s:
                    return d
            return sc["difficulty"][-1]
        if st == "fixed_linear":
            return self._fixed_root(global_step, 1)
        if st == "fixed_root":
            return self._fixed_root(global_step, sc["root_degree"])
        assert self.custom_get_difficulty is not None, "custom schedule needs set_custom_get_difficulty"
        return self.custom_get_difficulty(global_step)

    def update_difficulty(self, global_step):
        if self.state["current_difficulty"] < self.state["max_difficulty"]:
            self.state["current_difficulty"] = self.get_difficulty(global_step)
        return self.state["current_difficulty"]
