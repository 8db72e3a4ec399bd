"""Curriculum learning difficulty schedules.

Reference parity: runtime/data_pipeline/curriculum_scheduler.py (``CurriculumScheduler`` :11): schedule types
``fixed_discrete`` (step thresholds -> difficulties), ``fixed_root`` (difficulty grows as
(step / total)^(1/root_degree), rounded down to ``difficulty_step``), ``fixed_linear`` (root 1) and
``custom`` (user function); ``update_difficulty`` is monotone and stops at ``max_difficulty``. The engine
uses the difficulty as ``curriculum_seqlen`` (sequence-length curriculum, the common metric).
"""
import math


class CurriculumScheduler:

    def __init__(self, config):
        for key in ("min_difficulty", "max_difficulty", "schedule_type"):
            assert key in config, f"Curriculum learning requires the config '{key}'"
        self.state = {"min_difficulty": config["min_difficulty"], "max_difficulty": config["max_difficulty"],
                      "current_difficulty": config["min_difficulty"], "schedule_type": config["schedule_type"]}
        st = config["schedule_type"]
        sc = config.get("schedule_config", {})
        if st == "fixed_discrete":
            assert len(sc.get("difficulty", [])) == len(sc.get("max_step", [])) + 1 and sc["max_step"], \
                "fixed_discrete needs difficulty (n+1 values) and max_step (n values)"
        elif st in ("fixed_root", "fixed_linear"):
            assert "total_curriculum_step" in sc and "difficulty_step" in sc, \
                f"{st} needs total_curriculum_step and difficulty_step"
            if st == "fixed_root":
                assert "root_degree" in sc, "fixed_root needs root_degree"
        elif st == "custom":
            self.custom_get_difficulty = None
        else:
            raise RuntimeError(f"Unsupported curriculum schedule type {st}")
        self.state["schedule_config"] = sc

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

    def _discrete(self, step):
        sc = self.state["schedule_config"]
        for limit, diff in zip(sc["max_step"], sc["difficulty"]):
            if step <= limit:
                return diff
        return sc["difficulty"][-1]

    def _root(self, step, degree):
        sc = self.state["schedule_config"]
        lo, hi = self.state["min_difficulty"], self.state["max_difficulty"]
        frac = (float(step) / sc["total_curriculum_step"])**(1.0 / degree)
        d = math.floor(frac * (hi - lo) + lo)
        d -= d % sc["difficulty_step"]
        return min(d, hi)

    def get_difficulty(self, step):
        st = self.state["schedule_type"]
        if st == "fixed_discrete":
            return self._discrete(step)
        if st == "fixed_linear":
            return self._root(step, 1)
        if st == "fixed_root":
            return self._root(step, self.state["schedule_config"]["root_degree"])
        return self.custom_get_difficulty(step)

    def update_difficulty(self, step):
        if self.state["current_difficulty"] < self.state["max_difficulty"]:
            self.state["current_difficulty"] = self.get_difficulty(step)
        return self.state["current_difficulty"]
