"""Autotuner: search ZeRO stage x micro-batch size for the best measured throughput.

Reference parity: autotuning/autotuner.py (``Autotuner`` :42: ``tune`` :404 over ZeRO-0/1/2/3 tuning spaces,
``_generate_experiments`` :304, memory-based pruning ``get_instantiation_memory_required_per_gpu`` :278,
micro-batch search ``run_tuning_micro_batch_sizes`` :741 with plateau early-stop, ``write_optimal_config``
:1075, ``run_after_tuning`` :1103) and the engine's exit hook that writes the measured metric
(engine.py:2458-2480). Each experiment is a real short run of the user's script (launched through this
package's per-node launcher) with ``autotuning.enabled`` in its config; the engine measures steps
[start_profile_step, end_profile_step], writes ``{throughput, latency}`` to ``metric_path`` and exits.
Experiments whose model states cannot fit the GPU (mem_estimators) are skipped without being launched.

After the stage x micro-batch sweep, the best stage's ZeRO knobs (bucket sizes, overlap, ZeRO-3 prefetch /
persistence / MI355X prefetch depth -- ``DEFAULT_TUNING_SPACES`` or the user's ``autotuning.tuning_space``) are
searched at the chosen micro-batch by a tuner (reference autotuning/tuner/: ``gridsearch``, ``random``,
``model_based``) under ``tuner_num_trials`` / ``tuner_early_stopping``.
"""
import copy
import json
import os
import subprocess
import sys
import time

from ..runtime.zero.mem_estimators import estimate
from ..utils.logging import logger

DEFAULT_STAGES = (0, 1, 2, 3)

# knobs per ZeRO stage searched after the micro-batch sweep (sizes tuned for xGMI: bigger buckets, fewer calls)
DEFAULT_TUNING_SPACES = {
    1: {"zero_optimization": {"reduce_bucket_size": [int(5e7), int(2.5e8), int(5e8)],
                              "allgather_bucket_size": [int(5e7), int(5e8)]}},
    2: {"zero_optimization": {"reduce_bucket_size": [int(5e7), int(2.5e8), int(5e8)],
                              "allgather_bucket_size": [int(5e7), int(5e8)], "overlap_comm": [True, False]}},
    3: {"zero_optimization": {"reduce_bucket_size": [int(5e7), int(5e8)],
                              "stage3_prefetch_bucket_size": [int(5e7), int(2e8)],
                              "stage3_param_persistence_threshold": [int(1e4), int(1e6)]},
        "mi355x": {"zero3_prefetch_depth": [1, 2, 3]}},
}


class Autotuner:

    def __init__(self, args, active_resources):
        self.args = args
        self.active_resources = active_resources
        self.user_config = self._get_user_config(list(args.user_args))
        at = dict(self.user_config.get("autotuning", {}))
        self.at = at
        self.results_dir = at.get("results_dir", "autotuning_results")
        self.exps_dir = at.get("exps_dir", "autotuning_exps")
        os.makedirs(self.results_dir, exist_ok=True)
        os.makedirs(self.exps_dir, exist_ok=True)
        self.metric_name = at.get("metric", "throughput")
        self.start_step = int(at.get("start_profile_step", 3))
        self.end_step = int(at.get("end_profile_step", 5))
        self.max_mbs = int(at.get("max_train_micro_batch_size_per_gpu", 64))
        self.min_mbs = int(at.get("min_train_micro_batch_size_per_gpu", 1))
        self.num_mbs = int(at.get("num_tuning_micro_batch_sizes", 3))
        self.stages = tuple(at.get("zero_stages", DEFAULT_STAGES))
        self.model_params = int(at.get("model_num_params", 0))
        self.largest_layer = int(at.get("model_largest_layer_params", 0))
        self.gpu_mem = float(at.get("gpu_memory_gb", 288)) * 2**30
        self.n_gpus = sum(len(v) if isinstance(v, (list, tuple)) else int(v) for v in active_resources.values())
        self.records = {}
        self.optimal = None

    # ------------------------------------------------------------------------------------
    def _get_user_config(self, user_args):
        for i, a in enumerate(user_args):
            if a == "--deepspeed_config" and i + 1 < len(user_args):
                with open(user_args[i + 1]) as f:
                    self.config_path = user_args[i + 1]
                    return json.load(f)
            if a.startswith("--deepspeed_config="):
                path = a.split("=", 1)[1]
                self.config_path = path
                with open(path) as f:
                    return json.load(f)
        raise ValueError("autotuning needs --deepspeed_config <json> in the user arguments")

    def _fits(self, stage):
        if not self.model_params:
            return True
        gpu, _ = estimate(self.model_params, stage, self.n_gpus, self.largest_layer)
        return gpu < 0.8 * self.gpu_mem

    def _tuning_mbs(self):
        out, m = [], self.min_mbs
        while m <= self.max_mbs and len(out) < self.num_mbs:
            out.append(m)
            m *= 2
        return out

    def _generate_experiments(self):
        exps = []
        for stage in self.stages:
            if not self._fits(stage):
                logger.info(f"autotuning: skip ZeRO-{stage} (model states exceed GPU memory)")
                continue
            for mbs in self._tuning_mbs():
                cfg = copy.deepcopy(self.user_config)
                cfg.pop("train_batch_size", None)
                cfg["train_micro_batch_size_per_gpu"] = mbs
                cfg.setdefault("gradient_accumulation_steps", 1)
                cfg.setdefault("zero_optimization", {})["stage"] = stage
                name = f"z{stage}_mbs{mbs}"
                cfg["autotuning"] = {"enabled": True, "start_profile_step": self.start_step,
                                     "end_profile_step": self.end_step,
                                     "metric_path": os.path.abspath(os.path.join(self.exps_dir, name + ".metric.json"))}
                exps.append((name, stage, mbs, cfg))
        return exps

    def run_ds_config(self, ds_config, exp_name):
        path = os.path.join(self.exps_dir, exp_name + ".json")
        with open(path, "w") as f:
            json.dump(ds_config, f)
        user_args = list(self.args.user_args)
        for i, a in enumerate(user_args):
            if a == "--deepspeed_config":
                user_args[i + 1] = path
            elif a.startswith("--deepspeed_config="):
                user_args[i] = f"--deepspeed_config={path}"
        from ..launcher.runner import build_local_cmd, encode_world_info
        a = copy.copy(self.args)
        a.user_args = user_args
        cmd = build_local_cmd(a, encode_world_info(self.active_resources))
        env = dict(os.environ, HDS_AUTOTUNING_EXIT="1")
        t0 = time.time()
        rc = subprocess.call(cmd, env=env, timeout=int(self.at.get("exp_timeout_s", 1800)))
        metric_path = ds_config["autotuning"]["metric_path"]
        if rc != 0 or not os.path.exists(metric_path):
            logger.info(f"autotuning: {exp_name} failed (rc={rc})")
            return None
        with open(metric_path) as f:
            m = json.load(f)
        m["wall_s"] = time.time() - t0
        return m

    def tune(self):
        best = self._tune_stage_mbs()
        if best is not None and self.at.get("tuner_type", "gridsearch") != "none":
            self._tune_space(best)
        return self.optimal

    def _tune_space(self, best):
        from .tuner import GridSearchTuner, ModelBasedTuner, RandomTuner
        from .tuner.utils import gen_combinations, merge_dicts
        base_cfg = best[2]
        stage = base_cfg.get("zero_optimization", {}).get("stage", 0)
        space = self.at.get("tuning_space", DEFAULT_TUNING_SPACES.get(stage))
        if not space:
            return
        exps = []
        for i, knobs in enumerate(gen_combinations(space)):
            cfg = merge_dicts(copy.deepcopy(base_cfg), knobs)
            name = f"{best[1]}_t{i}"
            cfg["autotuning"] = dict(base_cfg["autotuning"],
                                     metric_path=os.path.abspath(os.path.join(self.exps_dir, name + ".metric.json")))
            exps.append({"name": name, "ds_config": cfg, "knobs": knobs})
        kind = self.at.get("tuner_type", "gridsearch")
        cls = {"gridsearch": GridSearchTuner, "random": RandomTuner, "model_based": ModelBasedTuner}[kind]

        def run(exp):
            m = self.run_ds_config(exp["ds_config"], exp["name"])
            self.records[exp["name"]] = {"knobs": exp["knobs"], "metric": m}
            return m

        kw = {"tuning_space": space} if kind == "model_based" else {}
        tuner = cls(exps, run, self.metric_name, **kw)
        tuner.tune(sample_size=1, n_trials=int(self.at.get("tuner_num_trials", 50)),
                   early_stopping=self.at.get("tuner_early_stopping", 5))
        if tuner.best_exp is not None and tuner.best_metric_val > self.optimal[0]:
            self.optimal = (tuner.best_metric_val, tuner.best_exp["name"], tuner.best_exp["ds_config"])

    def _tune_stage_mbs(self):
        best = None
        for name, stage, mbs, cfg in self._generate_experiments():
            m = self.run_ds_config(cfg, name)
            self.records[name] = {"stage": stage, "mbs": mbs, "metric": m}
            if m is None:
                break_mbs = True
                continue
            val = m.get(self.metric_name, 0.0)
            if self.metric_name == "latency":
                val = -val
            if best is None or val > best[0]:
                best = (val, name, cfg)
        if best is not None:
            self.optimal = best
        return self.optimal

    def print_tuning_results(self):
        for name, r in self.records.items():
            m = r["metric"]
            logger.info(f"{name}: {'failed' if m is None else json.dumps(m)}")
        if self.optimal:
            logger.info(f"best: {self.optimal[1]} ({self.metric_name}={abs(self.optimal[0]):.2f})")

    def write_optimal_config(self):
        if not self.optimal:
            return None
        cfg = copy.deepcopy(self.optimal[2])
        cfg.pop("autotuning", None)
        path = os.path.join(self.results_dir, "ds_config_optimal.json")
        with open(path, "w") as f:
            json.dump(cfg, f, indent=2)
        with open(os.path.join(self.results_dir, "summary.json"), "w") as f:
            json.dump(self.records, f, indent=2, default=str)
        return path

    def run_after_tuning(self):
        path = self.write_optimal_config()
        if path is None:
            return 1
        user_args = [(path if prev == "--deepspeed_config" else a)
                     for prev, a in zip([None] + list(self.args.user_args), self.args.user_args)]
        cmd = [sys.executable, "-u", self.args.user_script] + user_args
        return subprocess.call(cmd)
