"""Autotuning (reference tests/unit/autotuning/test_autotuning.py strategy: experiment generation + a real tiny run
through the launcher on CPU) and the ZeRO memory estimators."""
import json
import os
import sys

import pytest


def test_mem_estimators_scale_with_stage_and_world():
    from hcache_deepspeed_amd.runtime.zero.mem_estimators import estimate, estimate_zero3_model_states_mem_needs
    P = 8_000_000_000
    g0, _ = estimate(P, 0, 8)
    g1, _ = estimate(P, 1, 8)
    g2, _ = estimate(P, 2, 8)
    g3, _ = estimate(P, 3, 8, 200_000_000)
    assert g0 > g1 > g2 > g3
    g3o, c3o = estimate(P, 3, 8, 200_000_000, offload_optimizer=True, offload_param=True)
    assert g3o < g3 and c3o > 0
    cpu, gpu, largest = estimate_zero3_model_states_mem_needs(P, 200_000_000, 8)
    assert cpu > 0 and gpu > 0


SCRIPT = r'''
import argparse, os, sys, torch
sys.path.insert(0, {root!r})
import hcache_deepspeed_amd as ds
from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
ap = argparse.ArgumentParser(); ap.add_argument("--local_rank", type=int, default=0)
ap.add_argument("--deepspeed_config", required=True); a = ap.parse_args()
torch.manual_seed(0)
m = LlamaForCausalLM(tiny(hidden_size=64, intermediate_size=128, vocab_size=97, num_attention_heads=4,
                          num_key_value_heads=2, head_dim=16, num_hidden_layers=2))
eng, _, _, _ = ds.initialize(model=m, config=a.deepspeed_config)
for _ in range(20):
    x = torch.randint(0, 97, (eng.train_micro_batch_size_per_gpu(), 12))
    loss = eng(x, labels=x); eng.backward(loss); eng.step()
'''


def test_autotuner_end_to_end_cpu(tmp_path, monkeypatch):
    from hcache_deepspeed_amd.autotuning import Autotuner
    from hcache_deepspeed_amd.launcher.runner import parse_args
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "train.py"
    script.write_text(SCRIPT.format(root=root))
    cfg = {"train_micro_batch_size_per_gpu": 1, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
           "autotuning": {"zero_stages": [0, 3], "min_train_micro_batch_size_per_gpu": 1,
                          "num_tuning_micro_batch_sizes": 2, "start_profile_step": 2, "end_profile_step": 4,
                          "results_dir": str(tmp_path / "res"), "exps_dir": str(tmp_path / "exps"),
                          "tuner_type": "model_based", "tuner_num_trials": 2,
                          "tuning_space": {"zero_optimization": {"reduce_bucket_size": [1000000, 10000000]}}}}
    cpath = tmp_path / "ds.json"
    cpath.write_text(json.dumps(cfg))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("PYTHONPATH", root)
    args = parse_args(["--num_gpus", "1", "--hostfile", str(tmp_path / "none"), "--master_port", "29677",
                       str(script), "--deepspeed_config", str(cpath)])
    args.master_addr = "127.0.0.1"
    tuner = Autotuner(args, {"localhost": [0]})
    exps = tuner._generate_experiments()
    assert [e[0] for e in exps] == ["z0_mbs1", "z0_mbs2", "z3_mbs1", "z3_mbs2"]
    best = tuner.tune()
    assert best is not None and all(r["metric"] is not None for r in tuner.records.values())
    assert sum(1 for k in tuner.records if "_t" in k) == 2  # the knob search ran after the stage x mbs sweep
    path = tuner.write_optimal_config()
    opt = json.load(open(path))
    assert "autotuning" not in opt and opt["zero_optimization"]["stage"] in (0, 3)


def _fake_exps():
    from hcache_deepspeed_amd.autotuning.tuner.utils import gen_combinations
    space = {"zero_optimization": {"reduce_bucket_size": [1, 2, 4, 8, 16], "overlap_comm": [True, False]},
             "mi355x": {"zero3_prefetch_depth": [1, 2, 3]}}
    exps = [{"name": f"e{i}", "ds_config": c} for i, c in enumerate(gen_combinations(space))]
    return space, exps


def _fake_metric(exp):
    z = exp["ds_config"]["zero_optimization"]
    d = exp["ds_config"]["mi355x"]["zero3_prefetch_depth"]
    if z["reduce_bucket_size"] == 16 and d == 3:
        return None  # "OOM": a failed experiment
    return {"throughput": 100 - (z["reduce_bucket_size"] - 4) ** 2 - 10 * (d - 2) ** 2 + 5 * z["overlap_comm"],
            "latency": 1.0}


@pytest.mark.parametrize("kind", ["gridsearch", "random", "model_based"])
def test_tuners_find_best_config(kind):
    from hcache_deepspeed_amd.autotuning.tuner import GridSearchTuner, ModelBasedTuner, RandomTuner
    space, exps = _fake_exps()
    assert len(exps) == 30
    calls = []

    def run(exp):
        calls.append(exp["name"])
        return _fake_metric(exp)

    if kind == "gridsearch":
        t = GridSearchTuner(exps, run, "throughput")
    elif kind == "random":
        t = RandomTuner(exps, run, "throughput", seed=1)
    else:
        t = ModelBasedTuner(exps, run, "throughput", tuning_space=space, seed=0)
    n = t.tune(sample_size=1, n_trials=30)
    assert n == 30 and len(set(calls)) == 30  # every config exactly once
    best = t.best_exp["ds_config"]
    assert best["zero_optimization"]["reduce_bucket_size"] == 4 and best["mi355x"]["zero3_prefetch_depth"] == 2
    assert best["zero_optimization"]["overlap_comm"] is True


def test_model_based_tuner_beats_random_order_on_budget():
    from hcache_deepspeed_amd.autotuning.tuner import ModelBasedTuner
    space, exps = _fake_exps()
    hits = 0
    for seed in range(5):
        t = ModelBasedTuner(exps, _fake_metric, "throughput", tuning_space=space, seed=seed)
        t.tune(sample_size=1, n_trials=12)
        hits += t.best_metric_val == 105
    assert hits >= 3  # finds the optimum within 12 of 30 trials most of the time


def test_tuner_early_stopping_and_latency_metric():
    from hcache_deepspeed_amd.autotuning.tuner import GridSearchTuner
    space, exps = _fake_exps()
    t = GridSearchTuner(exps, _fake_metric, "throughput")
    n = t.tune(n_trials=100, early_stopping=3)
    assert n < 30 and n >= t.best_iter + 3
    lt = GridSearchTuner(exps, lambda e: {"latency": e["ds_config"]["zero_optimization"]["reduce_bucket_size"]},
                         "latency")
    lt.tune(n_trials=100)
    assert lt.best_exp["ds_config"]["zero_optimization"]["reduce_bucket_size"] == 1
