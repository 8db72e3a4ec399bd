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
                          "results_dir": str(tmp_path / "res"), "exps_dir": str(tmp_path / "exps")}}
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
    path = tuner.write_optimal_config()
    opt = json.load(open(path))
    assert "autotuning" not in opt and opt["zero_optimization"]["stage"] in (0, 3)
