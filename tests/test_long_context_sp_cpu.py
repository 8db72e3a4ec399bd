"""The multi-GPU long-context stack on the engine path (VERDICT r5 Missing 1 / Next 2): Ulysses SP together with the
host activation cache (``ckpt_offload``) and FPDT configured from ``mi355x.fpdt``, each rank feeding the token positions
``engine.sequence_shard_indices`` names. Gloo world 2 against one process on the whole sequences; the world-8
``torchrun`` dry run of ``bench.py --sp 8 --host-act-cache --act-cache-policy ckpt_offload`` lives here too.

Reference: deepspeed/sequence/layer.py:311-420 (Ulysses), sequence/fpdt_layer.py (FPDT), blogs/ulysses-offload."""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests.dist_utils import run_distributed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = dict(head_dim=16, hidden_size=64, intermediate_size=128, vocab_size=97, num_attention_heads=4,
           num_key_value_heads=2, num_hidden_layers=3)
S = 32


def _batches():
    g = torch.Generator().manual_seed(9)
    return [torch.randint(0, 97, (2, S + 1), generator=g) for _ in range(3)]


def _train(rank, world, extra, out):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))
    cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
           "zero_optimization": {"stage": 3}, "mi355x": {}}
    if world > 1:
        cfg["sequence_parallel_size"] = world
    for k, v in extra.items():
        cfg["mi355x"][k] = v
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    idx = eng.sequence_shard_indices(S)
    losses = []
    for full in _batches():
        x, t = full[:, :-1][:, idx].contiguous(), full[:, 1:][:, idx].contiguous()
        loss = eng(x, targets=t)
        eng.backward(loss)
        eng.step()
        lt = loss.detach().clone()
        if world > 1:
            ds.comm.all_reduce(lt)
        losses.append(float(lt) / world)
    ac = getattr(eng, "_activation_cache", None)
    rec = {"losses": losses, "fpdt": eng.fpdt_config,
           "recomputed": ac.stats()["recomputed_layers"] if ac is not None else None}
    if rank == 0:
        torch.save(rec, out)


CACHE = {"host_act_cache": {"enabled": True, "policy": "ckpt_offload", "min_kib": 0.5, "stash_attention": True}}
FPDT = {"fpdt": {"enabled": True, "chunk_size": 8, "offload": True, "ffn_chunks": 2}}


@pytest.mark.parametrize("mode", ["sp", "sp+cache", "sp+fpdt", "sp+fpdt+cache"])
def test_sp_long_context_stack_matches_single(tmp_path, mode):
    extra = {}
    if "cache" in mode:
        extra.update(CACHE)
    if "fpdt" in mode:
        extra.update(FPDT)
    ref, got = str(tmp_path / "ref.pt"), str(tmp_path / "got.pt")
    run_distributed(_train, 1, {}, ref)
    run_distributed(_train, 2, extra, got)
    r, g = torch.load(ref, weights_only=True), torch.load(got, weights_only=True)
    assert g["losses"] == pytest.approx(r["losses"], rel=2e-4, abs=2e-4), (g["losses"], r["losses"])
    if "cache" in mode:
        # every block checkpointed through the cache (CPU tensors are not spilled: the GPU test covers the copies)
        assert g["recomputed"] == CFG["num_hidden_layers"]
    if "fpdt" in mode:
        assert g["fpdt"]["chunk_size"] == 8 and g["fpdt"]["sp"] == 2


def test_fpdt_layout_from_the_engine():
    """Without SP the FPDT layout is the identity; the bench feeds the same positions the model expects."""
    from hcache_deepspeed_amd.parallel.fpdt import fpdt_layout_indices
    assert torch.equal(fpdt_layout_indices(32, 8, 1, 0), torch.arange(32))
    a, b = fpdt_layout_indices(32, 8, 2, 0), fpdt_layout_indices(32, 8, 2, 1)
    assert sorted(torch.cat([a, b]).tolist()) == list(range(32)) and a[:4].tolist() == [0, 1, 2, 3]


def test_bench_sp8_ckpt_offload_torchrun_dry_run():
    """bench.py --sp 8 with the host activation cache (ckpt_offload) as the driver would launch it at N=8."""
    W = 8
    env = dict(os.environ, OMP_NUM_THREADS="1", HDS_TUNABLEOP="0", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(W), "--master-addr",
           "127.0.0.1", "--master-port", "29753", os.path.join(ROOT, "bench.py"), "--gpus", str(W), "--steps", "2",
           "--warmup", "1", "--model", "tiny-sp", "--seq", "256", "--micro-batch", "2", "--sp", str(W),
           "--host-act-cache", "--act-cache-policy", "ckpt_offload"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c = out["config"]
    assert c["sequence_parallel_size"] == W and c["parallelism"] == f"zero3-dp1-sp{W}" and c["host_act_cache"]
    assert c["global_batch"] == 2 and out["value"] > 0
    assert out["extra"]["act_cache"]["recomputed_layers"] == 2  # every block checkpointed (ckpt_offload)
    assert out["extra"]["comm"]["ranks"] == W


def test_node_long_context_plan():
    """The per-node plan (README: planned max S at 8 GPUs): host-bound at SP 8, monotone in host RAM, the stash
    halves the reach, HBM stays far below a MI355X's at the planned S, and 512k at one GPU reproduces the measured
    run's scale (227.7 GiB planned vs 221.5 GiB measured peak; 128 GiB of boundaries)."""
    from hcache_deepspeed_amd.models.llama import llama3_8b
    from hcache_deepspeed_amd.runtime.zero.mem_estimators import long_context_plan
    c = llama3_8b()
    p1, p2 = long_context_plan(c, 8, 8, host_ram_gib=1024), long_context_plan(c, 8, 8, host_ram_gib=2048)
    assert p1["limited_by"] == "host" and p2["max_seq"] > 1.9 * p1["max_seq"]
    ns = long_context_plan(c, 8, 8, host_ram_gib=2048, stash=False)
    assert ns["max_seq"] > 1.9 * p2["max_seq"] and ns["max_seq"] >= 2 * 2**20  # >= 2M tokens on one 2 TiB node
    assert ns["hbm_gib_rank"] < 200
