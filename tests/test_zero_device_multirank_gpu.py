"""The partitioned ZeRO-3 path on real HIP devices at world 2 (both ranks share the one MI355X of the test box).

At dp = 1 every unit is aliased, so ``_gather`` / ``_release`` / ``_after_reduce`` / ``_retire`` and the in-place
reduce-scatter into the gradient shard never run on a GPU in the 1-GPU bench. RCCL refuses two ranks on one
device, so the two processes rendezvous over gloo; collectives on device tensors use gloo directly where it
accepts them and otherwise stage through host memory (``_staged``). Everything else -- flat-buffer kernels,
HIP streams, the events of the comm accounting, the fused Adam on the shard -- is the GPU path.

The world-2 run (micro-batch 2 per rank) must follow the world-1 run (micro-batch 4, same global batch) in loss and
in the final fp32 master weights within bf16 tolerance."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu

CFG = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=3, num_attention_heads=4,
           num_key_value_heads=2, head_dim=64, max_position_embeddings=256)


def _staged(fn_name):
    import hcache_deepspeed_amd.comm as hcomm
    import torch.distributed as tdist
    native = getattr(tdist, fn_name)

    def call(out, inp, *args, group=None, async_op=False, **kw):
        if group is not None and tdist.get_world_size(group) == 1:
            out.copy_(inp.view_as(out))
            return hcomm.comm._Done() if async_op else None
        try:
            w = native(out, inp, *args, group=group, async_op=async_op, **kw)
            return w
        except (RuntimeError, ValueError):
            o = out.detach().cpu()
            native(o, inp.detach().cpu(), *args, group=group, **kw)
            out.copy_(o)
            return hcomm.comm._Done() if async_op else None

    return call


def _run(rank, world, d, steps=3, symmetric=False, stage=3, dtype="bf16", zpp=False):
    import hcache_deepspeed_amd as hds
    import hcache_deepspeed_amd.comm as hcomm
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.utils.tensor_fragment import safe_get_full_fp32_param
    on_gpu = torch.cuda.is_available()
    if on_gpu:
        torch.cuda.set_device(0)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        setattr(hcomm, name, _staged(name))
        setattr(hcomm.comm, name, getattr(hcomm, name))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))  # same full weights on every rank; initialize() partitions them
    mb = 4 // world
    cfg = {"train_micro_batch_size_per_gpu": mb, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": stage},
           "mi355x": {"comm_stats": True}}
    if dtype != "bf16":
        cfg.pop("bf16")
    if dtype == "fp16":
        cfg["fp16"] = {"enabled": True, "loss_scale": 0, "initial_scale_power": 12}
    if zpp:  # ZeRO++: int8 weight all-gather (qwZ) and the quantized gradient all-to-all reduce (qgZ)
        cfg["zero_optimization"].update(zero_quantized_weights=True, zero_quantized_gradients=True)
        from tests.test_moe_device_multirank_gpu import _staged_all_to_all
        hcomm.all_to_all_single = _staged_all_to_all()
        hcomm.comm.all_to_all_single = hcomm.all_to_all_single
    if symmetric:
        cfg["compile"] = {"symmetric_memory": True}
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    if symmetric:
        eng.compile()
        if world > 1 and on_gpu:
            assert getattr(eng.optimizer, "_symm", None), "symmetric-memory collectives not enabled"
    assert eng.device.type == ("cuda" if on_gpu else "cpu")
    z = eng.optimizer
    if world > 1:
        assert z.partitioned and any(z._partitioned(u) for u in z.units)
    g = torch.Generator().manual_seed(7)
    losses = []
    for _ in range(steps):
        ids = torch.randint(0, CFG["vocab_size"], (4, 128), generator=g)
        mine = ids[rank * mb:(rank + 1) * mb].to(eng.device)
        loss = eng(mine, labels=mine)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    if on_gpu:
        torch.cuda.synchronize()
    if world > 1 and stage == 3:
        summ = z.comm_stats.summary()
        assert summ["collectives"]["all_gather"]["count"] > 0
        if not zpp:  # qgZ reduces gradients by all-to-all instead
            assert summ["collectives"]["reduce_scatter"]["count"] > 0
    full = {n: safe_get_full_fp32_param(p).float().cpu() for n, p in eng.module.named_parameters()}
    if symmetric and world > 1 and on_gpu:
        calls = {k: sum(sm.calls[k] for sm in z._symm.values()) for k in ("all_gather", "reduce_scatter")}
        assert calls["all_gather"] > 0 and calls["reduce_scatter"] > 0, calls
        assert all(sm.error() == 0 for sm in z._symm.values())
    ls = torch.tensor(losses)
    torch.distributed.all_reduce(ls)
    if rank == 0:
        tag = ("s" if symmetric else "") + ("" if (stage, dtype) == (3, "bf16") else f"_z{stage}{dtype}") + \
            ("_zpp" if zpp else "")
        torch.save({"losses": (ls / world).tolist(), "weights": full}, os.path.join(d, f"w{world}{tag}.pt"))


def test_zero3_partitioned_device_path_world2_matches_world1(tmp_path):
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d)
    a = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
    b = torch.load(os.path.join(d, "w2.pt"), weights_only=True)
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 2e-2 * abs(la), (a["losses"], b["losses"])
    for n, w in a["weights"].items():
        rel = float((b["weights"][n] - w).norm() / w.norm().clamp_min(1e-12))
        assert rel < 2e-2, (n, rel)


def test_zero3_symmetric_memory_world2_matches_world1(tmp_path):
    """compile.symmetric_memory at world 2 on one MI355X: the unit all-gathers and reduce-scatters run as the
    one-kernel symmetric-memory collectives (IPC-mapped buffers of the other process), and training follows the
    world-1 run like the RCCL/gloo path does."""
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d, 3, True)
    a = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
    b = torch.load(os.path.join(d, "w2s.pt"), weights_only=True)
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 2e-2 * abs(la), (a["losses"], b["losses"])
    for n, w in a["weights"].items():
        rel = float((b["weights"][n] - w).norm() / w.norm().clamp_min(1e-12))
        assert rel < 2e-2, (n, rel)


def _run_skip(rank, world, d):
    """Rank 1 silently skips one symmetric all-gather in step 2: the ranks' epochs desynchronise, rank 0's last
    exchange of the step times out. That step must be skipped on BOTH ranks (weights unchanged) and the next step
    must raise SymmetricMemoryError on both ranks -- within bounded time, never silently wrong weights."""
    import time
    import hcache_deepspeed_amd as hds
    import hcache_deepspeed_amd.comm as hcomm
    from hcache_deepspeed_amd.comm.symmetric import SymmetricMemoryError
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.cuda.set_device(0)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        setattr(hcomm, name, _staged(name))
        setattr(hcomm.comm, name, getattr(hcomm, name))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True}, "gradient_clipping": 1.0,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3},
           "compile": {"symmetric_memory": True}}
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    eng.compile()
    z = eng.optimizer
    assert z._symm
    g = torch.Generator().manual_seed(7)

    def batch():
        ids = torch.randint(0, CFG["vocab_size"], (4, 128), generator=g)
        return ids[rank * 2:(rank + 1) * 2].to(eng.device)

    def train_step():
        x = batch()
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()

    train_step()
    torch.cuda.synchronize()
    before = z.store.master.detach().clone()
    if rank == 1:
        orig, n = z._symm_issue, [0]

        def skipping(kind, group, nbytes, fn):
            if kind == "ag":
                n[0] += 1
                if n[0] == 2:
                    return hcomm.comm._Done()  # "forgot" this collective: no kernel, no epoch
            return orig(kind, group, nbytes, fn)

        z._symm_issue = skipping
    train_step()  # the desynchronised step
    torch.cuda.synchronize()
    if rank == 1:
        z._symm_issue = orig
    assert torch.equal(z.store.master, before), "a step with a timed-out symmetric collective updated the weights"
    t0 = time.time()
    raised = False
    try:
        train_step()
    except SymmetricMemoryError:
        raised = True
    assert raised, "no SymmetricMemoryError after a timed-out collective"
    assert time.time() - t0 < 120
    assert not z._symm  # fell back to RCCL for the unit collectives
    torch.save({"ok": True}, os.path.join(d, f"skip{rank}.pt"))


def test_zero3_symmetric_memory_skipped_collective_fails_loudly(tmp_path):
    d = str(tmp_path)
    run_distributed(_run_skip, 2, d, timeout=300)
    for r in range(2):
        assert torch.load(os.path.join(d, f"skip{r}.pt"), weights_only=True)["ok"]


@pytest.mark.parametrize("stage,dtype", [(1, "bf16"), (2, "bf16"), (2, "fp32"), (3, "fp16"), (1, "fp16")])
def test_zero12_device_path_world2_matches_world1(tmp_path, stage, dtype):
    """ZeRO-1 / ZeRO-2 (flat reduce-scatter of the gradients, sharded optimizer states, all-gather of the updated
    parameters) on device tensors at world 2; fp32 training (the compute copy is the master's dtype) and fp16 with
    dynamic loss scaling (fp16 compute copy refreshed from the fp32 master)."""
    d = str(tmp_path)
    run_distributed(_run, 1, d, 3, False, stage, dtype)
    run_distributed(_run, 2, d, 3, False, stage, dtype)
    a = torch.load(os.path.join(d, f"w1_z{stage}{dtype}.pt"), weights_only=True)
    b = torch.load(os.path.join(d, f"w2_z{stage}{dtype}.pt"), weights_only=True)
    tol = 2e-3 if dtype == "fp32" else 2e-2
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= tol * abs(la), (a["losses"], b["losses"])
    for n, w in a["weights"].items():
        rel = float((b["weights"][n] - w).norm() / w.norm().clamp_min(1e-12))
        assert rel < tol, (n, rel)


def test_zeropp_quantized_device_path_world2_follows_world1(tmp_path):
    """ZeRO++ qwZ + qgZ at world 2 on device tensors: the int8 quantize / dequantize kernels in the weight gather and
    the gradient all-to-all reduce run on the GPU; training follows plain world-1 ZeRO-3 within quantization noise."""
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d, 3, False, 3, "bf16", True)
    a = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
    b = torch.load(os.path.join(d, "w2_zpp.pt"), weights_only=True)
    for la, lb in zip(a["losses"], b["losses"]):
        assert abs(la - lb) <= 5e-2 * abs(la), (a["losses"], b["losses"])
    for n, w in a["weights"].items():
        rel = float((b["weights"][n] - w).norm() / w.norm().clamp_min(1e-12))
        assert rel < 5e-2, (n, rel)
