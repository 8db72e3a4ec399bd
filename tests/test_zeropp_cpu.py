"""ZeRO++ (qwZ quantized weight gather, qgZ quantized gradient all-to-all, hpZ secondary partition) and MiCS
on gloo (reference tests/unit/runtime/zero/test_zeropp.py and test_mics strategies: train a small model with
the feature on and compare with plain ZeRO-3; exact features must match, quantized ones within tolerance)."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_cpu import TINY


def _run(zero_extra, steps=4):
    import hcache_deepspeed_amd as ds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**TINY))
    cfg = {"train_micro_batch_size_per_gpu": 2,
           "optimizer": {"type": "AdamW", "params": {"lr": 3e-3}},
           "zero_optimization": dict({"stage": 3}, **zero_extra), "gradient_clipping": 1.0}
    eng, _, _, _ = ds.initialize(model=m, config=cfg)
    g = torch.Generator().manual_seed(11 + torch.distributed.get_rank())
    losses = []
    for _ in range(steps):
        x = torch.randint(0, 97, (2, 12), generator=g)
        loss = eng(x, labels=x)
        eng.backward(loss)
        eng.step()
        losses.append(float(loss))
    return losses, eng


def _zeropp(rank, world):
    base, _ = _run({})
    hpz, e = _run({"zero_hpz_partition_size": 2})
    assert e.optimizer.hpz == 2
    assert hpz == pytest.approx(base, rel=1e-5, abs=1e-5), (hpz, base)
    mics, e = _run({"mics_shard_size": 2})
    assert e.optimizer.layout_world == 2
    assert mics == pytest.approx(base, rel=1e-4, abs=1e-4), (mics, base)
    for st in (1, 2):
        b, _ = _run({"stage": st})
        mm, _ = _run({"stage": st, "mics_shard_size": 2})
        assert mm == pytest.approx(b, rel=1e-4, abs=1e-4), (st, mm, b)
    qw, e = _run({"zero_quantized_weights": True})
    assert e.optimizer.qwz
    assert qw == pytest.approx(base, rel=2e-2, abs=2e-2), (qw, base)
    qg, e = _run({"zero_quantized_gradients": True})
    assert e.optimizer.qgz
    assert qg == pytest.approx(base, rel=2e-2, abs=2e-2), (qg, base)
    both, _ = _run({"zero_quantized_weights": True, "zero_quantized_gradients": True,
                    "zero_hpz_partition_size": 2})
    assert both == pytest.approx(base, rel=3e-2, abs=3e-2), (both, base)


def test_zeropp_and_mics_world4():
    run_distributed(_zeropp, 4)


def test_quantizer_cpu_roundtrip():
    from hcache_deepspeed_amd.ops import quantizer as Q
    torch.manual_seed(0)
    x = torch.randn(8192)
    for bits in (8, 4):
        for sym in (True, False):
            q, s, m = Q.quantize(x, 512, bits, sym)
            assert q.numel() == x.numel() * bits // 8
            y = Q.dequantize(q, s, m, 512, bits, sym, torch.float32)
            assert (y - x).abs().max() <= s.max() * 0.5 + 1e-6
    q, s = Q.quantize_fp8(x, 512, "e4m3")
    y = Q.dequantize_fp8(q, s, 512, "e4m3", torch.float32)
    assert ((y - x).abs() <= x.abs() * 0.0625 + s.repeat_interleave(512) * 2**-6).all()
    fq = Q.FP_Quantize(group_size=256)
    qq = fq.quantize(x.view(32, 256).to(torch.bfloat16))
    back = fq.dequantize(qq)
    assert back.shape == (32, 256) and (back.float() - x.view(32, 256)).abs().max() < 0.5
    rows = fq.selective_dequantize(qq, torch.tensor([3, 7]))
    assert torch.equal(rows, back[[3, 7]])
    chunks = [Q.quantize(x * (r + 1), 512, 8, True) for r in range(3)]
    red = Q.dequant_reduce(torch.cat([c[0] for c in chunks]), torch.cat([c[1] for c in chunks]), 3, 8192, 512, 8)
    assert (red - 6 * x).abs().max() < 0.2
