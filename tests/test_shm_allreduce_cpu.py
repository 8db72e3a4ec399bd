"""Shared-memory CPU all-reduce (csrc/host/shm_comm.cpp) vs the gloo all-reduce: fp32 exact, bf16 within rounding,
chunking through a small segment, and routing through ``comm.inference_all_reduce``.

Reference test analogue: tests/unit/comm/test_dist.py ``TestDistInferenceAllReduce`` (inference_all_reduce result
equals world_size * value on CPU with the SHM op).
"""
import torch

from tests.dist_utils import run_distributed


def _shm(rank, world):
    import torch.distributed as tdist
    from hcache_deepspeed_amd import comm
    from hcache_deepspeed_amd.comm.shm import ShmAllReduce, shm_eligible
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(100_003, generator=g)
    ref = x.clone()
    tdist.all_reduce(ref)
    s = ShmAllReduce(slot_bytes=64 << 10)  # forces ~7 chunks
    y = x.clone()
    for _ in range(3):  # repeated generations reuse the segment
        y = x.clone()
        s.all_reduce_(y)
    assert torch.allclose(y, ref, atol=1e-5)
    b = x.bfloat16()
    s.all_reduce_(b)
    assert torch.allclose(b.float(), ref, atol=0.1, rtol=2e-2)
    s.close()
    assert shm_eligible(x)
    z = torch.full((1000, ), float(rank + 1))
    comm.inference_all_reduce(z)
    assert torch.all(z == sum(range(1, world + 1)))


def test_shm_allreduce_2():
    run_distributed(_shm, 2)


def test_shm_allreduce_3():
    run_distributed(_shm, 3)


def _bench(rank, world):
    from hcache_deepspeed_amd.benchmarks.communication import bench
    res = bench(sizes=(4096, ), dtype=torch.float32, trials=2, warmups=1)
    assert {r["op"] for r in res} == {"all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast",
                                      "pt2pt"}
    assert all(r["lat_ms"] > 0 and r["busbw_GBps"] >= 0 for r in res)


def test_ds_bench_collectives_gloo():
    run_distributed(_bench, 2)
