"""Symmetric-memory collectives (comm/symmetric.py, csrc/kernels/symm_comm.hip) at world 2 on one MI355X.

Both ranks run on the test box's one GPU: each allocates its uncached buffer, the IPC handles are exchanged over
gloo, and every collective is a single kernel per rank that signals / polls the peer's flags. Results must equal
the sum / concatenation computed locally from the seeded inputs of both ranks (fp32 accumulation in rank order, so
the bf16 result is compared against the same rounding). Also covers the parity reuse (many back-to-back calls on
one stream with alternating sizes) and that no wait timed out (error word)."""
import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu


def _inputs(rank, n, dtype, salt):
    g = torch.Generator().manual_seed(1000 * salt + rank)
    return torch.randn(n, generator=g).to(dtype)


def _run(rank, world):
    from hcache_deepspeed_amd.comm.symmetric import SymmetricMemory
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    sm = SymmetricMemory(None, cap_bytes=4 << 20)
    salt = 0
    for dtype in (torch.float32, torch.bfloat16):
        for n in (8, 4096, 8 * 1000, 512 * 1024):
            salt += 1
            x = _inputs(rank, n, dtype, salt).to(dev)
            ref = sum(_inputs(r, n, dtype, salt).float() for r in range(world)).to(dtype)
            out = sm.all_reduce(x.clone())
            torch.testing.assert_close(out.cpu(), ref, atol=0, rtol=0)
    # back-to-back all-reduces of changing sizes on one stream (both parities reused many times)
    xs = [_inputs(rank, 64 * (1 + i % 5), torch.float32, 100 + i).to(dev) for i in range(40)]
    outs = [sm.all_reduce(x, out=torch.empty_like(x)) for x in xs]
    for i, o in enumerate(outs):
        ref = sum(_inputs(r, 64 * (1 + i % 5), torch.float32, 100 + i) for r in range(world))
        torch.testing.assert_close(o.cpu(), ref, atol=0, rtol=0)
    # all-gather (bytes) and reduce-scatter
    for dtype, n in ((torch.bfloat16, 4096), (torch.float32, 40000)):
        salt += 1
        x = _inputs(rank, n, dtype, salt).to(dev)
        out = torch.empty(world * n, dtype=dtype, device=dev)
        sm.all_gather_into_tensor(out, x)
        ref = torch.cat([_inputs(r, n, dtype, salt) for r in range(world)])
        assert torch.equal(out.cpu(), ref)
        salt += 1
        full = _inputs(rank, world * n, dtype, salt).to(dev)
        rs = torch.empty(n, dtype=dtype, device=dev)
        sm.reduce_scatter_tensor(rs, full)
        ref = sum(_inputs(r, world * n, dtype, salt).float() for r in range(world))[rank * n:(rank + 1) * n]
        torch.testing.assert_close(rs.cpu(), ref.to(dtype), atol=0, rtol=0)
    torch.cuda.synchronize()
    assert sm.error() == 0
    assert sm.calls["all_reduce"] == 48 and sm.calls["all_gather"] == 2 and sm.calls["reduce_scatter"] == 2
    sm.close()


def test_symmetric_collectives_world2_gpu():
    run_distributed(_run, 2, timeout=240)


def _run_skip(rank, world):
    """Rank 1 skips one TP all-reduce. Collectives pair by order (as with RCCL), so the ranks run shifted by one
    until rank 0's extra call finds no partner and times out: rank 0's next call raises SymmetricMemoryError, and
    rank 1 -- whose next exchange has no partner any more -- raises within two more calls. Nothing hangs, and
    afterwards the group runs on torch.distributed with correct sums."""
    import time
    from hcache_deepspeed_amd.comm import symmetric
    from hcache_deepspeed_amd.comm.symmetric import SymmetricMemoryError
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x = torch.ones(1024, device=dev)
    for _ in range(3):
        y = symmetric.small_all_reduce(x.clone(), None, max_kb=64)
        torch.cuda.synchronize()
        assert torch.equal(y, torch.full_like(x, world))
    t0 = time.time()
    for i in range(4):
        if rank == 1 and i == 0:
            continue  # the skipped collective
        symmetric.small_all_reduce(x.clone(), None, max_kb=64)
        torch.cuda.synchronize()  # rank 0's last call times out here (bounded wait)
    torch.distributed.barrier()
    raised_at = None
    for i in range(3):
        try:
            symmetric.small_all_reduce(x.clone(), None, max_kb=64)
            torch.cuda.synchronize()
        except SymmetricMemoryError:
            raised_at = i
            break
    assert raised_at is not None, "no SymmetricMemoryError after a skipped collective"
    assert raised_at == 0 or rank == 1, (rank, raised_at)
    assert time.time() - t0 < 180
    torch.distributed.barrier()
    y = symmetric.small_all_reduce(x.clone(), None, max_kb=64)  # broken group: torch.distributed now
    torch.cuda.synchronize()
    assert torch.equal(y, torch.full_like(x, world))


def test_symmetric_skipped_collective_raises_world2_gpu():
    run_distributed(_run_skip, 2, timeout=240)
