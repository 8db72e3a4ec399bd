"""Failure-symmetric communicator setup (comm/setup.py) and the startup transport selection's handling of a transport
that fails on ONE rank (runtime/zero/transport.py): every rank reaches the same collectives, drops the transport
together, and nothing hangs (VERDICT r5 "Next round" item 4). Gloo, world 4."""
import pytest
import torch

from tests.dist_utils import run_distributed


def _setup_phases(rank, world):
    import torch.distributed as dist

    from hcache_deepspeed_amd.comm.setup import CollectiveSetupError, collective_setup
    cleaned = []

    def cleanup(state, fin):
        cleaned.append((state, fin))

    # all ranks fine: payloads exchanged in rank order
    st, fin = collective_setup(None, lambda: (rank * 10, f"h{rank}"), lambda s, p: (s, p), cleanup)
    assert st == rank * 10 and fin == (rank * 10, [f"h{r}" for r in range(world)]) and not cleaned

    # local failure on rank 2: every rank raises (and names rank 2); ranks that succeeded locally clean up
    def local():
        if rank == 2:
            raise MemoryError("1 GiB symmetric buffer: out of memory")
        return "buf", "handle"

    with pytest.raises(CollectiveSetupError, match="rank\\(s\\) 2"):
        collective_setup(None, local, lambda s, p: None, cleanup)
    assert cleaned == ([] if rank == 2 else [("buf", None)])
    cleaned.clear()

    # exchange (finish) failure on rank 1: every rank raises after the second agreement; every rank cleans up
    def finish(s, payloads):
        if rank == 1:
            raise RuntimeError("open peer handle failed")
        return "opened"

    with pytest.raises(CollectiveSetupError, match="exchange failed on rank\\(s\\) 1"):
        collective_setup(None, lambda: ("buf", None), finish, cleanup)
    assert cleaned == [("buf", None if rank == 1 else "opened")]
    dist.barrier()  # the group is still in lock-step


class _GoodComm:
    """A working third transport over the torch.distributed facade (gloo here)."""

    def __init__(self, group):
        self.group = group

    def all_gather_into_tensor(self, out, inp):
        from hcache_deepspeed_amd import comm
        comm.all_gather_into_tensor(out, inp, group=self.group)

    def reduce_scatter_tensor(self, out, inp):
        from hcache_deepspeed_amd import comm
        comm.reduce_scatter_tensor(out, inp, group=self.group)

    def close(self):
        pass


def _faulty_factory(kind, group, max_bytes, device):
    import torch.distributed as dist

    from hcache_deepspeed_amd.comm.setup import collective_setup

    def local():
        if dist.get_rank(group) == 1:
            raise MemoryError("injected: symmetric buffer allocation failed on this rank only")
        return None, b"handle"

    collective_setup(group, local, lambda s, p: None, what="faulty transport")
    return _GoodComm(group)


def _good_factory(kind, group, max_bytes, device):
    from hcache_deepspeed_amd.comm.setup import collective_setup
    collective_setup(group, lambda: (None, b"h"), lambda s, p: None, what="good transport")
    return _GoodComm(group)


def _selection(rank, world):
    from hcache_deepspeed_amd.runtime.zero import transport

    class U:  # a unit collective of 4 MiB shards over the world group
        world = 4
        expert_key = None
        ag_group = rs_group = None
        shard = 1 << 20
        padded = 4 << 20

    transport.FACTORIES["faulty"] = _faulty_factory
    transport.FACTORIES["good"] = _good_factory
    try:
        route, comms, table = transport.select_unit_transports(
            [U()], torch.device("cpu"), torch.float32, torch.float32, transports=("rccl", "faulty", "good"), iters=2)
    finally:
        transport.FACTORIES.pop("faulty")
        transport.FACTORIES.pop("good")
    down = [r for r in table if r.get("available") is False]
    # the one-rank failure dropped "faulty" on EVERY rank (rank 1 reports the cause, the others the peer's)
    assert {r["transport"] for r in down} == {"faulty"} and len(down) == 2
    assert "rank(s) 1" in down[0]["why"]
    rows = [r for r in table if "choice" in r]
    assert rows and all(set(r["ms"]) == {"rccl", "good"} for r in rows)
    assert set(route.values()) <= {"rccl", "good"}


def test_collective_setup_is_failure_symmetric():
    run_distributed(_setup_phases, 4, timeout=120)


def test_transport_selection_drops_a_one_rank_failure():
    run_distributed(_selection, 4, timeout=180)


def test_release_transports_closes_auto_state():
    """A forced compile switch first releases what the startup selection installed (communicators destroyed, symmetric
    buffers closed, route cleared) instead of leaking them and leaving symmetric routing on."""
    from hcache_deepspeed_amd.runtime.zero.optimizer import ZeroOptimizer
    calls = []

    class C:
        def destroy(self):
            calls.append("destroy")

        def close(self):
            calls.append("close")

    z = ZeroOptimizer.__new__(ZeroOptimizer)
    z.device = torch.device("cpu")
    z._native, z._symm, z._route = {1: C()}, {("ag", 1): C(), ("rs", 1): C()}, {("ag", 1, 8): "symmetric"}
    assert z.release_transports()
    assert sorted(calls) == ["close", "close", "destroy"]
    assert z._native is None and z._symm == {} and z._route is None
    assert not z.release_transports()  # idempotent
