"""Startup transport selection of the ZeRO-3 unit collectives (runtime/zero/transport.py) on the device path: two
ranks share the one MI355X of the test box (gloo rendezvous; torch.distributed collectives on device tensors staged
through host memory as in test_zero_device_multirank_gpu.py).

* the engine measures every unit all-gather / reduce-scatter size class at initialization: rccl (here gloo) and
  symmetric memory are timed, the native RCCL communicator drops out with its reason (two ranks on one GPU);
* with a stub timer whose numbers differ per rank, the choice follows the MAX over ranks (a collective is paced by
  its slowest rank) and is identical on both ranks; the routed collectives reproduce the reference results."""
import pytest
import torch

from tests.dist_utils import run_distributed
from tests.test_zero_device_multirank_gpu import CFG, _staged

pytestmark = pytest.mark.gpu


class _StubTimer:
    """Per-rank fake milliseconds: the transport decision must use the slowest rank's number."""

    def __init__(self, rank, table):
        self.rank, self.table = rank, table

    def run(self, fn, iters, transport=None):
        fn()  # still issued: the peers take part in the same collective
        return self.table[transport][self.rank]


def _run(rank, world):
    import hcache_deepspeed_amd as hds
    import hcache_deepspeed_amd.comm as hcomm
    import torch.distributed as tdist
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    from hcache_deepspeed_amd.runtime.zero import transport as T
    torch.cuda.set_device(0)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor"):
        setattr(hcomm, name, _staged(name))
        setattr(hcomm.comm, name, getattr(hcomm, name))
    torch.manual_seed(0)
    m = LlamaForCausalLM(tiny(**CFG))
    cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3}}
    eng, _, _, _ = hds.initialize(model=m, config=cfg)
    z = eng.optimizer
    sel = z.comm_selection
    rows = [r for r in sel if "choice" in r]
    assert {r["kind"] for r in rows} == {"ag", "rs"}, sel
    for r in rows:
        assert r["ms"]["rccl"] > 0 and r["ms"].get("symmetric") is not None and r["world"] == 2, r
    nat = [r for r in sel if r.get("transport") == "native"]
    assert nat and nat[0]["available"] is False and "one GPU" in nat[0]["why"], sel
    # the same choice on both ranks
    mine = [(r["kind"], r["msg_mib"], r["choice"]) for r in rows]
    both = [None, None]
    tdist.all_gather_object(both, mine)
    assert both[0] == both[1]
    # stub timing: rank 1 is slow on symmetric for all-gathers -> rccl wins them; reduce-scatters pick symmetric
    for kind, expect in (("ag", "rccl"), ("rs", "symmetric")):
        stub = _StubTimer(rank, {"rccl": [3.0, 3.0], "symmetric": [1.0, 5.0] if kind == "ag" else [1.0, 2.0]})
        units = [u for u in z.units]
        route, comms, table = T.select_unit_transports(units, z.device, z.dtype, z.comm_dtype,
                                                       transports=("rccl", "symmetric"), timer=stub)
        got = {k[2]: v for k, v in route.items() if k[0] == kind}
        assert got and set(got.values()) == {expect}, (kind, got, table)
        for c in comms.values():
            c.close()
    # a few routed training steps run and stay finite
    g = torch.Generator(device="cuda").manual_seed(7 + rank)
    for _ in range(2):
        b = torch.randint(0, CFG["vocab_size"], (2, 64), device="cuda", generator=g)
        loss = eng(b, labels=b)
        eng.backward(loss)
        eng.step()
        assert torch.isfinite(loss)
    ev = z.unit_events.summary()
    assert ev["backward_fetch_wait"]["count"] > 0
    tdist.barrier()


def test_transport_selection_world2_gpu():
    run_distributed(_run, 2, timeout=300)
