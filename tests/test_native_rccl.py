"""Native C++ RCCL executor (csrc/host/rccl_comm.cpp, comm/native_rccl.py) and the ZeRO native-comm path.

GPU tests run one rank (RCCL single-rank communicator: every collective must equal its world-1 identity, stream
ordering and completion handles must hold). The multi-rank numerics of the same calls are exercised through the
torch.distributed path by the gloo ZeRO tests; parity unpinned for >1 GPU here (one card per test box)."""
import ctypes
import os

import pytest
import torch


def test_library_loads_and_exports():
    from hcache_deepspeed_amd.ops import native
    lib = native.host_lib()
    for name in ("hds_rccl_load", "hds_rccl_init", "hds_rccl_all_gather", "hds_rccl_reduce_scatter",
                 "hds_rccl_all_reduce", "hds_rccl_all_to_all", "hds_rccl_wait"):
        assert getattr(lib, name, None) is not None, name
    assert lib.hds_rccl_load(b"/nonexistent/librccl.so") in (0, 1)  # 0 if an earlier test already loaded it
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if os.path.exists(path):
        assert lib.hds_rccl_load(path.encode()) == 0
        assert lib.hds_rccl_error_string(0) == b"success"


@pytest.mark.gpu
def test_native_collectives_single_rank(cuda):
    from hcache_deepspeed_amd.comm.native_rccl import RcclCommunicator
    c = RcclCommunicator(None)
    x = torch.randn(4096, device=cuda, dtype=torch.bfloat16)
    out = torch.empty_like(x)
    c.all_gather_into_tensor(out, x)
    assert torch.equal(out, x)
    rs = torch.empty_like(x)
    c.reduce_scatter_tensor(rs, x * 2)
    assert torch.equal(rs, x * 2)
    y = torch.randn(1000, device=cuda)
    y0 = y.clone()
    c.all_reduce(y, op="max")
    assert torch.equal(y, y0)
    c.broadcast(y)
    a2a = torch.empty_like(y)
    c.all_to_all_single(a2a, y)
    assert torch.equal(a2a, y0)
    # async: the op is ordered after producer work on the caller stream, consumer waits on the GPU
    big = torch.empty(1 << 24, device=cuda)
    big.fill_(3.0)
    dst = torch.empty_like(big)
    w = c.all_gather_into_tensor(dst, big, async_op=True)
    w.wait()
    assert dst.sum().item() == 3.0 * big.numel()
    torch.cuda.synchronize()
    assert w.is_completed()
    c.destroy()


@pytest.mark.gpu
def test_zero3_native_comm_matches_torch_distributed(cuda):
    import hcache_deepspeed_amd as hds
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, tiny
    os.environ.setdefault("MASTER_PORT", "29571")

    def run(native):
        torch.manual_seed(0)
        m = LlamaForCausalLM(tiny(num_hidden_layers=2))
        cfg = {"train_micro_batch_size_per_gpu": 2, "bf16": {"enabled": True},
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 3},
               "compile": {"native_comm": native}}
        eng, _, _, _ = hds.initialize(model=m, config=cfg)
        eng.compile()
        g = torch.Generator().manual_seed(5)
        losses = []
        for _ in range(3):
            x = torch.randint(0, 512, (2, 128), generator=g).to(eng.device)
            loss = eng(x, labels=x)
            eng.backward(loss)
            eng.step()
            losses.append(loss.item())
        return losses, eng

    ref, _ = run(False)
    got, eng = run(True)
    opt = eng.optimizer
    assert opt._native is not None, "native comm not enabled by compile()"
    assert got == pytest.approx(ref, rel=1e-3, abs=1e-3)
    # world 1 keeps every unit resident (no gathers): drive the optimizer's collective helpers directly
    x = torch.randn(8192, device=eng.device, dtype=torch.bfloat16)
    out = torch.empty_like(x)
    opt._all_gather(out, x, None).wait()
    rs = torch.empty_like(x)
    opt._reduce_scatter(rs, x, None).wait()
    assert torch.equal(out, x) and torch.equal(rs, x)
    assert len(opt._native) == 1
