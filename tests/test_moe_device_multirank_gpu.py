"""Expert parallelism on the HIP device path: EP = 2 with both ranks on the one MI355X of the test box.

The 1-GPU box cannot run RCCL with two ranks, so the processes rendezvous over gloo and the token all-to-all is
staged through host memory; everything else -- top-k routing, the dispatch / combine kernels, the grouped SwiGLU
expert GEMMs on each rank's two local experts, their backward -- is the GPU path that EP > 1 runs on a node.

Reference: a world-1 run of the same layer with all four experts local (EP = 1) on the concatenation of both
ranks' tokens. Outputs must match row for row and each rank's local expert gradients must equal the reference's
slices (the two ranks' tokens both reach a rank's experts through the all-to-all)."""
import os

import pytest
import torch

from tests.dist_utils import run_distributed

pytestmark = pytest.mark.gpu

H, I, E, T = 256, 512, 4, 96


def _staged_all_to_all():
    import hcache_deepspeed_amd.comm as hcomm
    import torch.distributed as tdist

    def call(output, tensor, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
        o = output.detach().cpu()
        tdist.all_to_all_single(o, tensor.detach().cpu().contiguous(), output_split_sizes, input_split_sizes,
                                group=group)
        output.copy_(o)
        return hcomm.comm._Done() if async_op else None

    return call


def _weights():
    g = torch.Generator().manual_seed(0)
    # gate weights and tokens on a 1/8 grid: every router logit is an exact fp32 sum (its bf16 rounding then does not
    # depend on how many rows the gate GEMM had), so both runs route every token identically, ties included
    return (torch.randn(E, 2 * I, H, generator=g) * 0.05, torch.randn(E, H, I, generator=g) * 0.05,
            torch.randint(-4, 5, (E, H), generator=g).float() / 8)


def _tokens(r):
    return torch.randint(-4, 5, (T, H), generator=torch.Generator().manual_seed(100 + r)).float() / 8


def _run(rank, world, d):
    import hcache_deepspeed_amd.comm as hcomm
    from hcache_deepspeed_amd.parallel.moe import MoE
    torch.cuda.set_device(0)
    hcomm.all_to_all_single = _staged_all_to_all()
    hcomm.comm.all_to_all_single = hcomm.all_to_all_single
    w13, w2, wg = _weights()
    moe = MoE(H, None, E, ep_size=world, k=2, capacity_factor=16.0, eval_capacity_factor=16.0,
              expert_intermediate_size=I)
    ex = moe.deepspeed_moe.experts
    n = E // world
    assert ex.num_local_experts == n
    with torch.no_grad():
        ex.w13.copy_(w13[n * rank:n * rank + n])
        ex.w2.copy_(w2[n * rank:n * rank + n])
        moe.deepspeed_moe.gate.wg.weight.copy_(wg)
    moe = moe.cuda().to(torch.bfloat16)
    x = (torch.cat([_tokens(0), _tokens(1)]) if world == 1 else _tokens(rank)).cuda().to(torch.bfloat16)
    x.requires_grad_(True)
    out, _, _ = moe(x)
    out.float().square().sum().backward()
    torch.cuda.synchronize()
    torch.save({"out": out.detach().float().cpu(), "dx": x.grad.float().cpu(), "w13": ex.w13.grad.float().cpu(),
                "w2": ex.w2.grad.float().cpu(), "experts": list(range(n * rank, n * rank + n))},
               os.path.join(d, f"w{world}r{rank}.pt"))


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def test_expert_parallel_device_path_world2_matches_world1(tmp_path):
    d = str(tmp_path)
    run_distributed(_run, 1, d)
    run_distributed(_run, 2, d)
    ref = torch.load(os.path.join(d, "w1r0.pt"), weights_only=True)
    for r in range(2):
        got = torch.load(os.path.join(d, f"w2r{r}.pt"), weights_only=True)
        rows = slice(r * T, (r + 1) * T)
        assert _rel(got["out"], ref["out"][rows]) < 1e-2, r
        assert _rel(got["dx"], ref["dx"][rows]) < 2e-2, r
        e = got["experts"]
        assert _rel(got["w13"], ref["w13"][e]) < 2e-2, r
        assert _rel(got["w2"], ref["w2"][e]) < 2e-2, r
