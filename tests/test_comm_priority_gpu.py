"""ZeRO-3 communicators created with high-priority RCCL streams (mi355x.comm_high_priority): the group builds
with ProcessGroupNCCL options on ROCm and its collectives are exact."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_high_priority_group_collectives():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hcache_deepspeed_amd as hds
    from hcache_deepspeed_amd import comm as dist
    os.environ.setdefault("MASTER_PORT", "29581")
    hds.init_distributed(verbose=False)
    g = dist.new_group(ranks=list(range(dist.get_world_size())), high_priority=True)
    x = torch.arange(1024, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(1024 * dist.get_world_size(), device="cuda", dtype=torch.bfloat16)
    torch.distributed.all_gather_into_tensor(out, x, group=g)
    torch.distributed.all_reduce(x, group=g)
    torch.cuda.synchronize()
    assert torch.equal(out[:1024], torch.arange(1024, device="cuda", dtype=torch.bfloat16))
    assert torch.equal(x, torch.arange(1024, device="cuda", dtype=torch.bfloat16) * dist.get_world_size())
