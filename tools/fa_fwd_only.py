"""Run the FlashAttention forward at the bench shape a few times (for rocprofv3 counter passes)."""
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import native  # noqa: E402
from hcache_deepspeed_amd.ops.attention import flash_attn  # noqa: E402

var = int(sys.argv[1]) if len(sys.argv) > 1 else 2
native.kernels().hds_attn_fwd_variant(var)
q = torch.randn(7, 4096, 32, 128, device="cuda", dtype=torch.bfloat16)
k = torch.randn(7, 4096, 8, 128, device="cuda", dtype=torch.bfloat16)
v = torch.randn(7, 4096, 8, 128, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    flash_attn(q, k, v, causal=True)
torch.cuda.synchronize()
