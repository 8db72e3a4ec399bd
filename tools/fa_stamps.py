"""Where a one-wave-per-SIMD forward tile spends its cycles: run forward variant 12 (variant 11 + s_memtime stamps at
the block boundaries) at the bench shape and print cycles per tile and wave for each segment.

Stamps live only in the A/B experiment library: build it with
``python -c "from hcache_deepspeed_amd.ops import build; build.build_kernels_diag()"`` (this script does it) and run
with ``HDS_KERNEL_LIB=hcache_deepspeed_amd/_lib/libhds_kernels_diag.so``."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from hcache_deepspeed_amd.ops import build as _build  # noqa: E402

if not os.environ.get("HDS_KERNEL_LIB"):
    os.environ["HDS_KERNEL_LIB"] = _build.build_kernels_diag()
from hcache_deepspeed_amd.ops import native  # noqa: E402
from hcache_deepspeed_amd.ops.attention import flash_attn  # noqa: E402

lib = native.kernels()
B, S, Hq, Hkv, D = 7, 4096, 32, 8, 128
q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
out = (ctypes.c_ulonglong * 32)()
VAR = int(sys.argv[1]) if len(sys.argv) > 1 else 12
lib.hds_attn_fwd_variant(VAR)
for _ in range(2):
    flash_attn(q, k, v, causal=True)
torch.cuda.synchronize()
lib.hds_attn_w64_stamps(out, 1)
for _ in range(3):
    flash_attn(q, k, v, causal=True)
torch.cuda.synchronize()
lib.hds_attn_w64_stamps(out, 1)
lib.hds_attn_fwd_variant(native.fwd_variant_default())
names = ["dma wait + barrier", "block A (S MFMAs + exp)", "P pack + mask", "block B (PV MFMAs + max)", "tail", "loop"]
tot = [sum(out[8 * w + i] for w in range(4)) for i in range(8)]
print(f"variant {VAR}: waves {tot[7]}, tiles per wave {tot[6] / max(1, tot[7]):.1f}; cycles per tile (all waves, then "
      f"wave 0 / 1 / 2 / 3: waves whose rows precede the last tiles idle there)")
for i, n in enumerate(names):
    per = [out[8 * w + i] / max(1, out[8 * w + 6]) for w in range(4)]
    print(f"{n:28s} {tot[i] / max(1, tot[6]):7.0f}   " + " / ".join(f"{x:5.0f}" for x in per))
print(f"{'MFMA floor (64 x 32)':28s} {2048:7d}")
