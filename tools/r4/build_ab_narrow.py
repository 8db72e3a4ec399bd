"""A/B build: the kernel library with the 8-B attention epilogue stores (HDS_NARROW_STORES) next to the default one,
for tools/r4/gpu_j.sh (load it with HDS_KERNEL_LIB)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hcache_deepspeed_amd.ops import build as b  # noqa: E402

flags = dict(b.FILE_FLAGS)
flags["flash_attn.hip"] = flags.get("flash_attn.hip", []) + ["-DHDS_NARROW_STORES"]
out = os.path.join(b.LIB_DIR, "libhds_kernels_narrow.so")
print(b.build_kernels(file_flags=flags, out=out, verbose=True))
