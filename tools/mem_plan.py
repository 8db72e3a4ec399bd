"""Print the per-GPU HBM plan of the bench configs (BASELINE.json configs 2 and 5) at dp=1/2/4/8.

    python tools/mem_plan.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hcache_deepspeed_amd.models import llama  # noqa: E402
from hcache_deepspeed_amd.runtime.zero.mem_estimators import estimate_llama_training  # noqa: E402


def main():
    rows = [("Llama-3-8B", llama.llama3_8b(), 7, 4096, {}),
            ("Llama-3-70B", llama.llama3_70b(), 1, 4096, {}),
            ("Llama-3-70B +ckpt", llama.llama3_70b(), 2, 4096, {"ckpt": True}),
            ("Llama-3-70B Infinity(opt+param->host)", llama.llama3_70b(), 2, 4096,
             {"ckpt": True, "offload_optimizer": True, "offload_param": True})]
    print(f"{'config':40s} {'dp':>3s} {'mb':>3s} {'states':>8s} {'act':>8s} {'total':>8s} {'host':>8s} fits(268GiB usable)")
    for name, cfg, mb, seq, kw in rows:
        for dp in (1, 2, 4, 8):
            r = estimate_llama_training(cfg, mb, seq, dp, **kw)
            print(f"{name:40s} {dp:3d} {mb:3d} {r['states_gib']:8.1f} {r['activations_gib']:8.1f} "
                  f"{r['total_gib']:8.1f} {r['host_gib']:8.1f} {r['fits']}")


if __name__ == "__main__":
    main()
