"""KV-cached generation throughput of Llama-3-8B (full width, random bf16 weights) on one MI355X: eager decode loop
against the HIP-graph decode step (models/generation.py). Prompt 128 tokens, 64 new tokens, greedy."""
import json
import os
import time

import torch

from hcache_deepspeed_amd.models.generation import KVCacheGenerator
from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, llama3_8b


def main():
    torch.manual_seed(0)
    with torch.device("cuda"):
        m = LlamaForCausalLM(llama3_8b())
    m = m.to(torch.bfloat16).eval()
    for B in (1, 8, 32):
        prompt = torch.randint(0, 128256, (B, 128), device="cuda")
        res = {"B": B, "prompt": 128, "new_tokens": 64}
        outs = {}
        for mode in ("0", "1"):
            os.environ["HDS_DECODE_GRAPH"] = mode
            gen = KVCacheGenerator(m)
            gen.generate(prompt, max_new_tokens=8)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            outs[mode] = gen.generate(prompt, max_new_tokens=64)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res["graph" if mode == "1" else "eager"] = {"s": round(dt, 4), "new_tok_per_s": round(B * 64 / dt, 1),
                                                        "used_graph": gen.used_graph}
        res["tokens_equal"] = bool(torch.equal(outs["0"], outs["1"]))
        res["speedup"] = round(res["eager"]["s"] / res["graph"]["s"], 3)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
