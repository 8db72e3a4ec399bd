"""Ragged serving decode throughput (inference v2 engine, HCache's serving path): Llama-3-8B random bf16 weights,
B sequences prefilled with 512 tokens, then 32 decode steps of one token per sequence through ``put``. Prints
generated tokens/s for the GEMV-routed linears (default) and with the GEMV off (HDS_GEMV_MAX_NUMEL=0 in a
separate process: the rule is read at import)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, llama3_8b
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        model = LlamaForCausalLM(llama3_8b()).to(torch.bfloat16).eval()
    P, steps = 512, 32
    for B in (1, 4, 8):
        econf = {"dtype": "bf16", "state_manager": {"max_ragged_batch_size": B * P, "max_context": P + steps + 64,
                                                     "kv_block_size": 64, "max_tracked_sequences": 4 * B}}
        eng = build_engine_from_model(model, econf, device=dev, num_kv_blocks=B * ((P + steps + 63) // 64) + 16)
        g = torch.Generator().manual_seed(1)
        uids = list(range(1, B + 1))
        prompts = [torch.randint(0, 128256, (P, ), generator=g) for _ in range(B)]
        logits, _ = eng.put(uids, prompts, capture_latents=False)
        nxt = logits.argmax(-1).cpu()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            logits, _ = eng.put(uids, [nxt[i:i + 1] for i in range(B)], capture_latents=False)
            nxt = logits.argmax(-1).cpu()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"B": B, "prompt": P, "decode_steps": steps, "gemv_max_numel":
                          os.environ.get("HDS_GEMV_MAX_NUMEL", "default"), "tok_per_s": round(B * steps / dt, 1),
                          "ms_per_step": round(dt / steps * 1e3, 2)}), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
