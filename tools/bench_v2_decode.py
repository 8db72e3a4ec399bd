"""Ragged serving decode throughput (inference v2 engine, HCache's serving path): Llama-3-8B random bf16 weights,
B sequences prefilled with 512 tokens, then 32 decode steps of one token per sequence through ``put``. Prints
generated tokens/s for the GEMV-routed linears (default) and with the GEMV off (HDS_GEMV_MAX_NUMEL=0 in a
separate process: the rule is read at import). ``--capture-latents``: each B also runs with HCache latent capture ON
in the decode steps (graph-captured device ring, drained in bulk; the timed region ends after ``wait_latents``, so
every latent is on the host) next to capture off."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--capture-latents", action="store_true")
    ap.add_argument("--latent-mode", default="hidden")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--batches", default="1,4,8", help="comma-separated decode batch sizes")
    args = ap.parse_args()
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, llama3_8b
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        model = LlamaForCausalLM(llama3_8b()).to(torch.bfloat16).eval()
    P, steps = 512, args.steps
    for B in [int(b) for b in args.batches.split(",")]:
        for cap in ((False, True) if args.capture_latents else (False, )):
            econf = {"dtype": "bf16", "latent_mode": args.latent_mode,
                     "state_manager": {"max_ragged_batch_size": B * P, "max_context": P + 2 * steps + 64,
                                       "kv_block_size": 64, "max_tracked_sequences": 4 * B}}
            eng = build_engine_from_model(model, econf, device=dev,
                                          num_kv_blocks=B * ((P + 2 * steps + 63) // 64) + 16)
            g = torch.Generator().manual_seed(1)
            uids = list(range(1, B + 1))
            prompts = [torch.randint(0, 128256, (P, ), generator=g) for _ in range(B)]
            logits, _ = eng.put(uids, prompts, capture_latents=cap)
            nxt = logits.argmax(-1).cpu()
            for _ in range(2):  # graph capture of this batch size outside the timed loop
                logits, _ = eng.put(uids, [nxt[i:i + 1] for i in range(B)], capture_latents=cap, sync_latents=False)
                nxt = logits.argmax(-1).cpu()
            eng.wait_latents()
            torch.cuda.synchronize()
            kept = []
            t0 = time.perf_counter()
            for _ in range(steps):
                logits, lats = eng.put(uids, [nxt[i:i + 1] for i in range(B)], capture_latents=cap, sync_latents=False)
                kept.append(lats)
                nxt = logits.argmax(-1).cpu()
            eng.wait_latents()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            rec = {"B": B, "prompt": P, "decode_steps": steps, "capture_latents": cap,
                   "gemv_max_numel": os.environ.get("HDS_GEMV_MAX_NUMEL", "default"),
                   "tok_per_s": round(B * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 2)}
            if cap:
                rec["latent_mode"] = args.latent_mode
                rec["graph_decode"] = (B, True) in eng._model._decode_graphs
                rec["latent_bytes_per_step"] = int(sum(t.numel() * t.element_size() for t in kept[-1] if t is not None))
            print(json.dumps(rec), flush=True)
            del eng, kept
            import gc
            gc.collect()  # the engine's captured graphs are freed here, not by a collection during the next capture
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
