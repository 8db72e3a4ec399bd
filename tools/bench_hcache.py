"""HCache serving benchmark (the fork's feature): how fast a sequence's KV cache comes back.

Llama-3-8B (random bf16 weights, full 32 layers) in the ragged serving engine on one MI355X. A batch of contexts
is prefilled, evicted, and brought back three ways:

* recompute   — full prefill again (``put`` without latent capture),
* HCache      — ``restore_kv`` from the per-layer hidden-state latents kept in pinned host memory
                (H2D of layer i+1 overlapped with layer i's QKV GEMM + fused RoPE/paged-KV scatter),
* KV offload  — ``restore_kv`` in ``latent_mode="kv"`` (pre-RoPE K|V rows on the host; RoPE + scatter only),
* HCache FP8  — ``latent_mode="hidden_fp8"``: e4m3 hidden states + a per-token fp32 scale (H + 4 bytes per token-layer,
                byte parity with KV for GQA), dequantized on the device before the K|V GEMM.

After each restore, sequence 1 decodes ``--gen`` greedy tokens; the FP8 run is compared with the bf16 hidden-state
run (first-step logit relative error, token agreement).

Reports restored tokens/s and host bytes per token for each, plus the cost of capturing latents during prefill.

    python tools/bench_hcache.py [--seqs 8] [--ctx 2048]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--model", default="llama3-8b", help="llama3-8b (GQA 32/8) or llama2-7b (MHA)")
    ap.add_argument("--gen", type=int, default=64, help="greedy tokens decoded after each restore")
    args = ap.parse_args()
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
    from hcache_deepspeed_amd.models.llama import PRESETS, LlamaForCausalLM

    dev = torch.device("cuda", 0)
    preset = PRESETS[args.model]
    cfg = preset() if not args.layers else preset(num_hidden_layers=args.layers)
    torch.manual_seed(0)
    with torch.device(dev):
        model = LlamaForCausalLM(cfg).to(torch.bfloat16).eval()
    S, C = args.seqs, args.ctx
    n_tok = S * C
    blocks = S * ((C + 63) // 64) + 16
    econf = {"dtype": "bf16", "state_manager": {"max_ragged_batch_size": n_tok, "max_context": C + 64,
                                                 "kv_block_size": 64, "max_tracked_sequences": 4 * S}}
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (C, ), generator=g) for _ in range(S)]
    uids = list(range(1, S + 1))
    res = {}
    gen = {}
    for mode in ("hidden", "kv", "hidden_fp8", "hidden_int8"):
        eng = build_engine_from_model(model, dict(econf, latent_mode=mode), device=dev, num_kv_blocks=blocks)

        def prefill(capture):

            def f():
                for u in uids:
                    eng.flush(u)
                return eng.put(uids, prompts, capture_latents=capture)

            return f

        if mode == "hidden":
            res["recompute (prefill)"] = timed(prefill(False))
            res["prefill + latent capture"] = timed(prefill(True))
        _, lats = prefill(True)()
        torch.cuda.synchronize()
        lat_bytes = sum(x.numel() * x.element_size() for x in lats)
        assert all(x.is_pinned() for x in lats), "latents must live in pinned host memory"

        def restore():
            for u in uids:
                eng.evict(u)
            eng.restore_kv(uids, prompts, lats)

        res[f"restore_kv latent_mode={mode}"] = timed(restore)
        res[f"host bytes/token latent_mode={mode}"] = lat_bytes / n_tok
        # greedy continuation of sequence 1 after the restore
        toks, first = [], None
        nxt = torch.tensor([int(prompts[0][-1])])
        for _ in range(args.gen):
            lg, _ = eng.put([uids[0]], [nxt], capture_latents=False)
            if first is None:
                first = lg[0].float().cpu()
            nxt = lg[0].argmax().view(1).cpu()
            toks.append(int(nxt))
        gen[mode] = (first, toks)
        del eng, lats
        torch.cuda.empty_cache()
    print(f"{args.model} ({cfg.num_hidden_layers} layers, {cfg.num_attention_heads}/{cfg.num_key_value_heads} heads) bf16, {S} sequences x {C} tokens = {n_tok} tokens")
    for k, v in res.items():
        if k.startswith("host bytes"):
            print(f"  {k:40s} {v / 1024:8.1f} KiB")
        else:
            print(f"  {k:40s} {v * 1e3:8.1f} ms  {n_tok / v:10.0f} tokens/s")
    rc = res["recompute (prefill)"]
    print(f"  HCache restore speedup vs recompute: {rc / res['restore_kv latent_mode=hidden']:.2f}x; "
          f"FP8 HCache: {rc / res['restore_kv latent_mode=hidden_fp8']:.2f}x; "
          f"KV-offload restore speedup vs recompute: {rc / res['restore_kv latent_mode=kv']:.2f}x")
    (f0, t0) = gen["hidden"]
    quality = {}
    for qm in ("hidden_fp8", "hidden_int8"):
        f1, t1 = gen[qm]
        rel = float((f0 - f1).norm() / f0.norm())
        agree = sum(a == b for a, b in zip(t0, t1))
        first_diff = next((i for i, (a, b) in enumerate(zip(t0, t1)) if a != b), None)
        quality[qm] = {"logit_rel_err": rel, "tokens_equal": agree, "first_diff": first_diff}
        print(f"  {qm} vs bf16 hidden restore: first-step logit rel err {rel:.2e}, greedy tokens equal "
              f"{agree}/{len(t0)} (first difference at {first_diff})")
    print(f"  kv vs hidden tokens equal {sum(a == b for a, b in zip(t0, gen['kv'][1]))}/{len(t0)}")
    rel, agree, first_diff = (quality["hidden_fp8"][k] for k in ("logit_rel_err", "tokens_equal", "first_diff"))
    import json
    print(json.dumps({"tokens": n_tok, "model": args.model, "layers": cfg.num_hidden_layers,
                      "restore_tok_s": {m: round(n_tok / res[f"restore_kv latent_mode={m}"]) for m in gen},
                      "host_bytes_per_token": {m: res[f"host bytes/token latent_mode={m}"] for m in gen},
                      "recompute_tok_s": round(n_tok / rc), "fp8_logit_rel_err": rel, "fp8_tokens_equal": agree,
                      "gen": len(t0), "fp8_first_token_diff": first_diff, "quantized": quality}))


if __name__ == "__main__":
    main()
