"""Where does an inference-v2 decode step spend its time? Llama-3-8B random bf16, B sequences after a 512-token
prefill: per-step wall of put() split into host phases (scheduling checks + state manager, finalize, forward /
graph replay, post) with the GPU time of the forward from events, graph vs eager."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hcache_deepspeed_amd.inference.v2 import build_engine_from_model
    from hcache_deepspeed_amd.models.llama import LlamaForCausalLM, llama3_8b
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        model = LlamaForCausalLM(llama3_8b()).to(torch.bfloat16).eval()
    P, steps = 512, 24  # +3 untimed graph-capture steps per case
    cases = [(1, "graph"), (1, "eager"), (8, "graph"), (8, "eager")]
    if len(sys.argv) > 1:  # e.g. "1:graph,8:graph"
        cases = [(int(c.split(":")[0]), c.split(":")[1]) for c in sys.argv[1].split(",")]
    for B, mode in cases:
        if True:
            econf = {"dtype": "bf16", "state_manager": {"max_ragged_batch_size": B * P, "max_context": P + steps + 128,
                                                         "kv_block_size": 64, "max_tracked_sequences": 4 * B}}
            eng = build_engine_from_model(model, econf, device=dev, num_kv_blocks=B * ((P + steps + 127) // 64) + 16)
            if mode == "eager":
                eng._model.decode_graph_max_batch = 0
            g = torch.Generator().manual_seed(1)
            uids = list(range(1, B + 1))
            logits, _ = eng.put(uids, [torch.randint(0, 128256, (P, ), generator=g) for _ in range(B)],
                                capture_latents=False)
            nxt = logits.argmax(-1).cpu()
            for _ in range(3):  # untimed: the decode graph for this batch size is captured here
                logits, _ = eng.put(uids, [nxt[i:i + 1] for i in range(B)], capture_latents=False)
                nxt = logits.argmax(-1).cpu()
            torch.cuda.synchronize()
            m = eng._model
            orig_fwd, orig_graph = m.forward, m.forward_decode_graph
            acc = {"fwd_host_ms": 0.0, "fwd_gpu_ms": 0.0}

            def timed(fn):
                def w(*a, **k):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    t0 = time.perf_counter()
                    e0.record()
                    r = fn(*a, **k)
                    e1.record()
                    acc["fwd_host_ms"] += (time.perf_counter() - t0) * 1e3
                    acc.setdefault("_ev", []).append((e0, e1))
                    return r
                return w

            m.forward, m.forward_decode_graph = timed(orig_fwd), timed(orig_graph)
            b = eng._batch
            orig_fin = b.finalize
            fin = {"ms": 0.0}

            def tfin():
                t0 = time.perf_counter()
                orig_fin()
                fin["ms"] += (time.perf_counter() - t0) * 1e3

            b.finalize = tfin
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                logits, _ = eng.put(uids, [nxt[i:i + 1] for i in range(B)], capture_latents=False)
                nxt = logits.argmax(-1).cpu()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps * 1e3
            gpu = sum(a.elapsed_time(b_) for a, b_ in acc.pop("_ev")) / steps
            print(json.dumps({"B": B, "mode": mode, "graphs": sorted(m._decode_graphs), "ms_per_step": round(dt, 2),
                              "tok_per_s": round(B * 1e3 / dt, 1), "finalize_ms": round(fin["ms"] / steps, 3),
                              "forward_host_ms": round(acc["fwd_host_ms"] / steps, 3),
                              "forward_gpu_ms": round(gpu, 3)}), flush=True)
            m.forward, m.forward_decode_graph = orig_fwd, orig_graph
            del eng
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
