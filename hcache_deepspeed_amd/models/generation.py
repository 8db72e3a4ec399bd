"""KV-cached autoregressive generation for this framework's Llama-family models, optionally tensor-parallel.

Reference parity: the RLHF hybrid engine's generation path (runtime/hybrid_engine.py ``generate`` :168-272) runs
the policy model through the kernel-injected inference containers with a KV cache (the ``softmax_context``
binding of csrc/transformer/inference/csrc/pt_binding.cpp) and, with ``inference_tp_size > 1``, slices every layer
over the model-parallel group (``apply_tensor_parallelism`` :200) after all-gathering the group's prompts (:217).

MI355X design:
* the cache is one preallocated ``[B, Hkv, S_max, D]`` bf16 buffer per layer (288 GB of HBM holds it next to a
  gathered 70B policy), laid out for the split-K HIP decode kernel (``ops/decode_attention.py``), which serves GQA
  without repeated K/V copies and takes the left-padding mask as an additive bias;
* prefill runs the training FlashAttention kernel on the fused QKV GEMM output after in-place HIP RoPE, exactly
  like the training forward; decode runs per-row positions through the same RoPE kernel;
* tensor parallelism slices the fused QKV / gate-up weights by heads / columns once per ``generate`` call and ends
  each block with one all-reduce (RCCL over xGMI), so per-rank HBM traffic per token falls with the TP degree.
"""
import math

import torch
import torch.nn.functional as F

from ..ops.activations import glu
from ..ops.attention import flash_attn
from ..ops.decode_attention import decode_attention, kv_append, sdpa_gqa
from ..ops.gemv import linear  # F.linear; decode-sized (<= 8 rows) bf16 inputs on the HIP GEMV
from ..ops.norm import rms_norm
from ..ops.rope import rope_


def _sample(logits, do_sample, temperature, top_k, top_p, generator):
    """logits [B, V] fp32 -> next ids [B] (greedy, or temperature / top-k / nucleus sampling)."""
    if not do_sample:
        return logits.argmax(-1)
    if temperature and temperature != 1.0:
        logits = logits / float(temperature)
    if top_k and top_k > 0:
        kth = torch.topk(logits, min(int(top_k), logits.shape[-1]), -1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p is not None and top_p < 1.0:
        srt, idx = torch.sort(logits, -1, descending=True)
        cum = torch.softmax(srt, -1).cumsum(-1)
        drop = cum - torch.softmax(srt, -1) > float(top_p)  # keep the smallest prefix whose mass reaches top_p
        srt = srt.masked_fill(drop, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, idx, srt)
    probs = torch.softmax(logits, -1)
    return torch.multinomial(probs, 1, generator=generator).squeeze(-1)


class _LayerShard:
    """One decoder block's weights as seen by this TP rank (views when tp == 1)."""

    def __init__(self, layer, cfg, tp, r):
        att, mlp = layer.self_attn, layer.mlp
        nq, nkv, D = att.n_q, att.n_kv, att.d
        assert nq % tp == 0 and nkv % tp == 0, f"inference_tp_size={tp} must divide heads ({nq} q, {nkv} kv)"
        self.nq, self.nkv, self.D = nq // tp, nkv // tp, D
        self.ln1, self.ln2 = layer.input_layernorm, layer.post_attention_layernorm
        self.act = mlp.act
        wqkv, bqkv = att.qkv_proj.weight, att.qkv_proj.bias
        wgu = mlp.gate_up_proj.weight
        I = wgu.shape[0] // 2
        if tp == 1:
            self.wqkv, self.bqkv, self.wo, self.bo = wqkv, bqkv, att.o_proj.weight, att.o_proj.bias
            self.wgu, self.wdown, self.bdown = wgu, mlp.down_proj.weight, mlp.down_proj.bias
            return
        qs = slice(r * self.nq * D, (r + 1) * self.nq * D)
        ks = slice(nq * D + r * self.nkv * D, nq * D + (r + 1) * self.nkv * D)
        vs = slice((nq + nkv) * D + r * self.nkv * D, (nq + nkv) * D + (r + 1) * self.nkv * D)
        self.wqkv = torch.cat([wqkv[qs], wqkv[ks], wqkv[vs]], 0)
        self.bqkv = torch.cat([bqkv[qs], bqkv[ks], bqkv[vs]], 0) if bqkv is not None else None
        self.wo = att.o_proj.weight[:, qs].contiguous()
        self.bo = att.o_proj.bias  # added once, after the all-reduce
        Is = I // tp
        self.wgu = torch.cat([wgu[r * Is:(r + 1) * Is], wgu[I + r * Is:I + (r + 1) * Is]], 0)
        self.wdown = mlp.down_proj.weight[:, r * Is:(r + 1) * Is].contiguous()
        self.bdown = mlp.down_proj.bias


class KVCacheGenerator:
    """``generate`` for :class:`models.llama.LlamaForCausalLM` (and models sharing its block layout).

    ``tp_group``: process group the layers are sliced over (every rank must pass the same prompts; the hybrid
    engine all-gathers them). Parameters must be materialised (ZeRO-3 callers gather them first).
    """

    def __init__(self, model, tp_group=None):
        from .. import comm as dist
        self.model = model
        self.cfg = model.config
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.tp_rank = dist.get_rank(tp_group) if tp_group is not None else 0
        self._dist = dist
        self.layers = [_LayerShard(l, self.cfg, self.tp, self.tp_rank) for l in model.model.layers]

    def _all_reduce(self, x):
        if self.tp > 1:
            self._dist.all_reduce(x, group=self.tp_group)
        return x

    def _block(self, li, h, residual, cos, sin, pos, cache, step_args):
        L = self.layers[li]
        if residual is None:
            x, residual = rms_norm(h, L.ln1.weight, L.ln1.eps), h
        else:
            x, residual = rms_norm(h, L.ln1.weight, L.ln1.eps, residual)
        T = x.shape[0]
        qkv = linear(x, L.wqkv, L.bqkv).view(T, L.nq + 2 * L.nkv, L.D)
        rope_(qkv, cos, sin, L.nq + L.nkv, pos_ids=pos)
        o = self._attend(li, qkv, cache, step_args).reshape(T, L.nq * L.D)
        a = self._all_reduce(linear(o, L.wo))
        if L.bo is not None:
            a = a + L.bo
        x, residual = rms_norm(a, L.ln2.weight, L.ln2.eps, residual)
        m = self._all_reduce(linear(glu(linear(x, L.wgu), L.act), L.wdown))
        if L.bdown is not None:
            m = m + L.bdown
        return m, residual

    def _attend(self, li, qkv, cache, a):
        L = self.layers[li]
        kc, vc = cache[li]
        q, k, v = qkv[:, :L.nq], qkv[:, L.nq:L.nq + L.nkv], qkv[:, L.nq + L.nkv:]
        B, scale, window = a["B"], 1.0 / math.sqrt(L.D), self.cfg.sliding_window or 0
        if a["phase"] == "prefill":
            S = a["S"]
            kc[:, :, :S] = k.view(B, S, L.nkv, L.D).transpose(1, 2)
            vc[:, :, :S] = v.view(B, S, L.nkv, L.D).transpose(1, 2)
            if a["mask"] is None:
                return flash_attn(q.reshape(B, S, L.nq, L.D), k.reshape(B, S, L.nkv, L.D),
                                  v.reshape(B, S, L.nkv, L.D), causal=True, softmax_scale=scale, window=window)
            # left-padded prompts: causal + key-padding mask (prefill runs once per generate call)
            o = sdpa_gqa(q.reshape(B, S, L.nq, L.D).transpose(1, 2), kc[:, :, :S], vc[:, :, :S], mask=a["mask"],
                         scale=scale)
            return o.transpose(1, 2).reshape(B * S, L.nq, L.D)
        if a["phase"] == "decode_graph":  # device-side position and length: one launch shape for every token
            B = a["B"]
            kv_append(k, v, kc, vc, a["cur_idx"])
            return decode_attention(q, kc, vc, scale, bias=a["bias"], lens=a["lens"], window=window)
        cur = a["cur"]
        kc[:, :, cur] = k
        vc[:, :, cur] = v
        lo = max(0, cur + 1 - window) if window > 0 else 0
        bias = a["bias"][:, lo:cur + 1] if a["bias"] is not None else None
        return decode_attention(q, kc[:, :, lo:cur + 1], vc[:, :, lo:cur + 1], scale, bias=bias)

    def _forward(self, ids, pos, cache, step_args):
        """ids [T] -> final normed hidden [T, H] (T = B*S at prefill, B at decode)."""
        m = self.model.model
        h = m.embed_tokens(ids)
        residual = None
        for li in range(len(self.layers)):
            h, residual = self._block(li, h, residual, self._cos, self._sin, pos, cache, step_args)
        h, _ = m.norm(h, residual)
        return h

    def _graph_ok(self, dev, B, max_new_tokens):
        """HIP-graph decode: single-GPU (no TP collectives in the step), the HIP decode kernel available."""
        import os
        from ..ops.decode_attention import decode_supported
        if dev.type != "cuda" or self.tp > 1 or int(max_new_tokens) < 3 or os.environ.get("HDS_DECODE_GRAPH", "1") == "0":
            return False
        L = self.layers[0]
        q = torch.empty(B, L.nq, L.D, device=dev, dtype=L.wqkv.dtype)
        return decode_supported(q, torch.empty(B, L.nkv, 1, L.D, device=dev, dtype=L.wqkv.dtype))

    def _decode_logits(self, ids, args, pos, cache):
        h = self._forward(ids, pos, cache, args)
        return linear(h, self.model.lm_head.weight).float()

    @torch.no_grad()
    def generate(self, input_ids, attention_mask=None, max_new_tokens=32, do_sample=False, temperature=1.0,
                 top_k=0, top_p=1.0, eos_token_id=None, pad_token_id=None, generator=None, min_new_tokens=0):
        """input_ids [B, S] (left-padded when ``attention_mask`` has zeros) -> [B, S + n] token ids."""
        B, S = input_ids.shape
        dev = input_ids.device
        cfg = self.cfg
        L0 = self.layers[0]
        dtype = L0.wqkv.dtype
        smax = S + int(max_new_tokens)
        self._cos, self._sin = self.model.model.rope(dev, smax)
        cache = [(torch.empty(B, L.nkv, smax, L.D, device=dev, dtype=dtype),
                  torch.empty(B, L.nkv, smax, L.D, device=dev, dtype=dtype)) for L in self.layers]
        padded = attention_mask is not None and not bool(attention_mask.all())
        if padded:
            am = attention_mask.to(dev).bool()
            pos = (am.long().cumsum(-1) - 1).clamp_min(0)
            causal = torch.ones(S, S, dtype=torch.bool, device=dev).tril()
            mask = causal[None, None] & am[:, None, None, :]
            if cfg.sliding_window:
                mask &= ~torch.ones(S, S, dtype=torch.bool, device=dev).tril(-cfg.sliding_window)[None, None]
            mask |= ~am[:, None, :, None]  # fully padded query rows attend somewhere (their output is unused)
            bias = torch.zeros(B, smax, device=dev, dtype=torch.float32)
            bias[:, :S].masked_fill_(~am, float("-inf"))
            next_pos = pos[:, -1] + 1
        else:
            pos = torch.arange(S, device=dev).expand(B, S)
            mask = bias = None
            next_pos = torch.full((B, ), S, device=dev, dtype=torch.long)
        h = self._forward(input_ids.reshape(-1), pos.reshape(-1).to(torch.int32), cache,
                          {"phase": "prefill", "B": B, "S": S, "mask": mask})
        head = self.model.lm_head.weight
        out = [input_ids]
        finished = torch.zeros(B, dtype=torch.bool, device=dev)
        last = h.view(B, S, -1)[:, -1]
        # Decode steps are launch-bound at small batch (~10 kernels per layer for one token): with ``graph`` the
        # step is captured once as a HIP graph over static buffers (token ids, positions, the cache slot and the
        # valid lengths live on the device and advance in place) and replayed for every further token.
        graph = self._graph_ok(dev, B, max_new_tokens)
        g = None
        if graph:
            ids_buf = torch.zeros(B, dtype=torch.long, device=dev)
            pos_buf = next_pos.to(torch.int32).clone()
            lens_buf = torch.full((B, ), S + 1, dtype=torch.int32, device=dev)
            cur_idx = torch.full((1, ), S, dtype=torch.long, device=dev)
            gargs = {"phase": "decode_graph", "B": B, "cur_idx": cur_idx, "lens": lens_buf, "bias": bias}
        logits = None
        for t in range(int(max_new_tokens)):
            if logits is None:
                logits = F.linear(last, head).float()
            if eos_token_id is not None and t < min_new_tokens:
                logits[:, eos_token_id] = float("-inf")
            nxt = _sample(logits, do_sample, temperature, top_k, top_p, generator)
            if self.tp > 1 and do_sample:  # one draw for the whole group
                self._dist.broadcast(nxt, self._dist.get_global_rank(self.tp_group, 0), group=self.tp_group)
            if eos_token_id is not None:
                fill = pad_token_id if pad_token_id is not None else eos_token_id
                nxt = torch.where(finished, torch.full_like(nxt, fill), nxt)
                finished |= nxt == eos_token_id
            out.append(nxt[:, None])
            if t + 1 == int(max_new_tokens) or (eos_token_id is not None and bool(finished.all())):
                break
            if graph:
                ids_buf.copy_(nxt)
                if g is None:  # first decode step: eager on a side stream (warms kernels / BLAS), then capture
                    side = torch.cuda.Stream(dev)
                    side.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(side):
                        logits = self._decode_logits(ids_buf, gargs, pos_buf, cache).clone()
                    torch.cuda.current_stream(dev).wait_stream(side)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        static_logits = self._decode_logits(ids_buf, gargs, pos_buf, cache)
                else:
                    g.replay()
                    logits = static_logits
                pos_buf += 1
                lens_buf += 1
                cur_idx += 1
                continue
            h = self._forward(nxt, next_pos.to(torch.int32), cache, {"phase": "decode", "B": B, "cur": S + t,
                                                                         "bias": bias})
            next_pos = next_pos + 1
            logits = F.linear(h, head).float()
        self.used_graph = g is not None
        return torch.cat(out, 1)


def generate(model, input_ids, tp_group=None, **kwargs):
    """Functional form of :meth:`KVCacheGenerator.generate`."""
    return KVCacheGenerator(model, tp_group).generate(input_ids, **kwargs)


def supports_kv_generation(model):
    m = getattr(model, "model", None)
    layers = getattr(m, "layers", None)
    if layers is None or len(layers) == 0 or not hasattr(model, "lm_head"):
        return False
    l0 = layers[0]
    return all(hasattr(l0, a) for a in ("input_layernorm", "self_attn", "post_attention_layernorm", "mlp")) and \
        hasattr(l0.self_attn, "qkv_proj") and hasattr(l0.mlp, "gate_up_proj")
