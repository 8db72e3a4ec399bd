"""Ragged paged-KV transformer for serving, with the HCache contract on every model.

Reference parity: inference/v2/model_implementations/llama_v2/model.py (``Llama2InferenceModel``,
HCache-modified forward :203-220 and ``restore_kv`` :222-244), mistral / qwen2 implementations, the
DSTransformerModelBase contract and the TP sharding helpers (model_implementations/sharding/*).

HCache, as implemented here (with the defects fixed):

* ``forward(batch, capture_latents=True)`` returns ``(logits, latents)``: the post-RMSNorm hidden state
  entering every layer's QKV projection, ``[L, T, H]``. Each layer's slice is copied D2H on a side HIP
  stream into a PINNED host buffer as soon as it is produced (event-ordered), so the transfer overlaps
  the remaining layers instead of one blocking pageable ``.cpu()`` at the end.
* ``restore_kv(batch, latents)`` rebuilds the paged KV cache from host latents: a copy stream streams
  layer i+1 host->device (pinned, async) while the compute stream runs layer i's QKV GEMM + fused
  RoPE/KV-scatter. Attention, O-projection and MLP are skipped (~1/4-1/6 of the layer FLOPs).
* ``latent_mode="kv"`` stores post-RoPE K|V per token-layer instead (2*Hkv*D elements; half of H for
  Llama-3 GQA) and restore becomes a pure scatter.
* every model type in this module implements the contract (the reference broke ``put`` for all
  non-Llama models).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import comm as dist
from ...ops.activations import glu
from ...ops.norm import rms_norm
from ...ops.paged import build_atoms, kv_rope_scatter, paged_attention
from ...ops.rope import rope_tables


class _LayerWeights:
    __slots__ = ("ln1", "qkv", "qkv_bias", "o", "ln2", "gate_up", "down", "moe")


class RaggedTransformer:
    """Llama / Mistral / Qwen2-style decoder over a paged KV cache (optionally tensor-parallel)."""

    def __init__(self, cfg, weights, device, dtype=torch.bfloat16, tp_group=None, latent_mode="hidden"):
        self.cfg = cfg
        self.device = device
        self.dtype = dtype
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.tp_rank = dist.get_rank(tp_group) if tp_group is not None else 0
        self.latent_mode = latent_mode
        H, D = cfg.hidden_size, cfg.head_dim
        assert cfg.num_attention_heads % self.tp == 0 and cfg.num_key_value_heads % self.tp == 0
        self.n_q = cfg.num_attention_heads // self.tp
        self.n_kv = cfg.num_key_value_heads // self.tp
        self.d = D
        self.I = cfg.intermediate_size // self.tp
        self._load(weights)
        self.cos, self.sin = rope_tables(max(cfg.max_position_embeddings, 8192), D, cfg.rope_theta, cfg.rope_scaling,
                                         device=device)
        self.scale = 1.0 / math.sqrt(D)
        self.kv_cache = None
        self.copy_stream = torch.cuda.Stream(device) if device.type == "cuda" else None

    # ------------------------------------------------------------------------------------------
    # weights (TP sharding: heads for QKV, rows for O/down, columns for gate|up; LM head by vocab)
    # ------------------------------------------------------------------------------------------
    def _load(self, sd):
        cfg, tp, r = self.cfg, self.tp, self.tp_rank
        D, Hq, Hkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads

        def t(x):
            return x.to(device=self.device, dtype=self.dtype).contiguous()

        self.embed = t(sd["model.embed_tokens.weight"])
        self.norm = t(sd["model.norm.weight"])
        lm = sd.get("lm_head.weight", sd["model.embed_tokens.weight"])
        V = lm.shape[0]
        vs = (V + tp - 1) // tp
        self.vocab = V
        self.lm_head = t(lm[r * vs:(r + 1) * vs])
        self.layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"model.layers.{i}."
            L = _LayerWeights()
            L.ln1 = t(sd[p + "input_layernorm.weight"])
            L.ln2 = t(sd[p + "post_attention_layernorm.weight"])
            qkv = sd[p + "self_attn.qkv_proj.weight"]
            q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], 0)
            nq, nkv = Hq // tp, Hkv // tp
            L.qkv = t(torch.cat([q[r * nq * D:(r + 1) * nq * D], k[r * nkv * D:(r + 1) * nkv * D],
                                 v[r * nkv * D:(r + 1) * nkv * D]], 0))
            qb = sd.get(p + "self_attn.qkv_proj.bias")
            if qb is not None:
                bq, bk, bv = qb.split([Hq * D, Hkv * D, Hkv * D], 0)
                L.qkv_bias = t(torch.cat([bq[r * nq * D:(r + 1) * nq * D], bk[r * nkv * D:(r + 1) * nkv * D],
                                          bv[r * nkv * D:(r + 1) * nkv * D]], 0))
            else:
                L.qkv_bias = None
            o = sd[p + "self_attn.o_proj.weight"]
            L.o = t(o[:, r * nq * D:(r + 1) * nq * D])
            gu = sd.get(p + "mlp.gate_up_proj.weight")
            L.moe = None
            if gu is not None:
                I = cfg.intermediate_size
                g, u = gu.split([I, I], 0)
                ii = I // tp
                L.gate_up = t(torch.cat([g[r * ii:(r + 1) * ii], u[r * ii:(r + 1) * ii]], 0))
                L.down = t(sd[p + "mlp.down_proj.weight"][:, r * ii:(r + 1) * ii])
            else:
                L.gate_up = L.down = None
                L.moe = self._load_moe(sd, p)
            self.layers.append(L)

    def _load_moe(self, sd, p):
        return None

    # ------------------------------------------------------------------------------------------
    def kv_cache_config(self):
        return dict(num_layers=self.cfg.num_hidden_layers, n_kv_heads=self.n_kv, head_dim=self.d)

    def set_kv_cache(self, kv_cache):
        self.kv_cache = kv_cache

    def _allreduce(self, x):
        if self.tp > 1:
            dist.all_reduce(x, group=self.tp_group)
        return x

    def _mlp(self, L, x):
        if L.moe is not None:
            return L.moe(x)
        return F.linear(glu(F.linear(x, L.gate_up), self.cfg.hidden_act), L.down)

    def _prep(self, batch):
        atoms, n_atoms = build_atoms(batch.seq_meta_host, self.n_q, self.n_kv)
        batch.atoms = atoms.to(self.device, non_blocking=True)
        batch.n_atoms = n_atoms

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def forward(self, batch, capture_latents=True):
        """Returns (logits [n_seqs, V], latents host [L, T, H] or [L, T, 2*n_kv*D] or None)."""
        cfg = self.cfg
        self._prep(batch)
        T = batch.current_tokens
        h = F.embedding(batch.input_ids, self.embed)
        residual = None
        lat = None
        events = []
        if capture_latents:
            width = cfg.hidden_size if self.latent_mode == "hidden" else 2 * self.n_kv * self.d
            lat = torch.empty(cfg.num_hidden_layers, T, width, dtype=self.dtype,
                              pin_memory=self.device.type == "cuda")
        nq, nkv, D = self.n_q, self.n_kv, self.d
        for i, L in enumerate(self.layers):
            if residual is None:
                x = rms_norm(h, L.ln1, cfg.rms_norm_eps)
                residual = h
            else:
                x, residual = rms_norm(h, L.ln1, cfg.rms_norm_eps, residual)
            qkv = F.linear(x, L.qkv, L.qkv_bias).view(T, nq + 2 * nkv, D)
            cache = self.kv_cache.get_cache(i)
            kv_rope_scatter(qkv, cache, batch.tok_seq, batch.tok_pos, batch.block_tables, self.cos, self.sin, nq, nkv)
            if capture_latents:
                src = x if self.latent_mode == "hidden" else qkv[:, nq:].reshape(T, -1)
                self._d2h(src, lat[i], events)
            o = paged_attention(qkv[:, :nq], cache, batch.atoms, batch.n_atoms, batch.seq_meta, batch.block_tables, nq,
                                nkv, self.scale, cfg.sliding_window, batch.seq_meta_host, batch.tables_host)
            a = self._allreduce(F.linear(o.view(T, nq * D), L.o))
            x, residual = rms_norm(a, L.ln2, cfg.rms_norm_eps, residual)
            h = self._allreduce(self._mlp(L, x))
        idx = batch.last_token_idx
        hl, _ = rms_norm(h[idx], self.norm, cfg.rms_norm_eps, residual[idx])
        logits = F.linear(hl, self.lm_head)
        if self.tp > 1:
            parts = [torch.empty_like(logits) for _ in range(self.tp)]
            dist.all_gather(parts, logits, group=self.tp_group)
            logits = torch.cat(parts, -1)[:, :self.vocab]
        if events:
            events[-1].synchronize()
        return logits, lat

    def _d2h(self, src, dst, events):
        if self.copy_stream is None:
            dst.copy_(src)
            return
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.copy_stream):
            self.copy_stream.wait_event(ev)
            dst.copy_(src, non_blocking=True)
            src.record_stream(self.copy_stream)
            done = torch.cuda.Event()
            done.record(self.copy_stream)
        events.append(done)

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def restore_kv(self, batch, latents):
        """Rebuild the paged KV of ``batch``'s sequences from host latents [L, T, W] (pinned preferred)."""
        cfg = self.cfg
        T = batch.current_tokens
        nq, nkv, D = self.n_q, self.n_kv, self.d
        L_ = cfg.num_hidden_layers
        if self.copy_stream is None:
            for i, L in enumerate(self.layers):
                self._restore_layer(i, L, latents[i].to(self.device), batch, T)
            return
        if not latents.is_pinned() and latents.device.type == "cpu":
            latents = latents.pin_memory()
        width = latents.shape[-1]
        bufs = [torch.empty(T, width, dtype=self.dtype, device=self.device) for _ in range(2)]
        loaded = [torch.cuda.Event() for _ in range(2)]
        freed = [torch.cuda.Event() for _ in range(2)]
        main = torch.cuda.current_stream()

        def issue(i):
            b = i & 1
            with torch.cuda.stream(self.copy_stream):
                if i >= 2:
                    self.copy_stream.wait_event(freed[b])
                bufs[b].copy_(latents[i], non_blocking=True)
                loaded[b].record(self.copy_stream)

        issue(0)
        if L_ > 1:
            issue(1)
        for i, L in enumerate(self.layers):
            b = i & 1
            main.wait_event(loaded[b])
            self._restore_layer(i, L, bufs[b], batch, T)
            freed[b].record(main)
            if i + 2 < L_:
                issue(i + 2)
        main.wait_stream(self.copy_stream)

    def _restore_layer(self, i, L, x, batch, T):
        nq, nkv, D = self.n_q, self.n_kv, self.d
        cache = self.kv_cache.get_cache(i)
        if self.latent_mode == "hidden":
            # only K|V rows of the projection are needed: GEMM against the k/v slice of W_qkv
            w = L.qkv[nq * D:]
            bias = L.qkv_bias[nq * D:] if L.qkv_bias is not None else None
            kv = F.linear(x, w, bias).view(T, 2 * nkv, D)
            kv_rope_scatter(kv, cache, batch.tok_seq, batch.tok_pos, batch.block_tables, self.cos, self.sin, 0, nkv,
                            rotate_q=False)
        else:
            # stored K is pre-RoPE (what the projection produced); rotation happens on the way in
            kv = x.view(T, 2 * nkv, D).contiguous()
            kv_rope_scatter(kv, cache, batch.tok_seq, batch.tok_pos, batch.block_tables, self.cos, self.sin, 0, nkv,
                            rotate_q=False)
