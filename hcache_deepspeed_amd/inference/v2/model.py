"""Ragged paged-KV decoder for serving, with the HCache contract on every supported family.

Reference parity: inference/v2/model_implementations/llama_v2/model.py (``Llama2InferenceModel``, HCache-modified
forward :203-220 and ``restore_kv`` :222-244) and the mistral / mixtral / qwen / qwen_v2 / qwen_v2_moe / phi /
phi3 / falcon / opt implementations, the DSTransformerModelBase contract and the TP sharding helpers
(model_implementations/sharding/*). One implementation, driven by :class:`arch.ArchSpec`: RMSNorm or
LayerNorm (+bias), gated (SwiGLU) or plain (GELU/ReLU) MLPs with optional biases, sequential or parallel
(shared-norm / two-norm) residual blocks, RoPE (full or partial) or learned positions, sliding windows, and
top-k MoE with optional shared expert.

HCache, as implemented here (with the defects fixed):

* ``forward(batch, capture_latents=True)`` returns ``(logits, latents)``: the normed hidden state entering
  every layer's QKV projection, ``[L, T, H]``. Each layer's slice is copied D2H on a side HIP stream into a
  PINNED host buffer as soon as it is produced (event-ordered), so the transfer overlaps the remaining
  layers instead of one blocking pageable ``.cpu()`` at the end.
* ``restore_kv(batch, latents)`` rebuilds the paged KV cache from host latents: a copy stream streams layer
  i+1 host->device (pinned, async) while the compute stream runs layer i's K|V GEMM + fused RoPE/KV-scatter.
  Attention, O-projection and MLP are skipped.
* ``latent_mode="kv"`` stores the PRE-RoPE K|V rows per token-layer instead (2*Hkv*D elements; half of H for
  Llama-3 GQA); restore then only rotates and scatters.
* ``latent_mode="hidden_fp8"`` stores the hidden state as OCP e4m3 with one fp32 scale per token (``fpq`` /
  ``quant.hip`` kernels), packed per token as [H bytes | 4 scale bytes]: H + 4 bytes per token-layer, byte parity
  with KV offload for Llama-3 GQA (2*Hkv*D*2 = H bytes) where bf16 hidden states are 2x KV;
  restore dequantizes on the device before the K|V GEMM. ``"hidden_int8"``: symmetric int8 with an fp32 scale per
  128 channels (H * 1.03 bytes; ~3.5x lower quantization error than e4m3 for near-Gaussian activations).
  ``"auto"`` picks the smaller LOSSLESS latent: K|V for GQA, the hidden state for MHA.
* latent host buffers come from a pinned pool (``offload/pinned.PinnedPool``) and return to it when the caller
  drops the latents -- no hipHostMalloc / torch pinned allocation per ``put()``.
* every family above implements the contract (the reference broke ``put`` for all non-Llama models).
"""
import math
import os as _os
import types

import torch
import torch.nn.functional as F

from ... import comm as dist
from ...ops.activations import glu
from ...ops.norm import layer_norm, rms_norm
from ...ops.paged import build_atoms, kv_rope_scatter
from ...ops.rope import rope_tables
from .modules import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig, instantiate_attention, instantiate_embed, instantiate_linear, instantiate_moe,
                      instantiate_pre_norm, instantiate_unembed)
from .modules.implementations import _PackedWeight


class _Layer:

    def __init__(self):
        self.w = {}

    def __getitem__(self, k):
        return self.w.get(k)


class RaggedTransformer:
    """Decoder over a paged KV cache (optionally tensor-parallel), configured by an ArchSpec."""

    def __init__(self, spec, weights, device, dtype=torch.bfloat16, tp_group=None, latent_mode="hidden",
                 engine_config=None):
        self.cfg = self.spec = spec
        self.device = device
        self.dtype = dtype
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.tp_rank = dist.get_rank(tp_group) if tp_group is not None else 0
        # "auto": the smaller lossless latent per token-layer -- pre-RoPE K|V for GQA models (2*Hkv*D < H), the hidden
        # state otherwise (HCache's byte advantage, MHA)
        if latent_mode == "auto":
            latent_mode = "kv" if 2 * spec.num_key_value_heads * spec.head_dim < spec.hidden_size else "hidden"
        assert latent_mode in ("hidden", "kv", "hidden_fp8", "hidden_int8"), latent_mode
        self.latent_mode = latent_mode
        D = spec.head_dim
        assert spec.num_attention_heads % self.tp == 0 and spec.num_key_value_heads % self.tp == 0, \
            "attention heads must divide the tensor-parallel size"
        self.n_q = spec.num_attention_heads // self.tp
        self.n_kv = spec.num_key_value_heads // self.tp
        self.d = D
        self.rot = spec.rotary_dim if 0 < spec.rotary_dim < D else D
        self.scale = 1.0 / math.sqrt(D)
        self._build_modules(engine_config)
        self._load(weights)
        if spec.pos == "rope":
            self.cos, self.sin = rope_tables(max(spec.max_position_embeddings, 8192), self.rot, spec.rope_theta,
                                             spec.rope_scaling, device=device)
        else:
            self.cos = self.sin = None
        self.kv_cache = None
        self.copy_stream = torch.cuda.Stream(device, priority=-1) if device.type == "cuda" else None
        self._decode_graphs = {}
        self._graph_pool = None
        import os as _os
        # HCache latents inside the decode graph (device ring drained every `decode_latent_ring_steps` steps)
        self.decode_graph_latents = _os.environ.get("HDS_V2_DECODE_GRAPH_LATENTS", "1") == "1"
        self.decode_latent_ring_steps = int(_os.environ.get("HDS_V2_LATENT_RING_STEPS", "16"))
        self.decode_graph_max_batch = int(_os.environ.get("HDS_V2_DECODE_GRAPH_MAX_B", "64"))

    def _build_modules(self, ec):
        """Compute modules chosen by the inference-v2 heuristics (modules/heuristics.py): the engine config's
        ``quantization.quantization_mode`` switches every projection to the FP6 / INT weight-only kernels."""
        spec, D, H = self.spec, self.d, self.spec.hidden_size
        nq, nkv = self.n_q, self.n_kv
        norm = DSNormConfig(H, "rms" if spec.norm == "rms" else "layer", spec.norm_eps)
        self.norm_mod = instantiate_pre_norm(norm, ec)
        self.embed_mod = instantiate_embed(DSEmbeddingsConfig(embedding_dim=H, positional_offset=spec.pos_offset), ec)
        self.attn_mod = instantiate_attention(
            DSSelfAttentionConfig(nq, nkv, D, scale_factor=self.scale, rotary_dim=self.rot,
                                  positional_embedding_type="rotate_half" if spec.pos == "rope" else "none",
                                  sliding_window=spec.sliding_window or 0), ec)
        self.qkv_lin = instantiate_linear(DSLinearConfig(H, (nq + 2 * nkv) * D), ec)
        self.o_lin = instantiate_linear(DSLinearConfig(nq * D, H), ec)
        act = self._act_name()
        I = spec.intermediate_size // self.tp
        if spec.moe is not None:
            m = spec.moe
            self.moe_mod = instantiate_moe(DSMoEConfig(H, I, int(m.get("num_experts", 0)), int(m["top_k"]),
                                                       f"{act}_glu", bool(m["normalize"])), ec)
        if spec.gated:
            self.up_lin = instantiate_linear(DSLinearConfig(H, 2 * I, activation=f"{act}_glu"), ec)
        else:
            self.up_lin = instantiate_linear(DSLinearConfig(H, I, activation=act), ec)
        self.down_lin = instantiate_linear(DSLinearConfig(I, H), ec)
        self.unembed_mod = instantiate_unembed(DSUnembedConfig(model_dim=H, vocab_size=spec.vocab_size,
                                                               norm_type="rms" if spec.norm == "rms" else "layer"), ec)

    def _transform(self, L):
        """Per-implementation weight layout (quantization happens here, once, on the device)."""
        w = L.w
        for key, mod in (("qkv.w", self.qkv_lin), ("o.w", self.o_lin), ("up.w", self.up_lin),
                         ("down.w", self.down_lin)):
            if w.get(key) is not None:
                w[key] = mod.transform_param(w[key])

    # ------------------------------------------------------------------------------------------
    # weights: canonical dict (arch.convert_*) -> this rank's shards
    # ------------------------------------------------------------------------------------------
    def _t(self, x):
        return None if x is None else x.to(device=self.device, dtype=self.dtype).contiguous()

    def _rows(self, x):
        if x is None or self.tp == 1:
            return x
        n = x.shape[0] // self.tp
        return x[self.tp_rank * n:(self.tp_rank + 1) * n]

    def _cols(self, x):
        if x is None or self.tp == 1:
            return x
        n = x.shape[-1] // self.tp
        return x[..., self.tp_rank * n:(self.tp_rank + 1) * n]

    def _gated_rows(self, x):
        """[gate; up] stacked on dim -2 -> this rank's gate rows and up rows."""
        if x is None or self.tp == 1:
            return x
        g, u = x.chunk(2, dim=-2)
        n = g.shape[-2] // self.tp
        sl = slice(self.tp_rank * n, (self.tp_rank + 1) * n)
        return torch.cat([g[..., sl, :], u[..., sl, :]], -2)

    def _load(self, sd):
        if sd.get("__presharded__"):  # reloaded serialize() shards: already this rank's slices
            self._rows = self._cols = self._gated_rows = lambda x: x
            return self._load_presharded(sd)
        spec, r = self.spec, self.tp_rank
        D, Hq, Hkv = spec.head_dim, spec.num_attention_heads, spec.num_key_value_heads
        nq, nkv = self.n_q, self.n_kv
        t = self._t
        self.embed = t(sd["embed"])
        self.pos_embed = t(sd.get("pos_embed"))
        self.final_w, self.final_b = t(sd.get("final.w")), t(sd.get("final.b"))
        lm = sd.get("lm_head.w")
        lm = sd["embed"] if lm is None else lm
        V = lm.shape[0]
        vs = (V + self.tp - 1) // self.tp
        self.vocab = V

        def vocab_shard(x):  # equal row counts on every rank (zero rows pad an uneven last shard): the logits
            s = x[r * vs:(r + 1) * vs]  # all-gather needs equal sizes; the padding columns are cut at ``vocab``
            if s.shape[0] < vs:
                s = torch.cat([s, s.new_zeros((vs - s.shape[0], ) + tuple(s.shape[1:]))])
            return s

        self.lm_head = t(vocab_shard(lm))
        lb = sd.get("lm_head.b")
        self.lm_head_b = t(vocab_shard(lb)) if lb is not None else None
        self.layers = []
        for Ls in sd["layers"]:
            L = _Layer()
            w = L.w
            for k in ("ln1.w", "ln1.b", "ln2.w", "ln2.b"):
                w[k] = t(Ls.get(k))

            def heads(x):
                if x is None:
                    return None
                q, k_, v = x.split([Hq * D, Hkv * D, Hkv * D], 0)
                return torch.cat([q[r * nq * D:(r + 1) * nq * D], k_[r * nkv * D:(r + 1) * nkv * D],
                                  v[r * nkv * D:(r + 1) * nkv * D]], 0)

            w["qkv.w"], w["qkv.b"] = t(heads(Ls["qkv.w"])), t(heads(Ls.get("qkv.b")))
            w["o.w"] = t(self._cols(Ls["o.w"]))
            w["o.b"] = t(Ls.get("o.b")) if r == 0 else None  # row-parallel bias added once
            if "w13" in Ls:
                w["router.w"] = t(Ls["router.w"])
                w["w13"] = t(self._gated_rows(Ls["w13"]))
                w["w2"] = t(self._cols(Ls["w2"]))
                w["shared.w13"] = t(self._gated_rows(Ls.get("shared.w13")))
                w["shared.w2"] = t(self._cols(Ls.get("shared.w2")))
                w["shared_gate.w"] = t(Ls.get("shared_gate.w"))
            else:
                up = Ls["up.w"]
                w["up.w"] = t(self._gated_rows(up) if self.spec.gated else self._rows(up))
                ub = Ls.get("up.b")
                if ub is not None:
                    w["up.b"] = t(self._gated_rows(ub[:, None])[:, 0] if self.spec.gated else self._rows(ub))
                w["down.w"] = t(self._cols(Ls["down.w"]))
                w["down.b"] = t(Ls.get("down.b")) if r == 0 else None
            self._transform(L)
            self.layers.append(L)

    def _load_presharded(self, sd):
        t = self._t
        self.embed, self.pos_embed = t(sd["embed"]), t(sd.get("pos_embed"))
        self.final_w, self.final_b = t(sd.get("final.w")), t(sd.get("final.b"))
        self.lm_head, self.lm_head_b = t(sd["lm_head.w"]), t(sd.get("lm_head.b"))
        self.vocab = self.spec.vocab_size
        self.layers = []
        for Ls in sd["layers"]:
            L = _Layer()
            L.w = {k: (_PackedWeight(v["q"].to(self.device), v["scales"].to(self.device), *[int(i) for i in v["meta"]])
                       if isinstance(v, dict) else t(v)) for k, v in Ls.items()}
            self._transform(L)
            self.layers.append(L)

    # ------------------------------------------------------------------------------------------
    def kv_cache_config(self):
        return dict(num_layers=self.spec.num_hidden_layers, n_kv_heads=self.n_kv, head_dim=self.d)

    def set_kv_cache(self, kv_cache):
        self.kv_cache = kv_cache

    def _allreduce(self, x):
        if self.tp > 1:
            from ...comm.symmetric import small_all_reduce
            small_all_reduce(x, self.tp_group)  # one-shot over xGMI for decode-sized messages when enabled
        return x

    def _norm(self, x, w, b, residual=None):
        """norm(x) or the fused (norm(x + residual), x + residual) through the registered pre-norm module."""
        if residual is None:
            return self.norm_mod(x, None, w, b)[1]
        r, y = self.norm_mod(residual, x, w, b)
        return y, r

    def _act_name(self):
        a = self.spec.act
        return {"gelu_new": "gelu_tanh", "gelu_pytorch_tanh": "gelu_tanh"}.get(a, a)

    def _mlp(self, L, x):
        if L["w13"] is not None:
            return self._moe(L, x)
        return self.down_lin(self.up_lin(x, L["up.w"], L["up.b"]), L["down.w"], L["down.b"])

    def _moe(self, L, x):
        out = self.moe_mod(x, L["router.w"], L["w13"], L["w2"])
        if L["shared.w13"] is not None:
            s = F.linear(glu(F.linear(x, L["shared.w13"]), self._act_name()), L["shared.w2"])
            gate = torch.sigmoid(F.linear(x.float(), L["shared_gate.w"].float())).to(s.dtype)
            out = out + gate * s
        return out

    def _prep(self, batch):
        if getattr(batch, "atoms", None) is not None and batch.n_atoms is not None:
            return  # built with the rest of the metadata (RaggedBatchWrapper.finalize, csrc/host/ragged_meta.cpp)
        atoms, n_atoms = build_atoms(batch.seq_meta_host, self.n_q, self.n_kv)
        batch.atoms = atoms.to(self.device, non_blocking=True)
        batch.n_atoms = n_atoms

    def _embed(self, batch):
        return self.embed_mod(batch, self.embed, self.pos_embed)

    def _attn(self, i, L, x, batch, T, capture, lat, events, sink=None, qkv=None):
        nq, nkv, D = self.n_q, self.n_kv, self.d
        qkv = (self.qkv_lin(x, L["qkv.w"], L["qkv.b"]) if qkv is None else qkv).view(T, nq + 2 * nkv, D)
        if capture and self.latent_mode == "kv":
            if sink is not None:  # stored in stream order before RoPE rotates K in place: no clone
                sink(i, qkv[:, nq:].reshape(T, -1))
            else:
                self._d2h(qkv[:, nq:].reshape(T, -1).clone(), lat[i], events)  # pre-RoPE K|V
        o = self.attn_mod(qkv, self.kv_cache.get_cache(i), batch, self.cos, self.sin)
        return self.o_lin(o, L["o.w"], L["o.b"])

    def _fused_decode_ok(self, T):
        """Single-token decode steps of a plain pre-RMSNorm, SwiGLU-style dense model on the bf16 BLAS linears: the pre-norms
        and the gated activation run inside the projection GEMVs (ops/gemv.fused_gemv), so a layer launches neither
        the RMSNorm nor the GLU kernel (``HDS_V2_FUSED_DECODE=0``: the separate kernels)."""
        ok = getattr(self, "_fused_static", None)
        if ok is None:
            from .modules.implementations import BlasFPLinear, DSPreRMSNorm
            ok = (bool(self.layers) and _os.environ.get("HDS_V2_FUSED_DECODE", "1") == "1"
                  and self.device.type == "cuda"
                  and self.dtype == torch.bfloat16 and self.tp == 1 and self.spec.moe is None
                  and self.spec.parallel not in ("shared_ln", "two_ln") and self.spec.gated
                  and isinstance(self.norm_mod, DSPreRMSNorm) and self._act_name() == "silu"
                  and all(isinstance(m, BlasFPLinear) for m in (self.qkv_lin, self.up_lin))
                  and all(L[k] is None for L in self.layers for k in ("ln1.b", "ln2.b", "qkv.b", "up.b"))
                  and all(L[k] is not None and L[k].dtype == torch.bfloat16 and torch.is_tensor(L[k])
                          for L in self.layers for k in ("ln1.w", "ln2.w", "qkv.w", "up.w")))
            self._fused_static = ok
        # one token row only: at B = 4 the per-row normalisation inside the (already VALU-bound) GEMV made the step
        # slower than the separate RMSNorm kernel (732 vs 773 tok/s); at B = 1: 247 vs 234 (profiles/r6/fused_decode/)
        return ok and T == 1

    # ------------------------------------------------------------------------------------------
    def decode_graph_eligible(self, batch, capture_latents):
        """A decode-only ragged batch (one new token per sequence) of a dense model without tensor parallelism:
        its whole forward depends on the batch size alone, so it replays from a HIP graph captured per size. With
        ``capture_latents`` the graph also stores every layer's latent into a device ring (``_LatentRing``)."""
        if (self.device.type != "cuda" or (capture_latents and not self.decode_graph_latents) or self.tp != 1
                or self.spec.moe is not None or self.decode_graph_max_batch <= 0):
            return False
        S = batch.current_sequences
        return (0 < S <= self.decode_graph_max_batch and batch.current_tokens == S
                and getattr(batch, "atoms", None) is not None and getattr(batch, "_dev_meta", None) is not None)

    @torch.no_grad()
    def forward_decode_graph(self, batch, capture_latents=False):
        """Replay the decode step for ``batch.current_sequences`` sequences: the step's token ids and packed
        metadata (same layout as ``RaggedBatchWrapper.finalize``) are copied into the graph's static buffers, the
        graph replays every layer's kernels with one launch, and the logits are copied out. The first step of a
        batch size runs the forward eagerly once (it writes the same KV the replay writes) and captures it.

        ``capture_latents``: the graph also stores each layer's latent rows into a device ring slot (HCache during
        decode, reference llama_v2/model.py:211-218 captures in every forward); returns ``(logits, latents)`` with
        ``latents`` a pinned host view [L, B, W] that is complete once the ring has been drained
        (``drain_latents`` / the engine's ``wait_latents``). Without: ``(logits, None)``."""
        B = batch.current_sequences
        key = (B, bool(capture_latents))
        g = self._decode_graphs.get(key)
        n = batch.seq_meta.numel() + batch.tok_seq.numel() + batch.tok_pos.numel() + batch.last_token_idx.numel() \
            + batch.block_tables.numel() + batch.atoms.numel()
        if g is None:
            ring = _LatentRing(self, B, self.decode_latent_ring_steps) if capture_latents else None
            g = self._decode_graphs[key] = _DecodeGraph(self, batch, n, ring)
        g.ids.copy_(batch.input_ids, non_blocking=True)
        g.meta.copy_(batch._dev_meta[:n], non_blocking=True)
        view = g.ring.begin_step() if g.ring is not None else None
        if g.graph is None:
            g.capture(self)
        g.graph.replay()
        if g.ring is not None:
            g.ring.end_step()
        return g.out.clone(), view

    def latent_rings(self):
        return [g.ring for g in self._decode_graphs.values() if g.ring is not None]

    def drain_latents(self):
        """Issue the D2H of every decode-graph latent not on the host yet; returns the copy-stream event after which
        every latent returned so far is complete (None if nothing was pending)."""
        ev = None
        for r in self.latent_rings():
            e = r.drain_all()
            ev = e if e is not None else ev
        return ev

    @torch.no_grad()
    def forward(self, batch, capture_latents=True, sync_latents=True, sink=None):
        """Returns (logits [n_seqs, V], latents host [L, T, H] or [L, T, 2*n_kv*D] or None). With
        ``sync_latents=False`` the host does not wait for the latent D2H copies: ``self.latent_event`` (HIP event on
        the copy stream) marks when the returned host tensor is complete. ``sink(layer, rows)``: latents go to it
        instead of to host memory (the decode graph's device ring)."""
        spec = self.spec
        self._prep(batch)
        T = batch.current_tokens
        h = self._embed(batch)
        residual = None
        lat = None
        events = []
        if capture_latents and sink is None:
            lat = self._latent_buffer(spec.num_hidden_layers, T)
        emit = sink if sink is not None else (lambda i, t: self._d2h(t, lat[i], events))
        if self._fused_decode_ok(T):
            from ...ops.gemv import fused_gemv
            eps = spec.norm_eps
            want_x = capture_latents and self.latent_mode in ("hidden", "hidden_fp8", "hidden_int8")
            ring = getattr(sink, "__self__", None) if sink is not None else None
            stage = ring.stage() if (capture_latents and self.latent_mode == "hidden"
                                     and isinstance(ring, _LatentRing)) else None
            for i, L in enumerate(self.layers):
                # pre-norm + qkv in one GEMV; the new residual stream (and the normed rows for hidden latents) too --
                # in a decode graph written straight into the step's latent stage
                qkv, residual, x = fused_gemv(h, L["qkv.w"], residual, L["ln1.w"], eps, want_x=want_x,
                                              x_out=None if stage is None else stage[i])
                if stage is not None:
                    if x.data_ptr() != stage[i].data_ptr():
                        stage[i].copy_(x.view_as(stage[i]))
                elif capture_latents and self.latent_mode == "hidden":
                    emit(i, x)
                elif capture_latents and self.latent_mode == "hidden_fp8":
                    emit(i, self._pack_fp8(x))
                elif capture_latents and self.latent_mode == "hidden_int8":
                    emit(i, self._pack_int8(x))
                a = self._attn(i, L, None, batch, T, capture_latents, lat, events, sink, qkv=qkv)
                # post-attention norm + gate|up + SwiGLU in one GEMV, then the down projection
                g, residual, _ = fused_gemv(a, L["up.w"], residual, L["ln2.w"], eps, glu=True)
                h = self.down_lin(g, L["down.w"], L["down.b"])
            if stage is not None:
                ring.flush_stage()  # every layer's latent rows into the ring slot, one store
        for i, L in (enumerate(self.layers) if not self._fused_decode_ok(T) else ()):
            if residual is None:
                x = self._norm(h, L["ln1.w"], L["ln1.b"])
                residual = h
            else:
                x, residual = self._norm(h, L["ln1.w"], L["ln1.b"], residual)
            if capture_latents and self.latent_mode == "hidden":
                emit(i, x)
            elif capture_latents and self.latent_mode == "hidden_fp8":
                emit(i, self._pack_fp8(x))
            elif capture_latents and self.latent_mode == "hidden_int8":
                emit(i, self._pack_int8(x))
            a = self._attn(i, L, x, batch, T, capture_latents, lat, events, sink)
            if spec.parallel == "shared_ln":
                h = self._allreduce(a + self._mlp(L, x))
            elif spec.parallel == "two_ln":
                xm = self._norm(residual, L["ln2.w"], L["ln2.b"])
                h = self._allreduce(a + self._mlp(L, xm))
            else:
                x2, residual = self._norm(self._allreduce(a), L["ln2.w"], L["ln2.b"], residual)
                h = self._allreduce(self._mlp(L, x2))
        logits = self.unembed_mod(h, residual, batch, self.lm_head, self.lm_head_b, self.final_w, self.final_b,
                                  spec.norm_eps, self.tp_group, self.vocab)
        self.latent_event = events[-1] if events else None
        if events and sync_latents:
            events[-1].synchronize()
        return logits, lat

    _latent_pool = None

    INT8_GROUP = 128  # hidden_int8: one fp32 scale per 128 channels (3 % of the bytes)

    def latent_width(self):
        """Elements of one token-layer latent (bytes for the quantized modes)."""
        H = self.spec.hidden_size
        return {"hidden": H, "kv": 2 * self.n_kv * self.d, "hidden_fp8": H + 4,
                "hidden_int8": H + 4 * (H // self.INT8_GROUP)}[self.latent_mode]

    def _latent_buffer(self, n_layers, T):
        dtype = torch.uint8 if self.latent_mode in ("hidden_fp8", "hidden_int8") else self.dtype
        shape = (n_layers, T, self.latent_width())
        if self.device.type != "cuda":
            return torch.empty(shape, dtype=dtype)
        from ...offload.pinned import PinnedPool
        pool = RaggedTransformer._latent_pool
        if pool is None:
            pool = RaggedTransformer._latent_pool = PinnedPool()
        # back to the pool once the caller has dropped the latents and every per-sequence view of them
        return pool.get_tracked(shape[0] * shape[1] * shape[2], dtype).view(shape)

    def _pack_fp8(self, x):
        """[T, H] activations -> [T, H + 4] uint8: e4m3 values, then the token's fp32 scale as 4 bytes."""
        from ...ops.quantizer import quantize_fp8
        T, H = x.shape
        q, sc = quantize_fp8(x, group_size=H)
        pk = torch.empty(T, H + 4, dtype=torch.uint8, device=x.device)
        pk[:, :H].copy_(q.view(T, H))
        pk[:, H:].copy_(sc.view(torch.uint8).view(T, 4))
        return pk

    def _pack_int8(self, x):
        """[T, H] -> [T, H + 4H/128] uint8: symmetric int8 with an fp32 scale per 128 channels (higher SNR than
        e4m3 for near-Gaussian activations: uniform 8-bit steps instead of a 3-bit mantissa)."""
        from ...ops.quantizer import quantize
        T, H = x.shape
        G = self.INT8_GROUP
        q, sc, _ = quantize(x, group_size=G, bits=8, symmetric=True)
        pk = torch.empty(T, H + 4 * (H // G), dtype=torch.uint8, device=x.device)
        pk[:, :H].copy_(q.view(torch.uint8).view(T, H))
        pk[:, H:].copy_(sc.view(torch.uint8).view(T, 4 * (H // G)))
        return pk

    def _unpack_int8(self, pk):
        from ...ops.quantizer import dequantize
        G = self.INT8_GROUP
        T, W = pk.shape
        H = W * G // (G + 4)
        q = pk[:, :H].contiguous().view(torch.int8).view(-1)
        sc = pk[:, H:].contiguous().view(torch.float32).view(-1)
        return dequantize(q, sc, group_size=G, bits=8, symmetric=True, dtype=self.dtype).view(T, H)

    def _unpack_fp8(self, pk):
        from ...ops.quantizer import dequantize_fp8
        T, W = pk.shape
        H = W - 4
        q = pk[:, :H].contiguous().view(-1)
        sc = pk[:, H:].contiguous().view(torch.float32).view(-1)
        return dequantize_fp8(q, sc, group_size=H, dtype=self.dtype).view(T, H)

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
        """Rebuild the paged KV of ``batch``'s sequences from host latents: one [L, T, W] tensor or a list of
        per-sequence [L, n_s, W] pieces in batch order (pinned preferred). Pieces are copied straight into the
        device layer buffer at their row offsets: no host-side concatenation (a pageable temporary that would also
        have to be re-pinned — 2 extra host copies of every latent byte)."""
        T = batch.current_tokens
        L_ = self.spec.num_hidden_layers
        pieces = list(latents) if isinstance(latents, (list, tuple)) else [latents]
        if self.copy_stream is None:
            for i, L in enumerate(self.layers):
                x = torch.cat([p[i] for p in pieces], 0) if len(pieces) > 1 else pieces[0][i]
                self._restore_layer(i, L, x.to(self.device), batch, T)
            return
        pieces = [p if p.device.type != "cpu" or p.is_pinned() else p.pin_memory() for p in pieces]
        offs = [0]
        for p in pieces:
            offs.append(offs[-1] + p.shape[1])
        assert offs[-1] == T, "latents must cover exactly the batch's tokens"
        width = pieces[0].shape[-1]
        bufs = [torch.empty(T, width, dtype=pieces[0].dtype, device=self.device) for _ in range(2)]
        loaded = [torch.cuda.Event() for _ in range(2)]
        freed = [torch.cuda.Event() for _ in range(2)]
        main = torch.cuda.current_stream()

        def issue(i):
            b = i & 1
            with torch.cuda.stream(self.copy_stream):
                if i >= 2:
                    self.copy_stream.wait_event(freed[b])
                for p, o0, o1 in zip(pieces, offs[:-1], offs[1:]):
                    bufs[b][o0:o1].copy_(p[i], non_blocking=True)
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
        if self.latent_mode == "hidden_fp8":
            x = self._unpack_fp8(x)
        elif self.latent_mode == "hidden_int8":
            x = self._unpack_int8(x)
        if self.latent_mode in ("hidden", "hidden_fp8", "hidden_int8"):
            # only the K|V rows of the projection are needed: GEMM against the k/v slice of W_qkv
            if isinstance(L["qkv.w"], _PackedWeight):  # packed rows cannot be sliced: full projection
                kv = self.qkv_lin(x, L["qkv.w"], L["qkv.b"]).view(T, nq + 2 * nkv, D)[:, nq:].contiguous()
            else:
                w = L["qkv.w"][nq * D:]
                bias = L["qkv.b"][nq * D:] if L["qkv.b"] is not None else None
                kv = F.linear(x, w, bias).view(T, 2 * nkv, D)
        else:
            kv = x.view(T, 2 * nkv, D).contiguous()  # stored pre-RoPE: rotation happens on the way in
        kv_rope_scatter(kv, cache, batch.tok_seq, batch.tok_pos, batch.block_tables, self.cos, self.sin, 0, nkv,
                        rotate_q=False, do_rope=self.cos is not None, rotary_dim=self.rot)


class _LatentRing:
    """Device ring of HCache latents written by a captured decode graph, drained to pinned host memory in bulk.

    Layout [2R, L, B, W] (R = ``decode_latent_ring_steps``): two halves of R decode steps. The graph stores layer i's
    latent rows at ``ring[slot, i]`` with ``slot`` read from device memory (ops/hostcopy.latent_slot_store) and
    advances ``slot`` as its last kernel, so each replay fills the next slot without any host work. The host mirrors
    the slot: when a half is full it is drained with ONE D2H on the copy stream (instead of L per-layer copies per
    token) into a pinned chunk [R, L, B, W] from the pool, while the graph fills the other half; ``drain_all`` also
    flushes a partly filled half (the engine's ``wait_latents`` / evict / restore). Before a half is written again
    the compute stream waits for its previous D2H (GPU-side). Each step's latents are returned as the view
    ``chunk[k]`` [L, B, W] of its half's chunk; chunks return to the pool when the caller drops every view."""

    def __init__(self, model, B, steps):
        self.model = model
        self.R = max(1, int(steps))
        L = model.spec.num_hidden_layers
        self.dtype = torch.uint8 if model.latent_mode in ("hidden_fp8", "hidden_int8") else model.dtype
        self.shape = (L, B, model.latent_width())
        self.dev = torch.empty((2 * self.R, ) + self.shape, dtype=self.dtype, device=model.device)
        self.slot = torch.zeros(1, dtype=torch.int32, device=model.device)
        self.host_slot = 0
        self.chunk = [None, None]
        self.filled = [0, 0]  # slots of each half written since the half was (re)started
        self.drained = [0, 0]  # of those, slots already copied to the chunk
        self.done = [None, None]  # copy-stream event of each half's last D2H
        self.fresh = [True, True]

    def sink(self, i, rows):
        from ...ops.hostcopy import latent_slot_store
        latent_slot_store(rows, self.dev, self.slot, i)

    def stage(self):
        """[L, B, W] device buffer the fused decode projections write every layer's latent rows into directly (the
        normed rows are produced there, no per-layer store kernel); ``flush_stage`` moves it into the ring slot with
        one store at the end of the step."""
        st = getattr(self, "_stage", None)
        if st is None:
            st = self._stage = torch.empty(self.shape, dtype=self.dtype, device=self.dev.device)
        return st

    def flush_stage(self):
        from ...ops.hostcopy import latent_slot_store
        L, B, W = self.shape
        latent_slot_store(self._stage.view(L * B, W), self.dev.view(2 * self.R, 1, L * B, W), self.slot, 0)

    def advance(self):
        from ...ops.hostcopy import slot_advance
        slot_advance(self.slot, 2 * self.R)

    def begin_step(self):
        h, k = divmod(self.host_slot, self.R)
        if self.fresh[h]:
            if self.done[h] is not None:  # the previous D2H out of this half must finish before the graph rewrites it
                torch.cuda.current_stream().wait_event(self.done[h])
            pool = RaggedTransformer._latent_pool
            if pool is None:
                from ...offload.pinned import PinnedPool
                pool = RaggedTransformer._latent_pool = PinnedPool()
            n = self.R * self.shape[0] * self.shape[1] * self.shape[2]
            self.chunk[h] = pool.get_tracked(n, self.dtype).view((self.R, ) + self.shape)
            self.filled[h] = self.drained[h] = 0
            self.fresh[h] = False
        return self.chunk[h][k]

    def end_step(self):
        h = self.host_slot // self.R
        self.filled[h] += 1
        self.host_slot = (self.host_slot + 1) % (2 * self.R)
        if self.filled[h] == self.R:
            self._drain(h)
            self.fresh[h] = True

    def _drain(self, h):
        a, b = self.drained[h], self.filled[h]
        if b <= a:
            return None
        cs = self.model.copy_stream
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(cs):
            cs.wait_event(ev)
            self.chunk[h][a:b].copy_(self.dev[h * self.R + a:h * self.R + b], non_blocking=True)
            done = torch.cuda.Event()
            done.record(cs)
        self.drained[h] = b
        self.done[h] = done
        return done

    def drain_all(self):
        """Flush both halves (the older one first); the returned event covers every latent returned so far."""
        cur = self.host_slot // self.R
        ev = None
        for h in (1 - cur, cur):
            e = self._drain(h)
            ev = e if e is not None else ev
        return ev

    def pending(self):
        return any(self.filled[h] > self.drained[h] for h in (0, 1))


class _DecodeGraph:
    """Static inputs, captured graph and output of one decode batch size (RaggedTransformer.forward_decode_graph),
    with its latent ring when the graph captures HCache latents."""

    def __init__(self, model, batch, n, ring=None):
        self.ring = ring
        dev = model.device
        B = batch.current_sequences
        mb = batch.block_tables.shape[1]
        A = batch.n_atoms
        self.ids = torch.zeros(B, dtype=batch.input_ids.dtype, device=dev)
        self.meta = torch.zeros(n, dtype=torch.int32, device=dev)
        o = 0

        def take(k, shape):
            nonlocal o
            v = self.meta[o:o + k].view(*shape)
            o += k
            return v

        sb = types.SimpleNamespace()
        sb.input_ids = self.ids
        sb.seq_meta = take(3 * B, (B, 3))
        sb.tok_seq = take(B, (B, ))
        sb.tok_pos = take(B, (B, ))
        sb.last_token_idx = take(B, (B, ))
        sb.block_tables = take(B * mb, (B, mb))
        sb.atoms = take(3 * A, (A, 3))
        sb.n_atoms = A
        sb.current_tokens = B
        sb.current_sequences = B
        sb.seq_meta_host = None
        sb.tables_host = None
        self.batch = sb
        self.graph = None
        self.out = None

    def capture(self, model):
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        cap = self.ring is not None
        sink = self.ring.sink if cap else None
        with torch.cuda.stream(side):
            # warm-up: hipBLASLt / GEMV handles, KV (idempotent); its latents go to the slot the replay rewrites
            model.forward(self.batch, capture_latents=cap, sink=sink)
        cur.wait_stream(side)
        if model._graph_pool is None:
            model._graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        # no Python GC while capturing: a collection that frees another engine's CUDAGraph calls hipGraphDestroy, which
        # is not permitted while a stream captures (the capture and the process abort)
        import gc
        was_enabled = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            with torch.cuda.graph(g, pool=model._graph_pool):
                self.out, _ = model.forward(self.batch, capture_latents=cap, sink=sink)
                if cap:
                    self.ring.advance()
        finally:
            if was_enabled:
                gc.enable()
        self.graph = g
