"""Architecture policies for the ragged serving engine: HF config -> ArchSpec, HF state dict -> canonical weights.

Reference parity: inference/v2/engine_factory.py (``build_hf_engine`` :69-130 policy selection by ``model_type``)
and model_implementations/{llama_v2, mistral, mixtral, qwen, qwen_v2, qwen_v2_moe, phi, phi3, falcon, opt}/
(containers mapping HF parameter names, ``policy.py`` per family). One decoder implementation
(model.RaggedTransformer) covers every family through the flags below; the HCache latent contract
(``put`` returns per-layer latents, ``restore_kv`` rebuilds the paged KV) holds for all of them.

Canonical per-layer weight names: ln1.{w,b}, ln2.{w,b} (absent for shared-norm parallel blocks), qkv.{w,b}
(q rows, then k, then v), o.{w,b}, up.{w,b} (gated MLPs: gate rows then up rows), down.{w,b}; MoE layers:
router.w [E, H], w13 [E, 2I, H], w2 [E, H, I], optional shared.{w13, w2} and shared_gate.w [1, H].
"""
from dataclasses import dataclass, field
from typing import Optional

import torch


@dataclass
class ArchSpec:
    model_type: str
    vocab_size: int
    hidden_size: int
    num_hidden_layers: int
    num_attention_heads: int
    num_key_value_heads: int
    head_dim: int
    intermediate_size: int
    norm: str = "rms"                  # rms | ln
    norm_eps: float = 1e-6
    act: str = "silu"                  # silu | gelu | gelu_tanh | relu
    gated: bool = True
    parallel: Optional[str] = None     # None | "shared_ln" (phi, falcon-7b) | "two_ln" (falcon new arch)
    pos: str = "rope"                  # rope | learned
    pos_offset: int = 0                # OPT learned positions start at 2
    rotary_dim: int = 0                # 0 = full head_dim
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    max_position_embeddings: int = 4096
    sliding_window: int = 0
    tie_embeddings: bool = False
    lm_head_bias: bool = False
    moe: Optional[dict] = None         # {num_experts, top_k, normalize, shared}
    extra: dict = field(default_factory=dict)

    # LlamaConfig-compatible aliases used by the engine / KV cache sizing
    @property
    def rms_norm_eps(self):
        return self.norm_eps

    @property
    def hidden_act(self):
        return self.act


def _g(hf, *names, default=None):
    for n in names:
        if n in hf and hf[n] is not None:
            return hf[n]
    return default


def spec_from_hf(hf):
    rp = hf.get("rope_parameters")
    if isinstance(rp, dict):  # transformers>=5 nests the RoPE fields
        flat = {k: rp[k] for k in ("rope_theta", "partial_rotary_factor") if k in rp}
        if rp.get("rope_type", "default") != "default":
            flat["rope_scaling"] = rp
        hf = {**flat, **{k: v for k, v in hf.items() if v is not None}}
    mt = hf.get("model_type", "llama")
    H = _g(hf, "hidden_size", "n_embd", "d_model")
    nh = _g(hf, "num_attention_heads", "n_head", "num_heads")
    nkv = _g(hf, "num_key_value_heads", default=nh)
    L = _g(hf, "num_hidden_layers", "n_layer", "num_layers")
    V = hf["vocab_size"]
    hd = _g(hf, "head_dim", default=H // nh) or H // nh
    common = dict(model_type=mt, vocab_size=V, hidden_size=H, num_hidden_layers=L, num_attention_heads=nh,
                  num_key_value_heads=nkv, head_dim=hd, rope_theta=float(_g(hf, "rope_theta", default=10000.0)),
                  rope_scaling=hf.get("rope_scaling"),
                  max_position_embeddings=int(_g(hf, "max_position_embeddings", "n_positions", default=4096)),
                  tie_embeddings=bool(hf.get("tie_word_embeddings", False)))
    if mt in ("llama", "mistral", "qwen2", "mixtral", "qwen2_moe", "phi3"):
        spec = ArchSpec(**common, intermediate_size=hf.get("intermediate_size", 4 * H), norm="rms",
                        norm_eps=float(_g(hf, "rms_norm_eps", default=1e-6)), act="silu", gated=True,
                        sliding_window=int(hf.get("sliding_window") or 0) if hf.get("use_sliding_window", True) else 0)
        if mt == "mixtral":
            spec.moe = dict(num_experts=hf["num_local_experts"], top_k=hf["num_experts_per_tok"], normalize=True,
                            shared=False)
        if mt == "qwen2_moe":
            spec.intermediate_size = hf["moe_intermediate_size"]
            spec.moe = dict(num_experts=hf["num_experts"], top_k=hf["num_experts_per_tok"],
                            normalize=bool(hf.get("norm_topk_prob", False)), shared=True,
                            shared_intermediate_size=hf["shared_expert_intermediate_size"])
        if mt == "phi3" and hf.get("partial_rotary_factor", 1.0) < 1.0:
            spec.rotary_dim = int(hd * hf["partial_rotary_factor"])
        return spec
    if mt == "falcon":
        new_arch = bool(hf.get("new_decoder_architecture", False))
        kv = nkv if new_arch else (1 if hf.get("multi_query", True) else nh)
        if new_arch:
            kv = _g(hf, "num_kv_heads", default=nh)
        return ArchSpec(**{**common, "num_key_value_heads": kv}, intermediate_size=hf.get("ffn_hidden_size") or 4 * H,
                        norm="ln", norm_eps=float(_g(hf, "layer_norm_epsilon", default=1e-5)), act="gelu", gated=False,
                        parallel="two_ln" if new_arch else ("shared_ln" if hf.get("parallel_attn", True) else None),
                        pos="rope" if not hf.get("alibi", False) else "alibi",
                        extra={"bias": bool(hf.get("bias", False))})
    if mt == "phi":
        return ArchSpec(**common, intermediate_size=hf.get("intermediate_size", 4 * H), norm="ln",
                        norm_eps=float(_g(hf, "layer_norm_eps", default=1e-5)), act="gelu_tanh", gated=False,
                        parallel="shared_ln", rotary_dim=int(hd * float(hf.get("partial_rotary_factor", 0.5))),
                        lm_head_bias=True)
    if mt == "opt":
        return ArchSpec(**{**common, "num_key_value_heads": nh, "tie_embeddings": True}, intermediate_size=hf["ffn_dim"],
                        norm="ln", norm_eps=1e-5, act=hf.get("activation_function", "relu"), gated=False,
                        pos="learned", pos_offset=2,
                        extra={"pre_ln": bool(hf.get("do_layer_norm_before", True))})
    if mt == "qwen":
        return ArchSpec(**{**common, "num_key_value_heads": nh}, intermediate_size=hf["intermediate_size"] // 2,
                        norm="rms", norm_eps=float(_g(hf, "layer_norm_epsilon", default=1e-6)), act="silu",
                        gated=True, rope_theta=float(hf.get("rotary_emb_base", 10000.0)))
    raise NotImplementedError(f"model_type {mt} is not supported by the serving engine")


# ---------------------------------------------------------------------------------------------
def _cat(*xs):
    xs = [x for x in xs if x is not None]
    return torch.cat(xs, 0) if xs else None


def _experts(sd, m, E, gate, up, down):
    """Stacked [E, 2I, H] gate|up and [E, H, I] down weights from either checkpoint layout: per-expert
    Linear weights (``experts.{e}.w1.weight`` on disk) or the fused ``experts.gate_up_proj`` /
    ``experts.down_proj`` tensors of in-memory transformers>=5 models (same gate-then-up order)."""
    if m + "gate_up_proj" in sd:
        return sd[m + "gate_up_proj"], sd[m + "down_proj"]
    w13 = torch.stack([_cat(sd[f"{m}{e}.{gate}.weight"], sd[f"{m}{e}.{up}.weight"]) for e in range(E)])
    return w13, torch.stack([sd[f"{m}{e}.{down}.weight"] for e in range(E)])


def convert_hf(sd, spec):
    """HF state dict -> {"embed", "pos_embed", "final.w", "final.b", "lm_head.w", "lm_head.b", "layers": [...]}"""
    mt = spec.model_type
    out = {"layers": []}
    g = sd.get
    if mt in ("llama", "mistral", "qwen2", "mixtral", "qwen2_moe", "phi3"):
        out["embed"] = sd["model.embed_tokens.weight"]
        out["final.w"] = sd["model.norm.weight"]
        out["lm_head.w"] = g("lm_head.weight", sd["model.embed_tokens.weight"])
        for i in range(spec.num_hidden_layers):
            p = f"model.layers.{i}."
            L = {"ln1.w": sd[p + "input_layernorm.weight"], "ln2.w": sd[p + "post_attention_layernorm.weight"]}
            if p + "self_attn.qkv_proj.weight" in sd:
                L["qkv.w"] = sd[p + "self_attn.qkv_proj.weight"]
            else:
                L["qkv.w"] = _cat(sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"],
                                  sd[p + "self_attn.v_proj.weight"])
                if p + "self_attn.q_proj.bias" in sd:
                    L["qkv.b"] = _cat(sd[p + "self_attn.q_proj.bias"], sd[p + "self_attn.k_proj.bias"],
                                      sd[p + "self_attn.v_proj.bias"])
            L["o.w"] = sd[p + "self_attn.o_proj.weight"]
            if mt == "mixtral":
                m = p + ("block_sparse_moe." if p + "block_sparse_moe.gate.weight" in sd else "mlp.")
                L["router.w"] = sd[m + "gate.weight"]
                L["w13"], L["w2"] = _experts(sd, m + "experts.", spec.moe["num_experts"], "w1", "w3", "w2")
            elif mt == "qwen2_moe" and p + "mlp.gate.weight" in sd:
                m = p + "mlp."
                L["router.w"] = sd[m + "gate.weight"]
                L["w13"], L["w2"] = _experts(sd, m + "experts.", spec.moe["num_experts"], "gate_proj", "up_proj",
                                             "down_proj")
                L["shared.w13"] = _cat(sd[m + "shared_expert.gate_proj.weight"], sd[m + "shared_expert.up_proj.weight"])
                L["shared.w2"] = sd[m + "shared_expert.down_proj.weight"]
                L["shared_gate.w"] = sd[m + "shared_expert_gate.weight"]
            elif p + "mlp.gate_up_proj.weight" in sd:
                L["up.w"] = sd[p + "mlp.gate_up_proj.weight"]
                L["down.w"] = sd[p + "mlp.down_proj.weight"]
            else:
                L["up.w"] = _cat(sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"])
                L["down.w"] = sd[p + "mlp.down_proj.weight"]
            out["layers"].append(L)
        return out
    if mt == "falcon":
        out["embed"] = sd["transformer.word_embeddings.weight"]
        out["final.w"], out["final.b"] = sd["transformer.ln_f.weight"], g("transformer.ln_f.bias")
        out["lm_head.w"] = g("lm_head.weight", out["embed"])
        for i in range(spec.num_hidden_layers):
            p = f"transformer.h.{i}."
            L = {}
            if spec.parallel == "two_ln":
                L["ln1.w"], L["ln1.b"] = sd[p + "ln_attn.weight"], g(p + "ln_attn.bias")
                L["ln2.w"], L["ln2.b"] = sd[p + "ln_mlp.weight"], g(p + "ln_mlp.bias")
            else:
                L["ln1.w"], L["ln1.b"] = sd[p + "input_layernorm.weight"], g(p + "input_layernorm.bias")
                if spec.parallel is None:
                    L["ln2.w"], L["ln2.b"] = sd[p + "post_attention_layernorm.weight"], \
                        g(p + "post_attention_layernorm.bias")
            qkv = sd[p + "self_attention.query_key_value.weight"]
            nq, nkv, D = spec.num_attention_heads, spec.num_key_value_heads, spec.head_dim
            if spec.parallel == "two_ln" or (nkv != 1 and nkv != nq):
                # grouped layout: [kv_group][q..., k, v] -> q | k | v
                G = nq // nkv
                w = qkv.view(nkv, G + 2, D, -1)
                qkv = torch.cat([w[:, :G].reshape(nq * D, -1), w[:, G].reshape(nkv * D, -1),
                                 w[:, G + 1].reshape(nkv * D, -1)], 0)
            elif nkv == nq:
                w = qkv.view(nq, 3, D, -1)
                qkv = torch.cat([w[:, 0].reshape(nq * D, -1), w[:, 1].reshape(nq * D, -1),
                                 w[:, 2].reshape(nq * D, -1)], 0)
            L["qkv.w"] = qkv
            L["o.w"] = sd[p + "self_attention.dense.weight"]
            L["up.w"], L["up.b"] = sd[p + "mlp.dense_h_to_4h.weight"], g(p + "mlp.dense_h_to_4h.bias")
            L["down.w"], L["down.b"] = sd[p + "mlp.dense_4h_to_h.weight"], g(p + "mlp.dense_4h_to_h.bias")
            out["layers"].append(L)
        return out
    if mt == "phi":
        out["embed"] = sd["model.embed_tokens.weight"]
        out["final.w"], out["final.b"] = sd["model.final_layernorm.weight"], sd["model.final_layernorm.bias"]
        out["lm_head.w"], out["lm_head.b"] = sd["lm_head.weight"], g("lm_head.bias")
        for i in range(spec.num_hidden_layers):
            p = f"model.layers.{i}."
            a = p + "self_attn."
            out["layers"].append({
                "ln1.w": sd[p + "input_layernorm.weight"], "ln1.b": sd[p + "input_layernorm.bias"],
                "qkv.w": _cat(sd[a + "q_proj.weight"], sd[a + "k_proj.weight"], sd[a + "v_proj.weight"]),
                "qkv.b": _cat(sd[a + "q_proj.bias"], sd[a + "k_proj.bias"], sd[a + "v_proj.bias"]),
                "o.w": sd[a + "dense.weight"], "o.b": sd[a + "dense.bias"],
                "up.w": sd[p + "mlp.fc1.weight"], "up.b": sd[p + "mlp.fc1.bias"],
                "down.w": sd[p + "mlp.fc2.weight"], "down.b": sd[p + "mlp.fc2.bias"]})
        return out
    if mt == "opt":
        pre = "model.decoder."
        out["embed"] = sd[pre + "embed_tokens.weight"]
        out["pos_embed"] = sd[pre + "embed_positions.weight"]
        out["final.w"], out["final.b"] = g(pre + "final_layer_norm.weight"), g(pre + "final_layer_norm.bias")
        out["lm_head.w"] = g("lm_head.weight", out["embed"])
        for i in range(spec.num_hidden_layers):
            p = f"{pre}layers.{i}."
            a = p + "self_attn."
            out["layers"].append({
                "ln1.w": sd[p + "self_attn_layer_norm.weight"], "ln1.b": sd[p + "self_attn_layer_norm.bias"],
                "ln2.w": sd[p + "final_layer_norm.weight"], "ln2.b": sd[p + "final_layer_norm.bias"],
                "qkv.w": _cat(sd[a + "q_proj.weight"], sd[a + "k_proj.weight"], sd[a + "v_proj.weight"]),
                "qkv.b": _cat(sd[a + "q_proj.bias"], sd[a + "k_proj.bias"], sd[a + "v_proj.bias"]),
                "o.w": sd[a + "out_proj.weight"], "o.b": sd[a + "out_proj.bias"],
                "up.w": sd[p + "fc1.weight"], "up.b": sd[p + "fc1.bias"],
                "down.w": sd[p + "fc2.weight"], "down.b": sd[p + "fc2.bias"]})
        return out
    if mt == "qwen":
        out["embed"] = sd["transformer.wte.weight"]
        out["final.w"] = sd["transformer.ln_f.weight"]
        out["lm_head.w"] = g("lm_head.weight", out["embed"])
        for i in range(spec.num_hidden_layers):
            p = f"transformer.h.{i}."
            out["layers"].append({
                "ln1.w": sd[p + "ln_1.weight"], "ln2.w": sd[p + "ln_2.weight"],
                "qkv.w": sd[p + "attn.c_attn.weight"], "qkv.b": g(p + "attn.c_attn.bias"),
                "o.w": sd[p + "attn.c_proj.weight"],
                # Qwen-1: intermediate = w1(x) * silu(w2(x)) -> gate = w2, up = w1
                "up.w": _cat(sd[p + "mlp.w2.weight"], sd[p + "mlp.w1.weight"]),
                "down.w": sd[p + "mlp.c_proj.weight"]})
        return out
    raise NotImplementedError(mt)


def spec_from_llama_config(cfg):
    """This framework's own LlamaConfig / MixtralConfig -> ArchSpec."""
    moe = None
    if getattr(cfg, "num_local_experts", 0):
        moe = dict(num_experts=cfg.num_local_experts, top_k=cfg.num_experts_per_tok, normalize=True, shared=False)
    return ArchSpec(model_type=getattr(cfg, "model_type", "llama"), vocab_size=cfg.vocab_size,
                    hidden_size=cfg.hidden_size, num_hidden_layers=cfg.num_hidden_layers,
                    num_attention_heads=cfg.num_attention_heads, num_key_value_heads=cfg.num_key_value_heads,
                    head_dim=cfg.head_dim, intermediate_size=cfg.intermediate_size, norm="rms",
                    norm_eps=cfg.rms_norm_eps, act=cfg.hidden_act, gated=True, rope_theta=cfg.rope_theta,
                    rope_scaling=cfg.rope_scaling, max_position_embeddings=cfg.max_position_embeddings,
                    sliding_window=cfg.sliding_window or 0, tie_embeddings=cfg.tie_word_embeddings, moe=moe)


def convert_own_llama(sd, spec):
    """State dict of models.llama.LlamaForCausalLM / models.mixtral.MixtralForCausalLM -> canonical."""
    out = {"layers": []}
    if "model.embed_tokens.weight" in sd:  # Llama
        out["embed"], out["final.w"] = sd["model.embed_tokens.weight"], sd["model.norm.weight"]
        pre = "model.layers."
    else:  # Mixtral (flat names)
        out["embed"], out["final.w"] = sd["embed_tokens.weight"], sd["norm.weight"]
        pre = "layers."
    out["lm_head.w"] = sd.get("lm_head.weight", out["embed"])
    for i in range(spec.num_hidden_layers):
        p = f"{pre}{i}."
        L = {"ln1.w": sd[p + "input_layernorm.weight"], "ln2.w": sd[p + "post_attention_layernorm.weight"],
             "qkv.w": sd[p + "self_attn.qkv_proj.weight"], "qkv.b": sd.get(p + "self_attn.qkv_proj.bias"),
             "o.w": sd[p + "self_attn.o_proj.weight"]}
        if p + "mlp.gate_up_proj.weight" in sd:
            L["up.w"], L["down.w"] = sd[p + "mlp.gate_up_proj.weight"], sd[p + "mlp.down_proj.weight"]
        else:
            m = p + "block_sparse_moe.deepspeed_moe."
            L["router.w"] = sd[m + "gate.wg.weight"]
            L["w13"], L["w2"] = sd[m + "experts.w13"], sd[m + "experts.w2"]
        out["layers"].append(L)
    return out
