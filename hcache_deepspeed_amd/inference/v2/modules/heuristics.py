"""Implementation selection for the inference-v2 modules (reference inference/v2/modules/heuristics.py
:36-195). The engine config's ``quantization.quantization_mode`` picks the weight-only linear ("wf6af16" -> FP6,
"int8"/"int4" -> group INT); everything else has one MI355X implementation per interface today, chosen here so
that adding a variant (e.g. an FP8 prefill GEMM) touches only this file and the registry."""
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig)
from .interfaces import (DSEmbeddingRegistry, DSLinearRegistry, DSMoERegistry, DSPostNormRegistry, DSPreNormRegistry,
                         DSSelfAttentionRegistry, DSUnembedRegistry)
from .module_registry import ConfigBundle
from . import implementations  # noqa: F401  (registers the implementations)


def _qmode(engine_config):
    q = getattr(engine_config, "quantization", None) or {}
    if not isinstance(q, dict):
        q = getattr(q, "__dict__", {})
    return q.get("quantization_mode")


def instantiate_attention(attention_config: DSSelfAttentionConfig, engine_config=None):
    return DSSelfAttentionRegistry.instantiate_config(ConfigBundle("dense_blocked_attention", attention_config))


def instantiate_embed(embed_config: DSEmbeddingsConfig, engine_config=None):
    return DSEmbeddingRegistry.instantiate_config(ConfigBundle("ragged_embedding", embed_config))


def instantiate_linear(linear_config: DSLinearConfig, engine_config=None):
    mode = linear_config.quantization_mode or _qmode(engine_config)
    linear_config.quantization_mode = mode
    if mode is None:
        name = "blas_fp_linear"
    elif mode == "wf6af16":
        name = "quantized_wf6af16_linear"
    elif mode in ("int8", "int4"):
        name = "quantized_int_linear"
    else:
        raise ValueError(f"Unsupported quantization_mode {mode!r} (wf6af16 | int8 | int4)")
    if not DSLinearRegistry.registry[name].supports_config(linear_config):
        linear_config.quantization_mode = None  # shapes the quantized kernels cannot take stay bf16
        name = "blas_fp_linear"
    return DSLinearRegistry.instantiate_config(ConfigBundle(name, linear_config))


def instantiate_moe(moe_config: DSMoEConfig, engine_config=None):
    return DSMoERegistry.instantiate_config(ConfigBundle("grouped_gemm_moe", moe_config))


def instantiate_post_norm(norm_config: DSNormConfig, engine_config=None):
    return DSPostNormRegistry.instantiate_config(ConfigBundle("ds_post_ln", norm_config))


def instantiate_pre_norm(norm_config: DSNormConfig, engine_config=None):
    name = "ds_pre_rms" if norm_config.type == "rms" else "ds_pre_ln"
    return DSPreNormRegistry.instantiate_config(ConfigBundle(name, norm_config))


def instantiate_unembed(unembed_config: DSUnembedConfig, engine_config=None):
    return DSUnembedRegistry.instantiate_config(ConfigBundle("ragged_unembed", unembed_config))
