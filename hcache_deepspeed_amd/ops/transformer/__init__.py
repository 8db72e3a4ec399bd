"""Fused training transformer layer (reference deepspeed/ops/transformer)."""
from .transformer import DeepSpeedTransformerConfig, DeepSpeedTransformerLayer, TransformerConfig  # noqa: F401
