"""DeepSpeed4Science ops (reference deepspeed/ops/deepspeed4science)."""
from .evoformer_attn import DS4Sci_EvoformerAttention, EvoformerFusedAttention  # noqa: F401
