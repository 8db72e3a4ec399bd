"""``deepspeed.ops.fp_quantizer`` import path (reference ops/fp_quantizer/__init__.py)."""
from ..quantizer import FP_Quantize  # noqa: F401
