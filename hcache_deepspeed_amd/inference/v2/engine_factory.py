"""``deepspeed.inference.v2.engine_factory`` import path (reference inference/v2/engine_factory.py:32,69)."""
from .engine import build_engine_from_ds_checkpoint, build_hf_engine  # noqa: F401
