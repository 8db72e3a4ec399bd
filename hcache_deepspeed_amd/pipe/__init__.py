"""``deepspeed.pipe`` import path (reference deepspeed/pipe/__init__.py)."""
from ..runtime.pipe.module import LayerSpec, PipelineModule, TiedLayerSpec  # noqa: F401
from ..runtime.pipe.topology import ProcessTopology  # noqa: F401
