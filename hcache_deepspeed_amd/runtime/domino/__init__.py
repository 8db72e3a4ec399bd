"""Reference import path (deepspeed/runtime/domino): Domino TP overlap lives in parallel/domino.py."""
from ...parallel.domino import DominoTransformer, domino_layer_forward, enable_domino  # noqa: F401
