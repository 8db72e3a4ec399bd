"""``deepspeed.sequence.layer`` import path (reference deepspeed/sequence/layer.py:311)."""
from ..parallel.ulysses import DistributedAttention, _SeqAllToAll  # noqa: F401
