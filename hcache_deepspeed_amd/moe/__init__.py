"""``deepspeed.moe`` import path (reference deepspeed/moe/)."""
