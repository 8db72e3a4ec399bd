"""``deepspeed.sequence`` import path (reference deepspeed/sequence/)."""
