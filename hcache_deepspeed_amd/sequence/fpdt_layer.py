"""``deepspeed.sequence.fpdt_layer`` import path (reference deepspeed/sequence/fpdt_layer.py)."""
from ..parallel.fpdt import (FPDT_Attention, FPDT_FFN, FPDT_LogitsLoss, FPDTInputConstruct,  # noqa: F401
                             fpdt_attention)
