from .config import LoRAConfig, QuantizationConfig
from .optimized_linear import LoRAOptimizedLinear, OptimizedLinear
from .quantization import QuantizedLinear, QuantizedParameter

__all__ = ["LoRAConfig", "QuantizationConfig", "OptimizedLinear", "LoRAOptimizedLinear", "QuantizedLinear",
           "QuantizedParameter"]
