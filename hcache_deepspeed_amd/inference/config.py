"""``init_inference`` configuration (reference inference/config.py ``DeepSpeedInferenceConfig`` and its
sub-configs: tensor_parallel, quant, moe, checkpoint). Unknown keys are kept in ``extra`` so configs
written for the reference load unchanged."""
from dataclasses import asdict, dataclass, field

import torch

_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "float": torch.float32, "fp16": torch.float16,
           "float16": torch.float16, "half": torch.float16, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           "int8": torch.int8}


@dataclass
class DeepSpeedTPConfig:
    enabled: bool = True
    tp_size: int = 1
    tp_grain_size: int = 1


@dataclass
class QuantizationConfig:
    enabled: bool = False
    bits: int = 8
    group_size: int = 128


@dataclass
class DeepSpeedMoEConfig:
    enabled: bool = True
    ep_size: int = 1
    moe_experts: list = field(default_factory=lambda: [1])
    type: str = "standard"


@dataclass
class DeepSpeedInferenceConfig:
    dtype: object = torch.float16
    tensor_parallel: DeepSpeedTPConfig = field(default_factory=DeepSpeedTPConfig)
    replace_with_kernel_inject: bool = False
    enable_cuda_graph: bool = False
    use_triton: bool = False
    triangular_masking: bool = True
    return_tuple: bool = True
    checkpoint: object = None
    base_dir: str = ""
    save_mp_checkpoint_path: str = None
    injection_policy: dict = None
    injection_policy_tuple: tuple = None
    max_out_tokens: int = 1024
    min_out_tokens: int = 1
    transposed_mode: bool = False
    quant: QuantizationConfig = field(default_factory=QuantizationConfig)
    moe: DeepSpeedMoEConfig = field(default_factory=DeepSpeedMoEConfig)
    keep_module_on_host: bool = False
    extra: dict = field(default_factory=dict)

    def __init__(self, **kw):
        self.dtype = torch.float16
        self.tensor_parallel = DeepSpeedTPConfig()
        self.replace_with_kernel_inject = False
        self.enable_cuda_graph = False
        self.use_triton = False
        self.triangular_masking = True
        self.return_tuple = True
        self.checkpoint = None
        self.base_dir = ""
        self.save_mp_checkpoint_path = None
        self.injection_policy = None
        self.injection_policy_tuple = None
        self.max_out_tokens = 1024
        self.min_out_tokens = 1
        self.transposed_mode = False
        self.quant = QuantizationConfig()
        self.moe = DeepSpeedMoEConfig()
        self.keep_module_on_host = False
        self.extra = {}
        for k, v in kw.items():
            if k in ("mp_size", "tp_size"):
                self.tensor_parallel.tp_size = int(v)
            elif k in ("tensor_parallel", "tp") and isinstance(v, dict):
                self.tensor_parallel = DeepSpeedTPConfig(**{a: b for a, b in v.items()
                                                            if a in DeepSpeedTPConfig.__dataclass_fields__})
            elif k == "dtype":
                self.dtype = _DTYPES[v] if isinstance(v, str) else v
            elif k == "quant" and isinstance(v, dict):
                self.quant = QuantizationConfig(**{a: b for a, b in v.items()
                                                   if a in QuantizationConfig.__dataclass_fields__})
            elif k == "moe" and isinstance(v, dict):
                self.moe = DeepSpeedMoEConfig(**{a: b for a, b in v.items()
                                                 if a in DeepSpeedMoEConfig.__dataclass_fields__})
            elif k == "kernel_inject":
                self.replace_with_kernel_inject = bool(v)
            elif hasattr(self, k):
                setattr(self, k, v)
            else:
                self.extra[k] = v

    def to_dict(self):
        d = {k: v for k, v in self.__dict__.items()}
        for k in ("tensor_parallel", "quant", "moe"):
            d[k] = asdict(d[k])
        d["dtype"] = str(self.dtype).replace("torch.", "")
        return d
