"""RLHF hybrid engine: one model that trains under ZeRO and generates at inference speed.

Reference parity: runtime/hybrid_engine.py ``DeepSpeedHybridEngine`` (:30-445): ``generate`` (:168) gathers
the ZeRO-3 partitioned parameters once for the whole generation, optionally fuses LoRA weights into
the base weights, runs the (kernel-injected) inference path, then unfuses and releases; ``eval``/``train``
switch modes; latency bookkeeping (``_generate_latency``, ``_training_latency``) for the RLHF loop.

MI355X: the gather is ONE all-gather per flat unit (288 GB HBM holds a gathered 70B model in bf16 with
room for the KV cache), generation reuses this framework's HIP kernels (RMSNorm / gated MLP / FlashAttention
via inference.injection for HF models; our own Llama is already fused), and LoRA fusion is a single
addmm per adapted linear.
"""
import time

import torch

from ..utils.logging import log_dist
from .engine import DeepSpeedEngine


class DeepSpeedHybridEngine(DeepSpeedEngine):
    inference_cuda_module = None

    def __init__(self, *args, **kwargs):
        model = kwargs.get("model")
        cfg = kwargs.get("config_class")
        he = (cfg.hybrid_engine if cfg is not None else {}) or {}
        self_injected = False
        if model is not None and he.get("kernel_inject", True):
            # before ZeRO partitions the model: trainable, name-preserving injection (norms + attention)
            from ..inference.injection import inject
            self_injected = inject(model, trainable=True, fuse_mlp=False) > 0
        super().__init__(*args, **kwargs)
        he = self._config.hybrid_engine or {}
        self.max_out_tokens = int(he.get("max_out_tokens", 512))
        self.inference_tp_size = int(he.get("inference_tp_size", 1))
        self.release_inference_cache = bool(he.get("release_inference_cache", False))
        self.pin_parameters = bool(he.get("pin_parameters", True))
        self.tp_gather_partition_size = int(he.get("tp_gather_partition_size", 8))
        self._generate_latency = 0.0
        self._training_latency = 0.0
        self._total_latency = 0.0
        self._iters = 0
        self._training_start_time = None
        self._t_start = time.time()
        self._in_generate = False
        self._injected = self_injected
        log_dist(f"DeepSpeedHybridEngine: max_out_tokens={self.max_out_tokens} injected={self._injected}", ranks=[0])

    # ---- LoRA ------------------------------------------------------------------------------
    def _lora_modules(self):
        return [m for m in self.module.modules() if hasattr(m, "fuse_lora_weight") and hasattr(m, "unfuse_lora_weight")]

    def fuse_lora_weight(self):
        for m in self._lora_modules():
            m.fuse_lora_weight()

    def unfuse_lora_weight(self):
        for m in self._lora_modules():
            m.unfuse_lora_weight()

    # ---- generation --------------------------------------------------------------------------
    @torch.no_grad()
    def generate(self, *args, **kwargs):
        t0 = time.time()
        if self._training_start_time is not None:
            self._training_latency += t0 - self._training_start_time
        zopt = self.optimizer
        gathered = zopt is not None and getattr(zopt, "stage", 0) == 3 and getattr(zopt, "partitioned", False)
        was_training = self.module.training
        self.module.eval()
        self._in_generate = True
        try:
            if gathered:
                zopt.gather_all()
            self.fuse_lora_weight()
            if "max_new_tokens" in kwargs:
                kwargs["max_new_tokens"] = min(kwargs["max_new_tokens"], self.max_out_tokens)
            gen = getattr(self.module, "generate", None)
            out = gen(*args, **kwargs) if gen is not None else self._greedy(*args, **kwargs)
            self.unfuse_lora_weight()
        finally:
            if gathered:
                zopt.release_all()
            self._in_generate = False
            self.module.train(was_training)
            if self.release_inference_cache and torch.cuda.is_available():
                torch.cuda.empty_cache()
        t1 = time.time()
        self._generate_latency += t1 - t0
        self._iters += 1
        self._training_start_time = t1
        return out

    def _greedy(self, input_ids, max_new_tokens=16, **kwargs):
        """Greedy decoding for models without ``.generate`` (e.g. this framework's LlamaForCausalLM)."""
        ids = input_ids
        for _ in range(int(max_new_tokens)):
            logits = self.module(ids)
            logits = logits.view(ids.shape[0], ids.shape[1], -1) if logits.dim() == 2 else logits
            nxt = logits[:, -1].argmax(-1, keepdim=True)
            ids = torch.cat([ids, nxt], 1)
        return ids

    def forward(self, *inputs, **kwargs):
        if self._in_generate:
            return self.module(*inputs, **kwargs)
        return super().forward(*inputs, **kwargs)

    def eval(self):
        self.module.eval()
        return self

    def train(self, mode=True):
        self.module.train(mode)
        if mode and self._training_start_time is None:
            self._training_start_time = time.time()
        return self

    def latency_stats(self):
        total = time.time() - self._t_start
        return {"generate_s": self._generate_latency, "training_s": self._training_latency, "total_s": total,
                "generate_calls": self._iters}
