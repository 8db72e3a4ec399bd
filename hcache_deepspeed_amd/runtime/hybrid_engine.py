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
        self._gather_latency = 0.0
        self._total_batch_size = None
        self._e2e_start = None
        self._eval_iters = 0
        self.last_latency_report = None
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
    def _mp_group(self):
        """Model-parallel group for ``inference_tp_size > 1``: consecutive ranks (reference
        create_inference_module :315-338), created once."""
        if self.inference_tp_size <= 1:
            return None
        if getattr(self, "_he_mp_group", None) is None:
            from .. import comm as dist
            tp, world, rank = self.inference_tp_size, dist.get_world_size(), dist.get_rank()
            assert world % tp == 0, f"inference_tp_size={tp} must divide world size {world}"
            for g in range(world // tp):
                ranks = list(range(g * tp, (g + 1) * tp))
                grp = dist.new_group(ranks)
                if rank in ranks:
                    self._he_mp_group = grp
        return self._he_mp_group

    def _kv_generate(self, input_ids, **kwargs):
        """KV-cached (optionally tensor-parallel) generation for this framework's Llama-family models."""
        from .. import comm as dist
        from ..models.generation import KVCacheGenerator
        grp = self._mp_group()
        am = kwargs.pop("attention_mask", None)
        if grp is not None:  # batch the group's prompts, generate once with sliced layers, keep own rows
            tp = self.inference_tp_size
            B = input_ids.shape[0]
            allx = torch.empty((B * tp, ) + tuple(input_ids.shape[1:]), dtype=input_ids.dtype,
                               device=input_ids.device)
            dist.all_gather_into_tensor(allx, input_ids.contiguous(), group=grp)
            if am is not None:
                alla = torch.empty((B * tp, ) + tuple(am.shape[1:]), dtype=am.dtype, device=am.device)
                dist.all_gather_into_tensor(alla, am.contiguous(), group=grp)
                am = alla
            out = KVCacheGenerator(self.module, grp).generate(allx, attention_mask=am, **kwargs)
            r = dist.get_rank(grp)
            return out[B * r:B * (r + 1)]
        return KVCacheGenerator(self.module).generate(input_ids, attention_mask=am, **kwargs)

    @torch.no_grad()
    def generate(self, *args, **kwargs):
        from ..models.generation import supports_kv_generation
        t0 = time.time()
        if self._training_start_time is not None:
            self._training_latency += t0 - self._training_start_time
        if self._total_batch_size is None:
            from .. import comm as dist
            x = args[0] if args else kwargs.get("input_ids")
            self._total_batch_size = x.shape[0] * (dist.get_world_size() if dist.is_initialized() else 1)
        zopt = self.optimizer
        gathered = zopt is not None and getattr(zopt, "stage", 0) == 3 and getattr(zopt, "partitioned", False)
        was_training = self.module.training
        self.module.eval()
        self._in_generate = True
        try:
            if gathered:
                zopt.gather_all()
            self._gather_latency = time.time() - t0
            self.fuse_lora_weight()
            if "max_new_tokens" in kwargs:
                kwargs["max_new_tokens"] = min(kwargs["max_new_tokens"], self.max_out_tokens)
            gen = getattr(self.module, "generate", None)
            if gen is not None:
                out = gen(*args, **kwargs)
            elif supports_kv_generation(self.module):
                if args:
                    kwargs["input_ids"] = args[0]
                out = self._kv_generate(kwargs.pop("input_ids"), **kwargs)
            else:
                out = self._greedy(*args, **kwargs)
            self.unfuse_lora_weight()
        finally:
            if gathered:
                zopt.release_all()
            self._in_generate = False
            self.module.train(was_training)
            if self.release_inference_cache and torch.cuda.is_available():
                torch.cuda.empty_cache()
        t1 = time.time()
        self._generate_latency += t1 - t0 - self._gather_latency
        self._iters += 1
        self._training_start_time = t1
        return out

    def _greedy(self, input_ids, max_new_tokens=16, **kwargs):
        """Greedy full-recompute decoding for models with neither ``.generate`` nor the Llama block layout."""
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
        """Switch to generation mode; logs the RLHF iteration breakdown since the previous ``eval`` (reference
        hybrid_engine.py :381-403: E2E / gather / generate / training latency and samples per second)."""
        now = time.time()
        if self._e2e_start is not None:
            lat = now - self._e2e_start
            self._total_latency += lat
            self._eval_iters += 1
            others = lat - (self._gather_latency + self._generate_latency + self._training_latency)
            msg = (f"|E2E latency={lat:.2f}s |Gather latency={self._gather_latency:.2f}s "
                   f"({100 * self._gather_latency / lat:.2f}%) |Generate time={self._generate_latency:.2f}s "
                   f"({100 * self._generate_latency / lat:.2f}%) |Training time={self._training_latency:.2f}s "
                   f"({100 * self._training_latency / lat:.2f}%) |Others={others:.2f} ({100 * others / lat:.2f}%)")
            if self._total_batch_size is not None:
                msg += (f"|CurSamplesPerSec={self._total_batch_size / lat:.2f} "
                        f"|AvgSamplesPerSec={self._total_batch_size * self._eval_iters / self._total_latency:.2f}")
            self.last_latency_report = msg
            log_dist(msg, ranks=[0])
        self._e2e_start = now
        self._training_start_time = None
        self._training_latency = self._generate_latency = self._gather_latency = 0.0
        self.module.eval()
        return self

    def train(self, mode=True):
        self.module.train(mode)
        if mode:
            self._training_start_time = time.time()
        return self

    def step(self, *args, **kwargs):
        out = super().step(*args, **kwargs)
        if self._training_start_time is not None:
            now = time.time()
            self._training_latency += now - self._training_start_time
            self._training_start_time = now
        return out

    def latency_stats(self):
        total = time.time() - self._t_start
        return {"generate_s": self._generate_latency, "gather_s": self._gather_latency,
                "training_s": self._training_latency, "total_s": total, "generate_calls": self._iters}
