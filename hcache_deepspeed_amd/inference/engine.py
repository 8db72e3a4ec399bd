"""``init_inference`` engine (v1): dtype conversion, AutoTP sharding, kernel injection, HIP-graph replay.

Reference parity: inference/engine.py ``InferenceEngine`` (:40-630): ``_create_model_parallel_group``
(TP groups), ``_apply_injection_policy`` / AutoTP, checkpoint loading, ``_create_cuda_graph`` (:494) and
``forward`` replay, ``generate`` passthrough, ``_generate`` max-token guard. On MI355X the "CUDA graph" is a
HIP graph captured through ``torch.cuda.CUDAGraph`` for fixed input shapes (one graph per shape key).
"""
import torch
import torch.nn as nn

from .. import comm as dist
from ..utils import groups
from ..utils.logging import log_dist
from .config import DeepSpeedInferenceConfig


class InferenceEngine(nn.Module):

    def __init__(self, model, config=None):
        super().__init__()
        self._config = config if isinstance(config, DeepSpeedInferenceConfig) else \
            DeepSpeedInferenceConfig(**(config or {}))
        cfg = self._config
        self.module = model
        self.mp_world_size = int(cfg.tensor_parallel.tp_size)
        self.mpu = None
        self.mp_group = None
        if self.mp_world_size > 1:
            if not dist.is_initialized():
                dist.init_distributed(verbose=False)
            if groups._State.topo is None or groups.get_model_parallel_world_size() != self.mp_world_size:
                groups.reset()
                groups.initialize(tp=self.mp_world_size)
            self.mp_group = groups._get_model_parallel_group()
        self.device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
            torch.device("cpu")
        if cfg.checkpoint is not None:
            self._load_checkpoint(cfg.checkpoint)
        if cfg.dtype in (torch.float16, torch.bfloat16, torch.float32):
            self.module.to(cfg.dtype)
        if self.mp_world_size > 1:
            from ..parallel.tp import AutoTP
            AutoTP(self.module, self.mp_group, self.mp_world_size).shard()
        if not cfg.keep_module_on_host:
            self.module.to(self.device)
        self.injected = 0
        if cfg.replace_with_kernel_inject or cfg.quant.enabled:
            from .injection import inject
            self.injected = inject(self.module, cfg.quant if cfg.quant.enabled else None)
        self.module.eval()
        self._graphs = {}
        log_dist(f"InferenceEngine: dtype={cfg.dtype} tp={self.mp_world_size} injected_blocks={self.injected} "
                 f"hip_graph={cfg.enable_cuda_graph}", ranks=[0])

    def _load_checkpoint(self, ckpt):
        import os
        from safetensors.torch import load_file
        files = ckpt if isinstance(ckpt, (list, tuple)) else ([ckpt] if isinstance(ckpt, str) else ckpt.get("checkpoints", []))
        sd = {}
        for f in files:
            f = os.path.join(self._config.base_dir, f) if self._config.base_dir else f
            sd.update(load_file(f) if f.endswith(".safetensors") else torch.load(f, map_location="cpu",
                                                                                 weights_only=True))
        missing, unexpected = self.module.load_state_dict(sd, strict=False)
        log_dist(f"loaded checkpoint: {len(sd)} tensors, missing={len(missing)} unexpected={len(unexpected)}",
                 ranks=[0])

    # ------------------------------------------------------------------------------------
    def _graph_key(self, args, kwargs):
        def sig(x):
            if isinstance(x, torch.Tensor):
                return ("T", tuple(x.shape), x.dtype)
            return ("O", repr(x))
        return tuple(sig(a) for a in args) + tuple((k, sig(v)) for k, v in sorted(kwargs.items()))

    def _graph_forward(self, *args, **kwargs):
        key = self._graph_key(args, kwargs)
        g = self._graphs.get(key)
        if g is None:
            static_args = [a.clone() if isinstance(a, torch.Tensor) else a for a in args]
            static_kwargs = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in kwargs.items()}
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up allocator / lazy inits outside the capture
                    self.module(*static_args, **static_kwargs)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self.module(*static_args, **static_kwargs)
            g = (graph, static_args, static_kwargs, out)
            self._graphs[key] = g
        graph, static_args, static_kwargs, out = g
        for a, s_ in zip(args, static_args):
            if isinstance(a, torch.Tensor):
                s_.copy_(a)
        for k, v in kwargs.items():
            if isinstance(v, torch.Tensor):
                static_kwargs[k].copy_(v)
        graph.replay()
        return out

    @torch.no_grad()
    def forward(self, *args, **kwargs):
        if self._config.enable_cuda_graph and torch.cuda.is_available():
            return self._graph_forward(*args, **kwargs)
        return self.module(*args, **kwargs)

    @torch.no_grad()
    def generate(self, *args, **kwargs):
        if "max_new_tokens" in kwargs and kwargs["max_new_tokens"] > self._config.max_out_tokens:
            raise ValueError(f"max_new_tokens {kwargs['max_new_tokens']} exceeds max_out_tokens "
                             f"{self._config.max_out_tokens}")
        return self.module.generate(*args, **kwargs)
