"""Training-side host activation cache ("Hcache" for training): spill saved activations to pinned host DRAM.

BASELINE north star: "activations ... spill to host DRAM without stalling backward". Reference analogues:
CPU activation checkpointing (runtime/activation_checkpointing/checkpointing.py:59,474-486), FPDT chunk
offload (sequence/fpdt_layer.py:462-508 ``SequenceChunk``) and the DeepCompile offload_activation pass
(compile/passes/offload_activation.py, csrc/compile/z3.cpp:268-341).

Mechanism (``torch.autograd.graph.saved_tensors_hooks``):

* forward/pack: a saved activation larger than ``min_bytes`` from a block that is not among the last
  ``min_layers_resident`` blocks is copied D2H on a dedicated HIP copy stream into a pinned host buffer
  from a reuse pool (``offload/pinned.py``, hipHostMalloc). The GPU tensor is released immediately with
  ``record_stream`` so the caching allocator recycles it once the DMA has drained -- forward never waits.
* backward/unpack: when block i's tensors are first needed, block i-1's tensors are prefetched H2D on the
  copy stream (reverse layer order), so the PCIe transfer overlaps block i's backward; the compute stream
  only waits on the per-tensor HIP event.
Parameters (autograd leaves) and small tensors are never offloaded.
"""
import contextlib

import torch
import torch.nn as nn

from ..utils.logging import log_dist
from .pinned import PinnedPool


class _Spilled:
    __slots__ = ("host", "shape", "dtype", "device", "layer", "d2h_done", "dev", "h2d_done", "stride_ok")

    def __init__(self):
        self.dev = None
        self.h2d_done = None


class HostActivationCache:

    def __init__(self, device, min_bytes=1 << 20, min_layers_resident=2, prefetch_layers=1):
        self.device = device
        self.min_bytes = int(min_bytes)
        self.keep = int(min_layers_resident)
        self.prefetch_layers = int(prefetch_layers)
        self.pool = PinnedPool()
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.cur_layer = -1
        self.n_layers = 0
        self.by_layer = {}
        self.bytes_offloaded = 0
        self._attached = []

    @classmethod
    def from_config(cls, cfg, device):
        return cls(device, min_bytes=1 << 20, min_layers_resident=cfg.min_layers_resident)

    # ---------------------------------------------------------------------------------------
    def attach(self, model):
        """Track which transformer block is running (every nn.ModuleList element counts as a block)."""
        blocks = []
        for m in model.modules():
            if isinstance(m, nn.ModuleList):
                blocks.extend(list(m))
        self.n_layers = len(blocks)
        for i, b in enumerate(blocks):
            self._attached.append(b.register_forward_pre_hook(lambda mod, args, i=i: self._enter(i)))
        return self

    def _enter(self, i):
        if torch.is_grad_enabled():
            self.cur_layer = i

    @contextlib.contextmanager
    def forward_context(self):
        self.cur_layer = -1
        self.by_layer = {}
        with torch.autograd.graph.saved_tensors_hooks(self._pack, self._unpack):
            yield

    # ---------------------------------------------------------------------------------------
    def _pack(self, t):
        if (not isinstance(t, torch.Tensor) or not t.is_cuda or t.is_leaf or self.cur_layer < 0
                or self.cur_layer >= self.n_layers - self.keep
                or t.numel() * t.element_size() < self.min_bytes):
            return t
        s = _Spilled()
        s.shape, s.dtype, s.device, s.layer = t.shape, t.dtype, t.device, self.cur_layer
        src = t if t.is_contiguous() else t.contiguous()
        s.host = self.pool.get(src.numel(), src.dtype)
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            s.host.copy_(src.view(-1), non_blocking=True)
            src.record_stream(self.stream)
            s.d2h_done = torch.cuda.Event()
            s.d2h_done.record(self.stream)
        self.bytes_offloaded += src.numel() * src.element_size()
        self.by_layer.setdefault(s.layer, []).append(s)
        return s

    def _prefetch(self, s):
        if s.dev is not None:
            return
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(s.d2h_done)
            s.dev = torch.empty(s.shape, dtype=s.dtype, device=s.device)
            s.dev.view(-1).copy_(s.host, non_blocking=True)
            s.h2d_done = torch.cuda.Event()
            s.h2d_done.record(self.stream)

    def _unpack(self, s):
        if not isinstance(s, _Spilled):
            return s
        self._prefetch(s)
        for j in range(1, self.prefetch_layers + 1):
            for o in self.by_layer.get(s.layer - j, ()):
                self._prefetch(o)
        torch.cuda.current_stream().wait_event(s.h2d_done)
        out = s.dev
        out.record_stream(torch.cuda.current_stream())
        s.dev = None
        self.pool.put(s.host)
        s.host = None
        return out

    def stats(self):
        return {"bytes_offloaded": self.bytes_offloaded, "pinned_pool_bytes": self.pool.bytes_allocated}
