"""ZeRO-Offload / ZeRO-Infinity optimizer tier: fp32 master + optimizer states in host DRAM (or NVMe).

Reference parity: ZeRO-Offload in stage_1_and_2.py:1189-1335,1874-1893 and stage3.py:607-641,1493-1522
(host fp32 partitions, D2H grads, DeepSpeedCPUAdam, H2D bf16 params), ZeRO-Offload++ partial offload
(``offload_optimizer.ratio`` < 1, offload_config.py:93), NVMe optimizer-state swapping
(runtime/swap_tensor/partitioned_optimizer_swapper.py, pipelined_optimizer_swapper.py:52-241).

Pipeline per step (sub-groups of ``sub_group_size`` elements; chunk k):
    copy stream : D2H grad[k+1] -> pinned host           (overlaps)
    host        : CPU Adam on chunk k (AVX-512, OpenMP) writing bf16 into pinned staging
    copy stream : H2D bf16[k] -> device lp shard
The gradient norm / clip coefficient is still computed on the GPU (one scalar read back per step).
With ``ratio < 1`` the first ``ratio`` fraction of the shard is offloaded and the rest keeps the
on-device fused-Adam path (Twin-Flow). With ``device: nvme`` the moments of each sub-group are
swapped in/out through the async file I/O handle around its CPU update.
"""
import os
from collections import OrderedDict

import torch

from ... import comm as dist
from ...ops import optimizers as fused
from ...ops.cpu_optimizers import cpu_adagrad_flat, cpu_adam_flat, cpu_lion_flat
from ...utils.logging import log_dist
from .optimizer import ZeroOptimizer


def _host_empty(numel, dtype, pin):
    if pin and torch.cuda.is_available():
        from ...offload.pinned import pinned_empty
        return pinned_empty((numel, ), dtype)
    return torch.empty(numel, dtype=dtype)


class OffloadZeroOptimizer(ZeroOptimizer):

    _STATE_KEYS = {"adam": ("exp_avg", "exp_avg_sq"), "lion": ("exp_avg", ), "adagrad": ("sum", )}

    def __init__(self, *args, **kwargs):
        config = args[2] if len(args) > 2 else kwargs["config"]
        oc0 = config.zero_config.offload_optimizer
        # full offload: never allocate device-side optimizer states (70B-class models)
        self._defer_states = (not oc0.enabled) or float(oc0.ratio) >= 1.0
        super().__init__(*args, **kwargs)
        if self.kind == "generic":  # host path implements Adam/Lion/Adagrad; other torch optimizers -> AdamW
            self.kind, self.adamw = "adam", True
            if not self._defer_states:
                self.store.states = {"exp_avg": torch.zeros_like(self.store.master),
                                     "exp_avg_sq": torch.zeros_like(self.store.master)}
        if self._defer_states:
            self.store.states = {k: None for k in self._STATE_KEYS[self.kind]}
        oc = self.zcfg.offload_optimizer
        self.offload_device = oc.device if oc.enabled else "cpu"
        self.ratio = float(oc.ratio if oc.enabled else 1.0)
        self.pin = bool(oc.pin_memory) or torch.cuda.is_available()
        s = self.store
        n = s.numel
        self.n_off = int(n * self.ratio) // 64 * 64 if self.ratio < 1.0 else n
        self.lp_on_host = s.lp.device.type == "cpu" and self.device.type == "cuda"
        assert not (self.lp_on_host and self.n_off < n), "offload_param requires offload_optimizer.ratio == 1"
        self.sub = max(1 << 20, min(int(self.zcfg.sub_group_size), self.n_off or 1))
        # host copies of the offloaded range
        self.h_master = _host_empty(self.n_off, torch.float32, False)
        self.h_master.copy_(s.master[:self.n_off].cpu())
        if self.n_off == n:
            s.master = None  # free before the host state buffers are allocated
        self.h_states = {k: torch.zeros(self.n_off, dtype=torch.float32) for k in s.states}
        # double-buffered pinned staging: grads D2H (chunk k+1) / bf16 params H2D (chunk k-1)
        self.h_grad = [_host_empty(self.sub, s.grad.dtype, self.pin) for _ in range(2)]
        self.h_lp = [_host_empty(self.sub, self.dtype, self.pin) for _ in range(2)]
        # free device memory of the offloaded part of master / states
        if self.n_off == n:
            s.master = None
            s.states = {k: None for k in s.states}
        self.copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None  # D2H
        self.h2d_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None  # H2D
        self.nvme = None
        if self.offload_device == "nvme":
            from ...ops.aio import aio_handle
            path = oc.nvme_path or "/tmp/hds_nvme"
            os.makedirs(path, exist_ok=True)
            self.nvme_dir = path
            aio = self.config.aio_config
            self.nvme = aio_handle(aio.get("block_size", 1 << 20), aio.get("queue_depth", 8),
                                   aio.get("single_submit", False), aio.get("overlap_events", True),
                                   aio.get("intra_op_parallelism", 4))
            for k, v in self.h_states.items():
                self.nvme.sync_pwrite(v, self._nvme_file(k))
            self.h_states = {k: None for k in self.h_states}
        log_dist(f"ZeRO-Offload: {self.n_off / 1e6:.1f}M of {n / 1e6:.1f}M elements on {self.offload_device} "
                 f"(sub-group {self.sub / 1e6:.1f}M)", ranks=[0])

    def _nvme_file(self, k):
        return os.path.join(self.nvme_dir, f"rank{dist.get_rank()}_{k}.bin")

    def _state_chunk(self, k, lo, hi, buf_cache):
        if self.nvme is None:
            return self.h_states[k][lo:hi]
        t = buf_cache.get(k)
        if t is None or t.numel() < hi - lo:
            t = torch.empty(hi - lo, dtype=torch.float32)
            buf_cache[k] = t
        t = t[:hi - lo]
        self.nvme.sync_pread(t, self._nvme_file(k), file_offset=lo * 4)
        return t

    @torch.no_grad()
    def step(self, closure=None):
        s = self.store
        inv = 1.0 / (self.layout_world_for_avg() * self.loss_scaler.loss_scale)
        self._norm_buf.zero_()
        self._inf_buf.zero_()
        fused.grad_sumsq([s.grad], out=self._norm_buf, found_inf=self._inf_buf)
        self._reduce_norm()
        if self.dp_world > 1 and not self.loss_scaler.dynamic:
            dist.all_reduce(self._inf_buf, op=dist.ReduceOp.MAX, group=self.dp_group)
        coef_t = fused.clip_coef(self._norm_buf, self.clip_grad, inv, coef=self._coef_buf)
        self.global_norm, self._norm_scale = self._norm_buf, inv
        overflow = bool(self._inf_buf.item())
        if self.loss_scaler.dynamic:
            self.loss_scaler.update_scale(overflow)
        if overflow:
            self.overflow = True
            self.zero_grad()
            return False
        coef = float(coef_t.item())
        for g in self.param_groups:
            g["step"] = g.get("step", 0) + 1
        # device part (Twin-Flow): segments beyond n_off use the fused GPU kernels
        if self.n_off < s.numel:
            self._device_tail_step(coef_t)
        # host part, chunked & pipelined
        bounds = []
        for seg in s.segments:
            lo = seg.store_off
            hi = min(seg.store_off + seg.numel, self.n_off)
            while lo < hi:
                e = min(hi, lo + self.sub)
                bounds.append((lo, e, seg.group))
                lo = e
        cache = {}
        dev_grad = s.grad
        gpu = self.copy_stream is not None
        d2h_ev, h2d_ev = [None, None], [None, None]

        def issue_d2h(i):
            lo, hi, _ = bounds[i]
            b = i & 1
            if not gpu:
                self.h_grad[b][:hi - lo].copy_(dev_grad[lo:hi])
                return
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(ev)
                self.h_grad[b][:hi - lo].copy_(dev_grad[lo:hi], non_blocking=True)
                d2h_ev[b] = torch.cuda.Event()
                d2h_ev[b].record(self.copy_stream)

        if bounds:
            issue_d2h(0)
        for idx, (lo, hi, gi) in enumerate(bounds):
            n = hi - lo
            b = idx & 1
            if idx + 1 < len(bounds):
                issue_d2h(idx + 1)  # next chunk's grads stream in while this one updates on the host
            if gpu:
                d2h_ev[b].synchronize()
                if h2d_ev[b] is not None:
                    h2d_ev[b].synchronize()  # staging buffer b is free again
            hg = self.h_grad[b][:n]
            g = self.param_groups[gi]
            p32 = self.h_master[lo:hi]
            # parameters offloaded too: the CPU optimizer writes bf16 straight into the pinned lp shard
            out = s.lp[lo:hi] if self.lp_on_host else self.h_lp[b][:n]
            if self.kind in ("adam", "generic"):
                m = self._state_chunk("exp_avg", lo, hi, cache)
                v = self._state_chunk("exp_avg_sq", lo, hi, cache)
                cpu_adam_flat(p32, hg, m, v, g["step"], g["lr"], tuple(g.get("betas", (0.9, 0.999))),
                              g.get("eps", 1e-8), g.get("weight_decay", 0.0), self.adamw,
                              g.get("bias_correction", True), bf16_out=out if self.dtype == torch.bfloat16 else None,
                              grad_scale=coef)
                if self.nvme is not None:
                    self.nvme.sync_pwrite(m, self._nvme_file("exp_avg"), file_offset=lo * 4)
                    self.nvme.sync_pwrite(v, self._nvme_file("exp_avg_sq"), file_offset=lo * 4)
            elif self.kind == "lion":
                m = self._state_chunk("exp_avg", lo, hi, cache)
                cpu_lion_flat(p32, hg, m, g["lr"], tuple(g.get("betas", (0.9, 0.99))), g.get("weight_decay", 0.0),
                              bf16_out=out if self.dtype == torch.bfloat16 else None, grad_scale=coef)
            else:
                st = self._state_chunk("sum", lo, hi, cache)
                cpu_adagrad_flat(p32, hg, st, g["lr"], g.get("eps", 1e-10), g.get("weight_decay", 0.0),
                                 bf16_out=out if self.dtype == torch.bfloat16 else None, grad_scale=coef)
            if self.dtype != torch.bfloat16:
                out.copy_(p32)
            if self.lp_on_host:
                continue
            if gpu:
                with torch.cuda.stream(self.h2d_stream):
                    s.lp[lo:hi].copy_(out, non_blocking=True)
                    h2d_ev[b] = torch.cuda.Event()
                    h2d_ev[b].record(self.h2d_stream)
            else:
                s.lp[lo:hi].copy_(out)
        if gpu:
            torch.cuda.current_stream().wait_stream(self.h2d_stream)
        self._post_step_gather()
        self.zero_grad()
        return True

    def _device_tail_step(self, coef):
        s = self.store
        for sg in s.segments:
            lo = max(sg.store_off, self.n_off)
            hi = sg.store_off + sg.numel
            if lo >= hi:
                continue
            g = self.param_groups[sg.group]
            fused.adam_flat(s.master[lo:hi], s.grad[lo:hi], s.states["exp_avg"][lo:hi],
                            s.states["exp_avg_sq"][lo:hi], g["step"], g["lr"], tuple(g.get("betas", (0.9, 0.999))),
                            g.get("eps", 1e-8), g.get("weight_decay", 0.0), self.adamw, True, lp_out=s.lp[lo:hi],
                            dev_scale=coef)

    # checkpoint hooks: the fp32 master / moments of the offloaded range live in host DRAM (or NVMe)
    def _ckpt_flats(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        out = OrderedDict()
        m = torch.empty(n, dtype=torch.float32)
        m[:k0].copy_(self.h_master)
        if k0 < n:
            m[k0:].copy_(s.master[k0:])
        out["fp32"] = m
        for k in self._STATE_KEYS[self.kind]:
            t = torch.empty(n, dtype=torch.float32)
            if self.nvme is None:
                t[:k0].copy_(self.h_states[k])
            elif k0:
                self.nvme.sync_pread(t[:k0], self._nvme_file(k))
            if k0 < n:
                t[k0:].copy_(s.states[k][k0:])
            out[k] = t
        return out

    def _ckpt_commit(self, flats):
        s, n, k0 = self.store, self.store.numel, self.n_off
        self.h_master.copy_(flats["fp32"][:k0])
        if k0 < n:
            s.master[k0:].copy_(flats["fp32"][k0:])
        for k, t in flats.items():
            if k == "fp32":
                continue
            if self.nvme is None:
                self.h_states[k].copy_(t[:k0])
            elif k0:
                self.nvme.sync_pwrite(t[:k0].contiguous(), self._nvme_file(k))
            if k0 < n:
                s.states[k][k0:].copy_(t[k0:])

    def _lp_to_master(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        self.h_master.copy_(s.lp[:k0])
        if k0 < n:
            s.master[k0:].copy_(s.lp[k0:])

    def _master_to_lp(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        s.lp[:k0].copy_(self.h_master)
        if k0 < n:
            s.lp[k0:].copy_(s.master[k0:])

    def full_fp32_state_dict(self, names):
        s = self.store
        saved = s.master
        m = self.h_master.to(self.device)
        if self.n_off < s.numel:
            m = torch.cat([m, saved[self.n_off:]])
        s.master = m
        try:
            return super().full_fp32_state_dict(names)
        finally:
            s.master = saved
