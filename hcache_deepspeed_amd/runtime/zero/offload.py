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
        # pipeline piece: sub_group_size, capped at 256M elements -- at the 1e9 default the first gradient D2H and the
        # last bf16 H2D of a step (4 GB / 2 GB each) sit outside the pipeline; Llama-3-8B mb10 Twin-Flow 0.4 on one
        # box: 19,772 tok/s at 2.5e8 vs 18,651 at 1e9 and 17,536 at 1e8 (per-piece overhead), profiles/r5/*_r5ay.json
        self.sub = max(1 << 20, min(int(self.zcfg.sub_group_size), 1 << 28, self.n_off or 1))
        self.nvme = None
        if self.offload_device == "nvme":
            # fp32 master + moments of the offloaded range on NVMe, streamed by the step in chunks of at most
            # 64M elements (3 pinned staging slots per state: read-ahead / in use / write-behind)
            from ..swap_tensor import PipelinedOptimizerSwapper
            from ..swap_tensor.aio_config import make_aio_handle
            self.sub = min(self.sub, 64 << 20)
            folder = os.path.join(oc.nvme_path or "/tmp/hds_nvme", "zero_stage_3", "optimizer", f"rank{dist.get_rank()}")
            self.nvme = make_aio_handle(self.config.aio_config)
            keys = ["fp32"] + list(self._STATE_KEYS[self.kind])
            self.opt_swapper = PipelinedOptimizerSwapper(self.nvme, folder, keys, self.n_off, self.sub)
            self.opt_swapper.write_full("fp32", s.master[:self.n_off].cpu())
            for k in keys[1:]:
                self.opt_swapper.write_full(k, None)
            self.h_master = None
            self.h_states = {k: None for k in keys[1:]}
        else:
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
        elif self.n_off > 0:
            self._compact_device_part()
        # copy streams at high priority: a stream that shares a hardware queue with the compute stream (HIP
        # spreads streams over GPU_MAX_HW_QUEUES=4 queues) cannot start a copy before the kernels queued ahead
        self.copy_stream = torch.cuda.Stream(self.device, priority=-1) if self.device.type == "cuda" else None  # D2H
        self.h2d_stream = torch.cuda.Stream(self.device, priority=-1) if self.device.type == "cuda" else None  # H2D
        log_dist(f"ZeRO-Offload: {self.n_off / 1e6:.1f}M of {n / 1e6:.1f}M elements on {self.offload_device} "
                 f"(sub-group {self.sub / 1e6:.1f}M)" + (", parameters on NVMe" if self.nvme_param else ""),
                 ranks=[0])

    @torch.no_grad()
    def _compact_device_part(self):
        """Twin-Flow (ratio < 1) uses only [n_off, n) of the fp32 master and of every moment on the device, but the
        store indexes them over the whole partition. The k + 1 full-length views are laid over ONE buffer of
        n + k * m elements (m = n - n_off, k moments) at offsets 0, m, 2m, ...: each view's device range [n_off, n)
        is its own, and its offloaded prefix -- which no device code reads or writes (the host holds that range) --
        lies over its neighbours' live ranges. Saves k + 1 times n_off fp32 elements of HBM (Llama-3-8B at ratio 0.6:
        38 GB), which is what lets the device part fit beside micro-batch-10 activations."""
        s = self.store
        n, k0 = s.numel, self.n_off
        m = n - k0
        keys = [k for k in s.states if s.states[k] is not None]
        buf = torch.empty(n + len(keys) * m, dtype=torch.float32, device=s.master.device)
        master = buf[0:n]
        master[k0:].copy_(s.master[k0:])
        states = {}
        for i, k in enumerate(keys, 1):
            v = buf[i * m:i * m + n]
            v[k0:].copy_(s.states[k][k0:])
            states[k] = v
        s.master = master
        s.states.update(states)
        if getattr(self, "_generic_params", None):  # views of the old master (the generic path runs as Adam here)
            self._generic_params, self._generic_opt = [], None

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
        dev_grad = s.grad
        gpu = self.copy_stream is not None
        d2h_ev, h2d_ev = [None, None], [None, None]
        lp_writes = [None, None]  # NVMe parameter tier: pending swap-file write of each bf16 staging buffer
        swap = self.opt_swapper.pipeline(bounds) if self.nvme is not None else None

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
            if swap is not None:  # NVMe: this chunk's master / moments, read ahead by the swapper
                _, st = next(swap)
                p32 = st["fp32"]
            else:
                st = {k: v[lo:hi] for k, v in self.h_states.items()}
                p32 = self.h_master[lo:hi]
            if self.nvme_param:
                if lp_writes[b] is not None:
                    lp_writes[b].wait()  # staging buffer b's previous swap-file write has landed
                    lp_writes[b] = None
                out = self.h_lp[b][:n]
            else:
                # parameters offloaded too: the CPU optimizer writes bf16 straight into the pinned lp shard
                out = s.lp[lo:hi] if self.lp_on_host else self.h_lp[b][:n]
            if self.kind in ("adam", "generic"):
                cpu_adam_flat(p32, hg, st["exp_avg"], st["exp_avg_sq"], g["step"], g["lr"],
                              tuple(g.get("betas", (0.9, 0.999))), g.get("eps", 1e-8), g.get("weight_decay", 0.0),
                              self.adamw, g.get("bias_correction", True),
                              bf16_out=out if self.dtype == torch.bfloat16 else None, grad_scale=coef)
            elif self.kind == "lion":
                cpu_lion_flat(p32, hg, st["exp_avg"], g["lr"], tuple(g.get("betas", (0.9, 0.99))),
                              g.get("weight_decay", 0.0), bf16_out=out if self.dtype == torch.bfloat16 else None,
                              grad_scale=coef)
            else:
                cpu_adagrad_flat(p32, hg, st["sum"], g["lr"], g.get("eps", 1e-10), g.get("weight_decay", 0.0),
                                 bf16_out=out if self.dtype == torch.bfloat16 else None, grad_scale=coef)
            if self.dtype != torch.bfloat16:
                out.copy_(p32)
            if self.nvme_param:
                lp_writes[b] = self.param_swapper.swap_out(lo, out)
                continue
            if self.lp_on_host:
                continue
            if gpu:
                with torch.cuda.stream(self.h2d_stream):
                    s.lp[lo:hi].copy_(out, non_blocking=True)
                    h2d_ev[b] = torch.cuda.Event()
                    h2d_ev[b].record(self.h2d_stream)
            else:
                s.lp[lo:hi].copy_(out)
        if swap is not None:
            next(swap, None)  # write back the last chunk; the generator waits for every outstanding transfer
        for w in lp_writes:
            if w is not None:
                w.wait()
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

    # checkpoint hooks: the fp32 master / moments of the offloaded range live in host DRAM or on NVMe
    def _host_range(self, key):
        """Full offloaded range of ``key`` ("fp32" or a moment) as a CPU fp32 tensor (read from NVMe if needed)."""
        if self.nvme is not None:
            return self.opt_swapper.read_full(key)
        return self.h_master if key == "fp32" else self.h_states[key]

    def _set_host_range(self, key, t):
        if self.nvme is not None:
            self.opt_swapper.write_full(key, t)
        elif key == "fp32":
            self.h_master.copy_(t)
        else:
            self.h_states[key].copy_(t)

    def _ckpt_flats(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        out = OrderedDict()
        for key in ["fp32"] + list(self._STATE_KEYS[self.kind]):
            t = torch.empty(n, dtype=torch.float32)
            if k0:
                t[:k0].copy_(self._host_range(key))
            if k0 < n:
                t[k0:].copy_((s.master if key == "fp32" else s.states[key])[k0:])
            out[key] = t
        return out

    def _ckpt_commit(self, flats):
        s, n, k0 = self.store, self.store.numel, self.n_off
        for key, t in flats.items():
            if k0:
                self._set_host_range(key, t[:k0])
            if k0 < n:
                (s.master if key == "fp32" else s.states[key])[k0:].copy_(t[k0:])

    def _lp_host(self):
        """This rank's compute-dtype shard as a host tensor (the NVMe tier reads the parameter swap file)."""
        if self.nvme_param:
            return self.param_swapper.read_sync(0, torch.empty(self.store.numel, dtype=self.dtype))
        return self.store.lp

    def _lp_to_master(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        lp = self._lp_host()
        if k0:
            self._set_host_range("fp32", lp[:k0].float().cpu())
        if k0 < n:
            s.master[k0:].copy_(lp[k0:])

    def _master_to_lp(self):
        s, n, k0 = self.store, self.store.numel, self.n_off
        m = self._host_range("fp32") if k0 else None
        if self.nvme_param:
            self.param_swapper.write_sync(0, m.to(self.dtype))
            return
        if k0:
            s.lp[:k0].copy_(m)
        if k0 < n:
            s.lp[k0:].copy_(s.master[k0:])

    def full_fp32_state_dict(self, names):
        s = self.store
        saved = s.master
        m = self._host_range("fp32").to(self.device)
        if self.n_off < s.numel:
            m = torch.cat([m, saved[self.n_off:]])
        s.master = m
        try:
            return super().full_fp32_state_dict(names)
        finally:
            s.master = saved
