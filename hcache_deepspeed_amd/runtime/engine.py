"""Training engine: ``engine(batch)`` / ``engine.backward(loss)`` / ``engine.step()``.

Reference parity: runtime/engine.py ``DeepSpeedEngine`` (construction :192-392, distributed model
setup :1242-1307, optimizer selection :1378-1776, forward :2041, backward :2204, step :2338-2445,
save/load_checkpoint :3274/:2928, no_sync :2184, offload_states :3943).

Every optimizer path goes through the flat-shard :class:`ZeroOptimizer` (stage 0 included), so the
hot path is identical for all stages and the bf16 step never synchronises with the host.
"""
import contextlib
import os

import torch
import torch.nn as nn

from .. import comm as dist
from ..utils import groups
from ..utils.logging import log_dist, logger
from ..utils.timer import NoopTimer, SynchronizedWallClockTimer, ThroughputTimer
from . import lr_schedules
from .config import DeepSpeedConfig
from .dataloader import DeepSpeedDataLoader
from .engine_api import EngineApiMixin
from .zero.optimizer import ZeroOptimizer

FORWARD_MICRO_TIMER = "fwd_microstep"
FORWARD_GLOBAL_TIMER = "fwd"
BACKWARD_MICRO_TIMER = "bwd_microstep"
BACKWARD_GLOBAL_TIMER = "bwd"
STEP_MICRO_TIMER = "step_microstep"
STEP_GLOBAL_TIMER = "step"


class EngineTimers:
    """Names of the engine timers (reference runtime/engine.py:154)."""

    def __init__(self, enable_micro_timers, enable_global_timers):
        self.forward_timers = [FORWARD_MICRO_TIMER] if enable_micro_timers else []
        self.backward_timers = [BACKWARD_MICRO_TIMER] if enable_micro_timers else []
        self.step_timers = [STEP_MICRO_TIMER] if enable_micro_timers else []
        if enable_global_timers:
            self.forward_timers.append(FORWARD_GLOBAL_TIMER)
            self.backward_timers.append(BACKWARD_GLOBAL_TIMER)
            self.step_timers.append(STEP_GLOBAL_TIMER)


def _dtype_of(cfg):
    if cfg.bfloat16_enabled:
        return torch.bfloat16
    if cfg.fp16_enabled:
        return torch.float16
    return torch.float32


def _truncate_seqlen(inputs, kwargs, d):
    """Sequence-length curriculum: cut every [B, S, ...] tensor argument to [B, d, ...]."""
    S = None
    for t in list(inputs) + list(kwargs.values()):
        if isinstance(t, torch.Tensor) and t.dim() >= 2:
            S = t.shape[1]
            break
    if S is None or d >= S:
        return inputs, kwargs

    def cut(t):
        return t[:, :d].contiguous() if isinstance(t, torch.Tensor) and t.dim() >= 2 and t.shape[1] == S else t

    return tuple(cut(t) for t in inputs), {k: cut(v) for k, v in kwargs.items()}


class DeepSpeedEngine(EngineApiMixin, nn.Module):

    def __init__(self, args=None, model=None, optimizer=None, model_parameters=None, training_data=None,
                 lr_scheduler=None, mpu=None, dist_init_required=None, collate_fn=None, config=None,
                 config_class=None, mesh_device=None, dont_change_device=False):
        super().__init__()
        dist.init_distributed(dist_init_required=dist_init_required)
        if config is None and args is not None:
            config = getattr(args, "deepspeed_config", None)
        self._config = config_class if config_class is not None else DeepSpeedConfig(config, mpu=mpu)
        cfg = self._config
        self.mpu = mpu
        self.global_steps = 0
        self.global_samples = 0
        self.micro_steps = 0
        self.skipped_steps = 0
        self.gradient_average = True
        self.warn_unscaled_loss = True
        self.loaded_checkpoint_dp_world_size = None
        self.enable_backward_allreduce = True
        self._is_in_no_sync = False

        # device / groups
        if torch.cuda.is_available():
            self.device = torch.device("cuda", dist.get_local_rank() % max(1, torch.cuda.device_count()))
            torch.cuda.set_device(self.device)
        else:
            self.device = torch.device("cpu")
        tp = int(cfg.tensor_parallel.get("autotp_size", 1) or 1)
        sp = int(cfg.sequence_parallel_size)
        pp = 1
        if groups._State.topo is None:
            groups.initialize(tp=tp, pp=pp, sp=sp)
        self.dp_group = groups._get_sequence_data_parallel_group() if sp > 1 else groups._get_data_parallel_group()
        self.dp_world_size = dist.get_world_size(self.dp_group)
        self.seq_parallel_group = groups._get_sequence_parallel_group()
        self.mp_group = groups._get_model_parallel_group() if groups.get_model_parallel_world_size() > 1 else None
        if self.mp_group is not None and not getattr(model, "_hds_tp_size", 0):
            from ..parallel.tp import AutoTP
            AutoTP(model, self.mp_group).shard()
            model._hds_tp_size = groups.get_model_parallel_world_size()
        if sp > 1:
            from ..parallel.ulysses import enable_sequence_parallel
            enable_sequence_parallel(model, self.seq_parallel_group)
        fp = cfg.mi355x.fpdt or {}
        self.fpdt_config = None
        if fp.get("enabled", True) and fp.get("chunk_size"):
            # FPDT from the config (reference sequence/fpdt_layer.py is wired by Megatron-DeepSpeed's model code; here
            # the engine converts the Llama attention / MLP modules): chunked Ulysses attention over the SP group
            from ..parallel.fpdt import enable_fpdt
            self.fpdt_config = {"chunk_size": int(fp["chunk_size"]), "offload": bool(fp.get("offload", True)),
                                "ffn_chunks": int(fp.get("ffn_chunks", 0)), "sp": sp}
            enable_fpdt(model, self.seq_parallel_group if sp > 1 else None, self.fpdt_config["chunk_size"],
                        offload=self.fpdt_config["offload"], ffn_chunks=self.fpdt_config["ffn_chunks"])

        # timers / monitoring
        self.wall_clock_breakdown_enabled = cfg.wall_clock_breakdown
        self.timers = SynchronizedWallClockTimer() if cfg.wall_clock_breakdown else NoopTimer()
        self.engine_timers = EngineTimers(cfg.wall_clock_breakdown, cfg.wall_clock_breakdown)
        self.tput_timer = ThroughputTimer(batch_size=cfg.train_batch_size, steps_per_output=cfg.steps_per_print)
        from ..monitor.monitor import MonitorMaster
        self.monitor = MonitorMaster(cfg.monitor_config)
        dist.configure(cfg)
        from ..utils.numa import configure_rank_threads
        self.host_threads = configure_rank_threads(getattr(cfg.mi355x, "cpu_threads_per_rank", "auto"))
        from ..utils.fault_injection import FaultInjector
        self.fault_injector = FaultInjector(cfg.raw.get("fault_injection"))

        # model
        self.module = model
        self.compute_dtype = _dtype_of(cfg)
        if not dont_change_device:
            self._configure_distributed_model(model)
        self._param_names = {id(p): n for n, p in model.named_parameters()}

        # optimizer
        self.client_optimizer = optimizer
        self.client_lr_scheduler = lr_scheduler
        self.optimizer = None
        self.basic_optimizer = None
        if optimizer is not None or cfg.optimizer_name is not None or model_parameters is not None:
            self._configure_optimizer(optimizer, model_parameters)
            self._param_names = {id(p): n for n, p in model.named_parameters()}  # zero.Init swapped params
        self.lr_scheduler = self._configure_lr_scheduler(lr_scheduler)

        # data
        self.training_dataloader = self.deepspeed_io(training_data, collate_fn=collate_fn) \
            if training_data is not None else None

        # activation checkpointing (reference: the user calls deepspeed.checkpointing.configure; a config section is
        # applied here so partition_activations / contiguous buffers / profile take effect without that call)
        from .activation_checkpointing import checkpointing as _ac
        if cfg.raw.get("activation_checkpointing") and not _ac.is_configured():
            _ac.configure(mpu, deepspeed_config=cfg)
        acc = cfg.activation_checkpointing_config
        self._ac_reset = bool(acc.partition_activations or acc.contiguous_memory_optimization or acc.profile)

        # flops profiler
        self.flops_profiler = None
        if cfg.flops_profiler_config.get("enabled", False):
            from ..profiling.flops_profiler import FlopsProfiler
            self.flops_profiler = FlopsProfiler(self.module, ds_engine=self)

        # data efficiency / training-dynamics features (reference engine.py:303-330, 1985-2000)
        self.curriculum_scheduler = None
        cl = cfg.curriculum_learning
        if cl.get("enabled", False):
            from .data_pipeline.curriculum_scheduler import CurriculumScheduler
            self.curriculum_scheduler = CurriculumScheduler(cl)
            self.curriculum_type = cl.get("curriculum_type", "seqlen")
        self.progressive_layer_drop = None
        if cfg.pld_config.get("enabled", False):
            from .progressive_layer_drop import ProgressiveLayerDrop
            self.progressive_layer_drop = ProgressiveLayerDrop(cfg.pld_config.get("theta", 0.5),
                                                               cfg.pld_config.get("gamma", 0.001))
        # compression training (reference engine.py:333-337 compression_scheduler + MoQ quantizer)
        self.compression_scheduler = None
        self._moq = None
        if "compression_training" in cfg.raw:
            from ..compression import compression_scheduler, get_compression_config
            cc = get_compression_config(cfg.raw)
            if any(cc[t]["shared_parameters"]["enabled"] for t in cc if t != "layer_reduction"):
                self.compression_scheduler = compression_scheduler(self.module, cc)
                self.compression_scheduler.step(step_zero_check=True)
                wq = cc["weight_quantization"]["shared_parameters"]
                if wq["enabled"] and not wq["quantize_weight_in_forward"]:
                    from .quantize import Quantizer
                    self._moq = Quantizer(q_groups=wq["quantize_groups"],
                                          q_mixed_fp16=wq["fp16_mixed_quantize"]["enabled"],
                                          q_change_ratio=wq["fp16_mixed_quantize"]["quantize_change_ratio"],
                                          q_type=0 if wq["quantization_type"] == "symmetric" else 1,
                                          q_rounding=0 if wq["rounding"] == "nearest" else 1)
        self._activation_cache = None
        if cfg.mi355x.host_act_cache.enabled:
            from ..offload.activation_cache import build_activation_cache
            self._activation_cache = build_activation_cache(cfg.mi355x.host_act_cache, self.device).attach(self.module)
        log_dist(f"DeepSpeedEngine ready: dtype={self.compute_dtype} zero_stage={self.zero_optimization_stage()} "
                 f"dp={self.dp_world_size} micro_bs={self.train_micro_batch_size_per_gpu()} "
                 f"gas={self.gradient_accumulation_steps()}", ranks=[0])

    # ------------------------------------------------------------------------------------
    # configuration
    # ------------------------------------------------------------------------------------
    def _configure_distributed_model(self, model):
        # zero.Init-partitioned parameters stay partitioned for ZeRO-3 (the optimizer moves the per-parameter
        # partitions into its flat units); other stages need the full values back
        from .zero.partition_parameters import is_init_partitioned, unpartition_init_param
        if self.zero_optimization_stage() != 3:
            for p in model.parameters():
                if is_init_partitioned(p):
                    unpartition_init_param(p, device=self.device)
        with torch.no_grad():
            for p in model.parameters():
                if p.is_meta or is_init_partitioned(p):
                    continue
                if p.is_floating_point() and p.dtype != self.compute_dtype:
                    p.data = p.data.to(self.compute_dtype)
                if p.device != self.device:
                    p.data = p.data.to(self.device)
            for m in model.modules():
                for n, b in list(m._buffers.items()):
                    if b is not None and not b.is_meta and b.device != self.device:
                        m._buffers[n] = b.to(self.device)
        # identical initial weights on every data-parallel rank
        if self.dp_world_size > 1:
            src = dist.get_global_rank(self.dp_group, 0) if self.dp_group is not None else 0
            with torch.no_grad():
                for p in model.parameters():
                    if p.is_meta or is_init_partitioned(p):
                        continue  # Init partitions were built from rank 0's broadcast values
                    eg = groups.expert_data_group_of(p)
                    if eg is not False:
                        # expert params: replicas live in the expert-data-parallel group only
                        if eg is not None and dist.get_world_size(eg) > 1:
                            dist.broadcast(p.data, dist.get_global_rank(eg, 0), group=eg)
                        continue
                    dist.broadcast(p.data, src, group=self.dp_group)
                for b in model.buffers():
                    if not b.is_meta:
                        dist.broadcast(b.data, src, group=self.dp_group)

    def _basic_optimizer(self, model_parameters):
        cfg = self._config
        name = cfg.optimizer_name or "adamw"
        params = dict(cfg.optimizer_params)
        from ..ops import optimizers as fo
        if model_parameters is None:
            model_parameters = [p for p in self.module.parameters() if p.requires_grad]
        model_parameters = list(model_parameters)
        if name in ("adam", "adamw", "fusedadam"):
            adam_w_mode = params.pop("adam_w_mode", True)
            if name == "adamw":
                adam_w_mode = True
            params.pop("torch_adam", None)
            params.pop("fused", None)
            return fo.FusedAdam(model_parameters, adam_w_mode=adam_w_mode, **params)
        if name == "lion":
            return fo.FusedLion(model_parameters, **params)
        if name == "lamb":
            return fo.FusedLamb(model_parameters, **params)
        if name == "adagrad":
            return torch.optim.Adagrad(model_parameters, **params)
        if name == "sgd":
            return torch.optim.SGD(model_parameters, **params)
        if name in ("muadam", "muadamw", "musgd"):
            from ..ops import mup
            cls = {"muadam": mup.MuAdam, "muadamw": mup.MuAdamW, "musgd": mup.MuSGD}[name]
            params.pop("torch_adam", None)
            return cls(model_parameters, **params)
        if name in ("onebitadam", "zerooneadam", "onebitlamb"):
            from .fp16.onebit import make_onebit
            return make_onebit(name, model_parameters, params, self)
        return getattr(torch.optim, cfg.optimizer_name)(model_parameters, **params)

    def _configure_optimizer(self, client_optimizer, model_parameters):
        cfg = self._config
        if client_optimizer is not None and not callable(client_optimizer):
            basic = client_optimizer
        elif client_optimizer is not None:
            basic = client_optimizer(model_parameters or self.module.parameters())
        else:
            basic = self._basic_optimizer(model_parameters)
        self.basic_optimizer = basic
        stage = cfg.zero_optimization_stage
        zc = cfg.zero_config
        from .fp16.onebit import OnebitZeroOptimizer, _OnebitBase
        if isinstance(basic, _OnebitBase):
            cls = OnebitZeroOptimizer
        elif zc.offload_optimizer.enabled or zc.offload_param.enabled:
            from .zero.offload import OffloadZeroOptimizer
            cls = OffloadZeroOptimizer
        else:
            cls = ZeroOptimizer
        leaf = getattr(self.module, "_z3_leaf_modules", ())
        self.optimizer = cls(basic, self.module, cfg, stage, dp_group=self.dp_group, dtype=self.compute_dtype,
                             device=self.device, grad_accum_steps=cfg.gradient_accumulation_steps,
                             timers=self.timers, mpu=self.mpu, leaf_modules=leaf, param_names=self._param_names,
                             mp_group=self.mp_group)

    def _configure_lr_scheduler(self, client_lr_scheduler):
        cfg = self._config
        if client_lr_scheduler is not None:
            if callable(client_lr_scheduler) and not hasattr(client_lr_scheduler, "step"):
                return client_lr_scheduler(self.basic_optimizer)
            return client_lr_scheduler
        if cfg.scheduler_name is not None and self.optimizer is not None:
            return lr_schedules.get_scheduler(cfg.scheduler_name, self.optimizer, cfg.scheduler_params)
        return None

    # ------------------------------------------------------------------------------------
    # config accessors (reference names)
    # ------------------------------------------------------------------------------------
    @property
    def config(self):
        return self._config.raw

    def train_batch_size(self):
        return self._config.train_batch_size

    def train_micro_batch_size_per_gpu(self):
        return self._config.train_micro_batch_size_per_gpu

    def gradient_accumulation_steps(self):
        return self._config.gradient_accumulation_steps

    def set_gradient_accumulation_boundary(self, is_boundary):
        self._force_boundary = is_boundary

    def zero_optimization(self):
        return self._config.zero_enabled

    def zero_optimization_stage(self):
        return self._config.zero_optimization_stage

    def bfloat16_enabled(self):
        return self._config.bfloat16_enabled

    def fp16_enabled(self):
        return self._config.fp16_enabled

    def gradient_clipping(self):
        return self._config.gradient_clipping

    def steps_per_print(self):
        return self._config.steps_per_print

    def get_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups] if self.optimizer else []

    def get_global_grad_norm(self):
        return self.optimizer.get_global_norm() if self.optimizer else None

    def is_gradient_accumulation_boundary(self):
        forced = getattr(self, "_force_boundary", None)
        if forced is not None:
            return forced
        return (self.micro_steps + 1) % self.gradient_accumulation_steps() == 0

    def sequence_shard_indices(self, seq_len):
        """Global token positions of a length-``seq_len`` sequence this rank feeds the model: all of them without
        sequence parallelism, its contiguous 1/sp slice under Ulysses, its load-balanced chunk set under FPDT
        (parallel/fpdt.FPDTInputConstruct). Index both the inputs and the next-token targets with it."""
        sp = int(self._config.sequence_parallel_size)
        rank = dist.get_rank(self.seq_parallel_group) if sp > 1 else 0
        if self.fpdt_config is not None:
            from ..parallel.fpdt import fpdt_layout_indices
            return fpdt_layout_indices(seq_len, self.fpdt_config["chunk_size"], sp, rank)
        n = seq_len // sp
        return torch.arange(rank * n, (rank + 1) * n)

    fpdt_input_indices = sequence_shard_indices

    def get_data_parallel_world_size(self):
        return self.dp_world_size

    @property
    def data_parallel_group(self):
        return self.dp_group

    def wall_clock_breakdown(self):
        return self.wall_clock_breakdown_enabled

    # ------------------------------------------------------------------------------------
    # training loop
    # ------------------------------------------------------------------------------------
    def deepspeed_io(self, dataset, batch_size=None, route="train", pin_memory=None, data_sampler=None,
                     collate_fn=None, num_local_io_workers=None):
        bs = batch_size or self.train_micro_batch_size_per_gpu()
        return DeepSpeedDataLoader(dataset, bs, pin_memory=pin_memory, collate_fn=collate_fn,
                                   num_local_io_workers=num_local_io_workers, data_sampler=data_sampler,
                                   data_parallel_world_size=self.dp_world_size,
                                   data_parallel_rank=dist.get_rank(self.dp_group))

    def forward(self, *inputs, **kwargs):
        if self.flops_profiler is not None and self.global_steps == self._config.flops_profiler_config.get(
                "profile_step", 1):
            self.flops_profiler.start_profile()
        self.timers(FORWARD_MICRO_TIMER).start()
        if self.curriculum_scheduler is not None and self.module.training:
            d = self.curriculum_scheduler.update_difficulty(self.global_steps + 1)
            if self.curriculum_type == "seqlen":
                inputs, kwargs = _truncate_seqlen(inputs, kwargs, int(d))
            else:
                kwargs["curriculum_seqlen"] = d
        if self.progressive_layer_drop is not None and self.module.training:
            kwargs.update(self.progressive_layer_drop.get_state())
        if self.optimizer is not None:
            self.optimizer.pre_forward()
        if self._ac_reset and self.module.training:
            from .activation_checkpointing import checkpointing as _ac
            _ac.reset()  # rewind the contiguous checkpoint buffers, log the profile
        ctx = self._activation_cache.forward_context() if (self._activation_cache is not None and
                                                             self.module.training) else contextlib.nullcontext()
        with ctx:
            out = self.module(*inputs, **kwargs)
        if self.optimizer is not None:
            self.optimizer.post_forward()
        self.timers(FORWARD_MICRO_TIMER).stop()
        if self.flops_profiler is not None and self.flops_profiler.started:
            self.flops_profiler.stop_profile()
            if dist.get_rank() == 0:
                self.flops_profiler.print_model_profile(profile_step=self.global_steps)
            self.flops_profiler.end_profile()
        return out

    def backward(self, loss, allreduce_gradients=True, release_loss=False, retain_graph=False, scale_wrt_gas=True):
        assert self.optimizer is not None, "engine.backward() requires an optimizer"
        self.timers(BACKWARD_MICRO_TIMER).start()
        if scale_wrt_gas and self.gradient_accumulation_steps() > 1:
            loss = loss / self.gradient_accumulation_steps()
        boundary = self.is_gradient_accumulation_boundary() and not self._is_in_no_sync
        z = self.optimizer
        hold = not allreduce_gradients and self.zero_optimization_stage() < 3 and hasattr(z, "hold_reduction")
        if hold:  # reduced by a later engine.allreduce_gradients() (reference engine.py:2245)
            self._pipe_hold = bool(z.hold_reduction)
            z.hold_reduction = True
        z.prepare_backward(boundary)
        z.backward(loss, retain_graph=retain_graph)
        z.finish_backward()
        self.timers(BACKWARD_MICRO_TIMER).stop()
        if self.monitor.enabled and dist.get_rank() == 0 and boundary:
            self.summary_events = [("Train/Samples/train_loss", float(loss.detach().item()), self.global_samples)]
            self.monitor.write_events(self.summary_events)
        return loss

    @contextlib.contextmanager
    def no_sync(self):
        assert self.zero_optimization_stage() < 2, "no_sync is incompatible with ZeRO-2/3 (gradient partitioning)"
        prev = self._is_in_no_sync
        self._is_in_no_sync = True
        try:
            yield
        finally:
            self._is_in_no_sync = prev

    def step(self, lr_kwargs=None):
        self.timers(STEP_MICRO_TIMER).start()
        boundary = self.is_gradient_accumulation_boundary()
        if boundary:
            if getattr(self.optimizer, "_held", None):  # backward(allreduce_gradients=False) without the call
                self.allreduce_gradients()
            ok = self.optimizer.step()
            self._step_applied = ok is not False
            if ok is False:
                self.skipped_steps += 1
            elif self.lr_scheduler is not None:
                self.lr_scheduler.step(**(lr_kwargs or {}))
            self.global_steps += 1
            self.global_samples += self.train_batch_size()
            if self.fault_injector.enabled:
                self.fault_injector.maybe_fire(dist.get_rank(), self.global_steps)
            if self.compression_scheduler is not None:
                self.compression_scheduler.step()
                if self._moq is not None and self.compression_scheduler.weight_quantization_enabled:
                    qparams = [p for p in self.module.parameters() if getattr(p, "start_bits", None)]
                    self._moq.quantize([qparams], overflow=ok is False)
            if self.progressive_layer_drop is not None:
                self.progressive_layer_drop.update_state(self.global_steps)
            if self._config.autotuning.get("enabled", False):
                self._autotuning_step()
            if self.monitor.enabled and dist.get_rank() == 0:
                self.monitor.write_events([("Train/Samples/lr", self.get_lr()[0], self.global_samples)])
            if self.global_steps % self.steps_per_print() == 0 and self.wall_clock_breakdown():
                self.timers.log([FORWARD_MICRO_TIMER, BACKWARD_MICRO_TIMER, STEP_MICRO_TIMER])
        if boundary and getattr(self, "_dc_backend", None) is not None:
            self._dc_backend.on_step_end()
        self.micro_steps += 1
        self._force_boundary = None
        self.timers(STEP_MICRO_TIMER).stop()

    def _autotuning_step(self):
        """Autotuning experiment hook (reference engine.py:2458-2480): time steps (start, end], write the
        metric file and, when launched by the autotuner, end the process."""
        import json
        import sys
        import time
        at = self._config.autotuning
        start, end = int(at.get("start_profile_step", 3)), int(at.get("end_profile_step", 5))
        if self.global_steps == start:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._at_t0 = time.time()
        elif self.global_steps == end and getattr(self, "_at_t0", None) is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            dt = (time.time() - self._at_t0) / max(1, end - start)
            metric = {"throughput": self.train_batch_size() / dt, "latency": dt,
                      "train_micro_batch_size_per_gpu": self.train_micro_batch_size_per_gpu(),
                      "zero_stage": self.zero_optimization_stage()}
            path = at.get("metric_path")
            if path and dist.get_rank() == 0:
                with open(path, "w") as f:
                    json.dump(metric, f)
            if os.environ.get("HDS_AUTOTUNING_EXIT") == "1":
                dist.barrier()
                sys.exit(0)

    def set_custom_curriculum_learning_schedule(self, schedule_func_dict):
        if self.curriculum_scheduler is not None:
            self.curriculum_scheduler.set_custom_get_difficulty(schedule_func_dict)

    def get_pld_theta(self):
        return self.progressive_layer_drop.get_theta() if self.progressive_layer_drop else None

    def zero_grad(self):
        if self.optimizer is not None:
            self.optimizer.zero_grad()

    def train(self, mode=True):
        self.module.train(mode)
        return self

    def eval(self):
        self.module.eval()
        return self

    # ------------------------------------------------------------------------------------
    # checkpointing (layout: runtime/checkpointing.py)
    # ------------------------------------------------------------------------------------
    def _settle_host_step(self):
        """An asynchronous host step (state offload host_step) or an overlapped device step may still be writing
        parameters: finish it before anything reads the parameters or states outside the forward's per-unit
        waits."""
        so = getattr(self.optimizer, "state_offload", None)
        if so is not None and hasattr(so, "join"):
            so.join()
        join = getattr(self.optimizer, "_join_step", None)
        if join is not None:
            join()  # an overlapped device step (ZeRO-3) may still be updating shards on its stream

    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True, exclude_frozen_parameters=False):
        self._settle_host_step()
        from .checkpointing import save_checkpoint
        return save_checkpoint(self, save_dir, tag, client_state or {}, save_latest, exclude_frozen_parameters)

    def load_checkpoint(self, load_dir, tag=None, load_module_strict=True, load_optimizer_states=True,
                        load_lr_scheduler_states=True, load_module_only=False, custom_load_fn=None):
        self._settle_host_step()
        from .checkpointing import load_checkpoint
        return load_checkpoint(self, load_dir, tag, load_module_strict, load_optimizer_states,
                               load_lr_scheduler_states, load_module_only)

    def save_16bit_model(self, save_dir, save_filename="pytorch_model.bin", exclude_frozen_parameters=False):
        """Consolidated 16-bit weights. Under ZeRO-3 this needs ``stage3_gather_16bit_weights_on_model_save``, as in
        the reference (engine.py:3835): without it nothing is gathered and False is returned."""
        from .checkpointing import save_16bit_model
        self._settle_host_step()
        if self.zero_optimization_partition_weights() and getattr(self.optimizer, "partitioned", False) and \
                not self.zero_gather_16bit_weights_on_model_save():
            logger.warning("Did not save the model: zero_optimization.stage3_gather_16bit_weights_on_model_save is "
                           "false under ZeRO-3 (use zero_to_fp32 on a checkpoint instead)")
            return False
        return save_16bit_model(self, save_dir, save_filename)

    def module_state_dict(self, destination=None, prefix="", keep_vars=False, exclude_frozen_parameters=False):
        self._settle_host_step()
        if self.zero_optimization_stage() == 3 and self.optimizer.partitioned:
            return None
        return self.module.state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)

    # ------------------------------------------------------------------------------------
    # DeepCompile entry (reference engine.py:3876-3941); see runtime/compile.py
    # ------------------------------------------------------------------------------------
    def compile(self, backend="native", compile_kwargs=None, schedule=None):
        if getattr(self, "_is_compiled", False):
            return
        from .compile import compile_engine
        self._compile_times = compile_engine(self, backend, compile_kwargs or {}, schedule)
        self._is_compiled = True

    @property
    def is_compiled(self):
        return getattr(self, "_is_compiled", False)

    def is_deepcompile_enabled(self):
        return bool(self._config.raw.get("compile", {}).get("deepcompile", False))

    def get_compile_time(self):
        return dict(getattr(self, "_compile_times", {}))

    def register_compile_pass(self, pass_name, pass_fn):
        from .compile import register_compile_pass
        register_compile_pass(pass_name, pass_fn)

    def offload_states(self, include=None, device="cpu", pin_memory=True, non_blocking=False):
        from .zero.offload_states import offload_states
        offload_states(self.optimizer, include, device, pin_memory, non_blocking)

    def reload_states(self, non_blocking=False):
        from .zero.offload_states import reload_states
        reload_states(self.optimizer, non_blocking)
