"""DeepSpeed-schema JSON config (same keys, same batch triangulation) + an ``mi355x`` section.

Reference parity: runtime/config.py (``DeepSpeedConfig`` :708, batch triangulation :923-960),
runtime/zero/config.py (``DeepSpeedZeroConfig`` :86, field defaults :91-344),
runtime/zero/offload_config.py, runtime/constants.py. Users' existing ds_config.json files load
unchanged; unknown keys are kept in ``raw`` and ignored.

MI355X-specific knobs live under ``"mi355x"``::

    "mi355x": {
        "xgmi_bucket_mb": 256,          # default ZeRO-1/2 bucket / ZeRO-3 prefetch granularity
        "zero3_prefetch_depth": 2,      # units all-gathered ahead of compute
        "zero3_max_reduce_inflight": 2, # gradient reduce-scatters in flight before the oldest is retired
        "host_act_cache": {"enabled": false, "slots": 8, "slot_mb": 512, "min_layers_resident": 2},
        "fused_lm_head_ce": true,
        "comm_high_priority": true      # ZeRO-3 AG/RS communicators on high-priority streams
    }
"""
import copy
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, Optional

from ..utils.logging import logger

ADAM, ADAMW, LAMB, LION, ADAGRAD, SGD, ONEBIT_ADAM, ONEBIT_LAMB, ZERO_ONE_ADAM, CPU_ADAM = (
    "adam", "adamw", "lamb", "lion", "adagrad", "sgd", "onebitadam", "onebitlamb", "zerooneadam", "cpuadam")


def _get(d, key, default):
    v = d.get(key, default) if isinstance(d, dict) else default
    return default if v is None else v


class ConfigError(ValueError):
    pass


@dataclass
class OffloadDeviceConfig:
    device: str = "none"  # none | cpu | nvme
    nvme_path: Optional[str] = None
    buffer_count: int = 5
    buffer_size: int = int(1e8)
    max_in_cpu: int = int(1e9)
    pin_memory: bool = False
    pipeline_read: bool = False
    pipeline_write: bool = False
    fast_init: bool = False
    ratio: float = 1.0

    @classmethod
    def from_dict(cls, d):
        d = d or {}
        kw = {f.name: d[f.name] for f in fields(cls) if f.name in d}
        return cls(**kw)

    @property
    def enabled(self):
        return self.device not in (None, "none")


@dataclass
class ZeroConfig:
    stage: int = 0
    contiguous_gradients: bool = True
    reduce_scatter: bool = True
    reduce_bucket_size: int = int(5e8)
    use_multi_rank_bucket_allreduce: bool = True
    allgather_partitions: bool = True
    allgather_bucket_size: int = int(5e8)
    overlap_comm: bool = True
    load_from_fp32_weights: bool = True
    elastic_checkpoint: bool = False
    offload_param: OffloadDeviceConfig = field(default_factory=OffloadDeviceConfig)
    offload_optimizer: OffloadDeviceConfig = field(default_factory=OffloadDeviceConfig)
    sub_group_size: int = int(1e9)
    prefetch_bucket_size: int = int(5e7)
    param_persistence_threshold: int = int(1e5)
    model_persistence_threshold: int = 2**63 - 1
    max_live_parameters: int = int(1e9)
    max_reuse_distance: int = int(1e9)
    gather_16bit_weights_on_model_save: bool = False
    module_granularity_threshold: int = 0
    use_all_reduce_for_fetch_params: bool = False
    stage3_gather_fp16_weights_on_model_save: bool = False
    ignore_unused_parameters: bool = True
    legacy_stage1: bool = False
    round_robin_gradients: bool = False
    zero_hpz_partition_size: int = 1
    zero_quantized_weights: bool = False
    zero_quantized_nontrainable_weights: bool = False
    zero_quantized_gradients: bool = False
    mics_shard_size: int = -1
    mics_hierarchical_params_gather: bool = False
    memory_efficient_linear: bool = True
    pipeline_loading_checkpoint: bool = False
    override_module_apply: bool = True
    log_trace_cache_warnings: bool = False
    safe_mode: bool = False

    _ALIASES = {
        "stage3_prefetch_bucket_size": "prefetch_bucket_size",
        "stage3_param_persistence_threshold": "param_persistence_threshold",
        "stage3_model_persistence_threshold": "model_persistence_threshold",
        "stage3_max_live_parameters": "max_live_parameters",
        "stage3_max_reuse_distance": "max_reuse_distance",
        "stage3_gather_16bit_weights_on_model_save": "gather_16bit_weights_on_model_save",
        "cpu_offload": None,
    }

    @classmethod
    def from_dict(cls, d):
        d = dict(d or {})
        kw = {}
        for k, v in list(d.items()):
            if k in cls._ALIASES:
                tgt = cls._ALIASES[k]
                if tgt is None:
                    if v:
                        kw["offload_optimizer"] = OffloadDeviceConfig(device="cpu", pin_memory=True)
                    continue
                kw[tgt] = v
        names = {f.name for f in fields(cls)}
        for k, v in d.items():
            if k in names:
                kw[k] = v
        for k in ("offload_param", "offload_optimizer"):
            if k in kw and not isinstance(kw[k], OffloadDeviceConfig):
                kw[k] = OffloadDeviceConfig.from_dict(kw[k])
        for k in ("reduce_bucket_size", "allgather_bucket_size", "sub_group_size", "prefetch_bucket_size",
                  "param_persistence_threshold", "max_live_parameters", "max_reuse_distance"):
            if k in kw:
                kw[k] = int(kw[k])
        z = cls(**kw)
        if z.stage not in (0, 1, 2, 3):
            raise ConfigError(f"zero_optimization.stage must be 0..3, got {z.stage}")
        return z


@dataclass
class LossScaleConfig:
    enabled: bool = False
    loss_scale: float = 0.0  # 0 -> dynamic
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    hysteresis: int = 2
    consecutive_hysteresis: bool = False
    min_loss_scale: float = 1.0
    auto_cast: bool = False


@dataclass
class ActivationCheckpointingConfig:
    partition_activations: bool = False
    contiguous_memory_optimization: bool = False
    cpu_checkpointing: bool = False
    number_checkpoints: Optional[int] = None
    synchronize_checkpoint_boundary: bool = False
    profile: bool = False


@dataclass
class HostActCacheConfig:
    enabled: bool = False
    slots: int = 8
    slot_mb: int = 512
    min_layers_resident: int = 2
    # "budget": spill only what exceeds gpu_budget_gib; "recompute": checkpoint those layers instead of spilling;
    # "all": spill every eligible layer; "ckpt_offload": checkpoint EVERY block and spill its inputs (the only
    # tensors a checkpointed block keeps) -- long context, where even the checkpoints do not fit in HBM; "auto":
    # "recompute", then the earliest planned blocks switch to spilling as far as PCIe can hide them
    policy: str = "budget"
    spill_overlap: float = 0.5  # policy "auto": fraction of the forward the spilled blocks' D2H may take
    gpu_budget_gib: float = 0.0  # 0: 92% of device memory
    prefetch_layers: int = 4  # spilled blocks whose H2D starts when backward reaches a later block
    host_budget_gib: float = 0.0  # pinned host bytes the cache may hold (0: 40% of host RAM over the node's ranks, <= 160 GiB)
    copy_window_gib: float = 0.0  # queued-but-unfinished copy bytes per direction (0: from the HBM headroom)
    # policy "plan" (offload/act_plan.py): per-tensor keep / spill / recompute. The modelled cost of a hidden spill
    # (concurrent kernels slow down while a copy runs), and optional fixed {tensor class: action} overrides
    spill_cost_ms_per_gb: float = 0.6
    # policy "ckpt_offload": also keep (and spill) each block's attention output + LSE so the recompute skips the
    # FlashAttention forward
    stash_attention: bool = True
    forced_actions: Optional[dict] = None
    # accept spills through unlimited runtime blit kernels (DEBUG_CLR_LIMIT_BLIT_WG missing when HIP loaded)
    allow_unlimited_blit: bool = False
    # refuse (BlitLimitError) instead of warning when spills would run as unlimited blit kernels
    strict_blit_limit: bool = False
    # smallest saved tensor the cache moves (KiB); smaller ones stay on the device
    min_kib: float = 1024.0


AUTO = -1


def _auto_or(v, typ):
    return AUTO if isinstance(v, str) and v.lower() == "auto" else typ(v)


@dataclass
class MI355XConfig:
    xgmi_bucket_mb: int = 256
    zero3_prefetch_depth: int = 2
    zero3_max_reduce_inflight: int = 2
    zero3_unit_bucket_mb: float = 128  # per-submodule ZeRO-3 units of ModuleList-free models are bucketed to this
    direct_wgrad: bool = True  # weight-gradient GEMMs write into the flat gradient buffer (runtime/zero/linear.py)
    # ZeRO-3 with device-resident optimizer states: step() queues the fused update unit by unit (forward order) on a
    # side HIP stream and returns; each unit's forward waits only for its own piece (runtime/zero/optimizer.py
    # ``_overlap_ok``). Off by default: on one MI355X the headline ran 24,837 / 24,883 tok/s with it against 24,909 /
    # 24,913 without -- hipBLASLt's GEMM workgroups leave no room on a CU for the update's waves, so the two take
    # turns instead of overlapping (profiles/r6/overlap_step/)
    overlap_step: bool = False
    fused_lm_head_ce: bool = True
    # ZeRO-3 all-gather / reduce-scatter communicators run their RCCL kernels on high-priority HIP streams, so
    # the few workgroups a collective needs are dispatched ahead of queued GEMM tiles (overlap under full load)
    comm_high_priority: bool = True
    # per-step exposed-communication / busbw accounting of the ZeRO collectives (runtime/zero/comm_stats.py)
    comm_stats: bool = False
    # ZeRO-3 unit collectives: "auto" measures rccl / native / symmetric per size class at dp > 1 and routes each
    # class to the fastest (runtime/zero/transport.py); "auto:rccl,symmetric" limits the candidates; "rccl" keeps
    # torch.distributed
    zero_comm_transport: str = "auto"
    # the ZeRO-3 fetch / wait / prefetch events also start / stop the engine timers (reference ENABLE_PROFILER)
    zero3_event_timers: bool = False
    # host threads per rank of the C++ kernels (CPU Adam / Lion / Adagrad, host-step tails, NVMe tier) and of torch's
    # CPU ops: "auto" = the rank's share of the node's CPUs (its NUMA node's when sysfs says where its GPU sits) when
    # several ranks share the host and the count was not set explicitly (torchrun forces OMP_NUM_THREADS=1), else
    # left alone; an int forces it
    cpu_threads_per_rank: object = "auto"
    # FPDT (Ulysses-Offload) attention from the config (parallel/fpdt.py): {"enabled": bool, "chunk_size": global
    # tokens per attention segment, "offload": park each segment's q/k/v/o/lse in pinned host memory between forward
    # and backward, "ffn_chunks": > 1 also runs the MLPs in sequence chunks}; inputs in the FPDT layout
    # (engine.fpdt_input_indices)
    fpdt: Optional[dict] = None
    host_act_cache: HostActCacheConfig = field(default_factory=HostActCacheConfig)


class DeepSpeedConfig:
    """Parsed config. ``config`` may be a dict, a JSON path, or a JSON string."""

    def __init__(self, config, mpu=None, mesh_device=None, world_size=None):
        if isinstance(config, DeepSpeedConfig):
            config = config.raw
        if isinstance(config, str):
            if os.path.exists(config):
                with open(config) as f:
                    config = json.load(f)
            else:
                config = json.loads(config)
        if config is None:
            config = {}
        self.raw = copy.deepcopy(config)
        c = self.raw
        if world_size is None:
            from .. import comm as dist
            world_size = dist.get_world_size()
            if mpu is not None and hasattr(mpu, "get_data_parallel_world_size"):
                world_size = mpu.get_data_parallel_world_size()
            elif mesh_device is not None:
                world_size = mesh_device.get_group(mesh_dim="data_parallel").size()
        self.world_size = world_size

        # batch
        self.train_batch_size = c.get("train_batch_size")
        self.train_micro_batch_size_per_gpu = c.get("train_micro_batch_size_per_gpu")
        self.gradient_accumulation_steps = c.get("gradient_accumulation_steps")
        if (c.get("elasticity") or {}).get("enabled", False):
            self._apply_elasticity(c)
        self._triangulate_batch()

        # optimizer / scheduler
        opt = c.get("optimizer") or {}
        self.optimizer_name = opt.get("type", None)
        self.optimizer_name = self.optimizer_name.lower() if self.optimizer_name else None
        self.optimizer_params = dict(opt.get("params", {}) or {})
        self.optimizer_legacy_fusion = opt.get("legacy_fusion", False)
        sch = c.get("scheduler") or {}
        self.scheduler_name = sch.get("type")
        self.scheduler_params = dict(sch.get("params", {}) or {})

        # precision
        bf = c.get("bf16") or c.get("bfloat16") or {}
        self.bfloat16_enabled = bool(_get(bf, "enabled", False))
        self.bfloat16_immediate_grad_update = bool(_get(bf, "immediate_grad_update", False))
        fp = c.get("fp16") or {}
        self.fp16_enabled = bool(_get(fp, "enabled", False))
        self.loss_scale_config = LossScaleConfig(
            enabled=self.fp16_enabled, loss_scale=float(_get(fp, "loss_scale", 0.0)),
            initial_scale_power=int(_get(fp, "initial_scale_power", 16)),
            loss_scale_window=int(_get(fp, "loss_scale_window", 1000)), hysteresis=int(_get(fp, "hysteresis", 2)),
            consecutive_hysteresis=bool(_get(fp, "consecutive_hysteresis", False)),
            min_loss_scale=float(_get(fp, "min_loss_scale", 1.0)), auto_cast=bool(_get(fp, "auto_cast", False)))
        if self.fp16_enabled and self.bfloat16_enabled:
            raise ConfigError("bf16 and fp16 cannot both be enabled")
        self.amp_enabled = bool(_get(c.get("amp") or {}, "enabled", False))
        dt = c.get("data_types") or {}
        self.grad_accum_dtype = dt.get("grad_accum_dtype")
        self.communication_data_type = c.get("communication_data_type")
        self.seq_parallel_communication_data_type = c.get("seq_parallel_communication_data_type", "fp32")

        # zero
        self.zero_config = ZeroConfig.from_dict(c.get("zero_optimization") or {})
        self.zero_optimization_stage = self.zero_config.stage
        self.zero_enabled = self.zero_optimization_stage > 0
        self.zero_allow_untested_optimizer = c.get("zero_allow_untested_optimizer", True)
        self.zero_force_ds_cpu_optimizer = c.get("zero_force_ds_cpu_optimizer", True)

        # misc training
        self.gradient_clipping = float(c.get("gradient_clipping", 0.0) or 0.0)
        self.prescale_gradients = bool(c.get("prescale_gradients", False))
        self.gradient_predivide_factor = float(c.get("gradient_predivide_factor", 1.0))
        self.sparse_gradients_enabled = bool(c.get("sparse_gradients", False))
        self.steps_per_print = int(c.get("steps_per_print", 10) or 10)
        self.wall_clock_breakdown = bool(c.get("wall_clock_breakdown", False))
        self.memory_breakdown = bool(c.get("memory_breakdown", False))
        self.dump_state = bool(c.get("dump_state", False))
        self.disable_allgather = bool(c.get("disable_allgather", False))
        self.seed = c.get("seed", 1234)

        ac = c.get("activation_checkpointing") or {}
        self.activation_checkpointing_config = ActivationCheckpointingConfig(
            **{f.name: ac[f.name] for f in fields(ActivationCheckpointingConfig) if f.name in ac})

        self.comms_logger = c.get("comms_logger")
        self.flops_profiler_config = c.get("flops_profiler") or {}
        self.monitor_config = {k: c.get(k) for k in ("tensorboard", "wandb", "csv_monitor", "comet") if k in c}
        self.checkpoint_config = c.get("checkpoint") or {}
        self.checkpoint_tag_validation_enabled = self.checkpoint_config.get("tag_validation", "Warn") != "Ignore"
        self.checkpoint_tag_validation_fail = self.checkpoint_config.get("tag_validation", "Warn") == "Fail"
        self.load_universal_checkpoint = bool(self.checkpoint_config.get("load_universal", False))
        self.use_node_local_storage = bool(self.checkpoint_config.get("use_node_local_storage", False))
        self.pipeline = c.get("pipeline") or {}
        self.tensor_parallel = c.get("tensor_parallel") or {}
        self.sequence_parallel_size = int(c.get("sequence_parallel_size", 1) or 1)
        self.elasticity = c.get("elasticity") or {}
        self.autotuning = c.get("autotuning") or {}
        self.compile_config = c.get("compile") or {}
        self.aio_config = c.get("aio") or {}
        self.hybrid_engine = c.get("hybrid_engine") or {}
        self.curriculum_learning = c.get("curriculum_learning") or {}
        self.pld_config = c.get("progressive_layer_drop") or {}
        self.eigenvalue_config = c.get("eigenvalue") or {}
        self.quantize_training = c.get("quantize_training") or {}
        self.data_efficiency = c.get("data_efficiency") or {}
        self.compression_training = c.get("compression_training") or {}

        m = c.get("mi355x") or {}
        hac = m.get("host_act_cache") or {}
        self.mi355x = MI355XConfig(
            # "auto": sized from an alpha-beta fit of the data-parallel all-gather measured at startup (AUTO = -1)
            # default "auto": at dp > 1 the buckets follow the measured xGMI all-gather (at dp = 1: 256 / 128 MiB)
            xgmi_bucket_mb=_auto_or(m.get("xgmi_bucket_mb", "auto"), int),
            zero3_prefetch_depth=int(m.get("zero3_prefetch_depth", 2)),
            zero3_max_reduce_inflight=int(m.get("zero3_max_reduce_inflight", 2)),
            zero3_unit_bucket_mb=_auto_or(m.get("zero3_unit_bucket_mb", "auto"), float),
            comm_stats=bool(m.get("comm_stats", False)),
            zero_comm_transport=str(m.get("zero_comm_transport", "auto")),
            zero3_event_timers=bool(m.get("zero3_event_timers", False)),
            cpu_threads_per_rank=m.get("cpu_threads_per_rank", "auto"),
            fpdt=dict(m["fpdt"]) if m.get("fpdt") else None,
            direct_wgrad=bool(m.get("direct_wgrad", True)),
            overlap_step=bool(m.get("overlap_step", False)),
            fused_lm_head_ce=bool(m.get("fused_lm_head_ce", True)),
            comm_high_priority=bool(m.get("comm_high_priority", True)),
            host_act_cache=HostActCacheConfig(**{f.name: hac[f.name]
                                                 for f in fields(HostActCacheConfig) if f.name in hac}))

    # -------------------------------------------------------------------------------------
    def _triangulate_batch(self):
        """train_batch = micro * gas * world (reference runtime/config.py:923-960)."""
        tb, mb, gas, ws = self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps, \
            self.world_size
        if tb is not None and mb is not None and gas is not None:
            pass
        elif tb is not None and mb is not None:
            gas = tb // (mb * ws)
        elif tb is not None and gas is not None:
            mb = tb // (gas * ws)
        elif mb is not None and gas is not None:
            tb = mb * gas * ws
        elif tb is not None:
            gas = 1
            mb = tb // ws
        elif mb is not None:
            gas = 1
            tb = mb * ws
        else:
            mb, gas, tb = 1, 1, ws
        if gas is None or gas < 1 or mb is None or mb < 1:
            raise ConfigError(f"invalid batch config: train_batch_size={tb} micro={mb} gas={gas} world={ws}")
        if tb != mb * gas * ws:
            raise ConfigError(f"Check batch related parameters. train_batch_size is not equal to micro_batch_per_gpu "
                              f"* gradient_acc_step * world_size {tb} != {mb} * {gas} * {ws}")
        self.train_batch_size, self.train_micro_batch_size_per_gpu, self.gradient_accumulation_steps = tb, mb, gas

    def _apply_elasticity(self, c):
        """Elastic batch plan overrides the batch keys (reference runtime/config.py:758-800)."""
        from ..elasticity import compute_elastic_config, ensure_immutable_elastic_config
        from ..elasticity.elasticity import ElasticityConfig
        from ..version import __version__
        ec = ElasticityConfig(c["elasticity"])
        ensure_immutable_elastic_config(c["elasticity"])
        bs, gpus, mbs = compute_elastic_config(c, __version__, world_size=self.world_size)
        if not ec.ignore_non_elastic_batch_info:
            for k in ("train_batch_size", "train_micro_batch_size_per_gpu", "gradient_accumulation_steps"):
                if c.get(k) is not None:
                    raise ConfigError(f"elasticity is enabled: remove '{k}' or set ignore_non_elastic_batch_info")
        self.train_batch_size = bs
        self.train_micro_batch_size_per_gpu = mbs
        self.gradient_accumulation_steps = bs // (mbs * self.world_size)
        self.elastic_valid_gpus = gpus

    def print(self, name="DeepSpeedEngine configuration"):
        logger.info(f"{name}: {json.dumps(self.raw, indent=2, default=str)}")

    def __getitem__(self, k):
        return self.raw[k]

    def get(self, k, default=None):
        return self.raw.get(k, default)
