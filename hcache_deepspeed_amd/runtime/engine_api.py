"""The rest of ``DeepSpeedEngine``'s public surface: config accessors under the reference's names and the behavioural
methods HF Accelerate / Trainer and Megatron-DeepSpeed call.

Reference: /root/reference/deepspeed/runtime/engine.py -- the accessor block :580-1010 (``*_enabled``, ``zero_*``,
``flops_profiler_*``, ``eigenvalue_*``, ``autotuning_*``), ``destroy`` :499, ``get_batch_info`` :528,
``set_train_batch_size`` / ``set_train_micro_batch_size`` :544-571, ``set_data_post_process_func`` :573,
``random_ltd_initialize`` :691, ``is_first_weights_partition_group`` :873, ``load_universal_checkpoint`` :958,
``dump_state`` :1012, ``was_step_applied`` :1844, ``print_forward_breakdown`` :2080, ``allreduce_gradients`` :2104,
``clip_fp32_gradients`` :2269, ``get_mom`` :2530, the DDP helpers ``allreduce_bucket`` ... ``all_gather_scalar``
:2596-2770, ``load_moe_state_dict`` :2771, ``load_module_state_dict`` :2826, ``save_fp16_model`` :3813,
``empty_partition_cache`` :3867.

Every accessor reads the parsed ``DeepSpeedConfig`` (runtime/config.py); defaults are the reference's constants. The
behavioural methods act on this framework's flat ZeRO store (runtime/zero/optimizer.py), not on per-parameter
partitions, so e.g. ``empty_partition_cache`` releases every gathered unit buffer and ``allreduce_gradients`` reduces
the units whose reduction ``backward(allreduce_gradients=False)`` held back.
"""
import os
from collections import deque

import torch

from .. import comm as dist
from ..utils.logging import log_dist, logger


def _sec(raw, *path, default=None):
    d = raw
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return default
        d = d[k]
    return d


class EngineApiMixin:
    """Mixed into ``DeepSpeedEngine``: needs ``self._config``, ``self.optimizer``, ``self.module``, ``self.dp_group``."""

    # ------------------------------------------------------------------------------------------------------------
    # batch size
    # ------------------------------------------------------------------------------------------------------------
    def get_batch_info(self):
        """(train_batch_size, train_micro_batch_size_per_gpu, gradient_accumulation_steps)."""
        return self.train_batch_size(), self.train_micro_batch_size_per_gpu(), self.gradient_accumulation_steps()

    def _set_batch(self, micro, gas):
        cfg = self._config
        cfg.train_micro_batch_size_per_gpu = int(micro)
        cfg.gradient_accumulation_steps = int(gas)
        cfg.train_batch_size = int(micro) * int(gas) * self.dp_world_size
        if self.optimizer is not None and hasattr(self.optimizer, "gas"):
            # the flat store keeps the gradient-accumulation dtype it was built with (fp32 when gas > 1 at init)
            self.optimizer.gas = int(gas)
        if getattr(self, "tput_timer", None) is not None:
            self.tput_timer.batch_size = cfg.train_batch_size

    def set_train_batch_size(self, train_batch_size):
        """Change the global batch by changing the gradient-accumulation steps (the micro batch stays): must divide
        by micro batch x data-parallel size."""
        micro, ws = self.train_micro_batch_size_per_gpu(), self.dp_world_size
        if train_batch_size % (micro * ws) != 0:
            raise ValueError(f"Train batch size {train_batch_size} must be divisible by micro-batch {micro} x data "
                             f"parallelism {ws}")
        self._set_batch(micro, train_batch_size // (micro * ws))

    def set_train_micro_batch_size(self, micro_batch_size):
        """Change the micro batch; the gradient-accumulation steps stay, so the global batch follows."""
        self._set_batch(int(micro_batch_size), self.gradient_accumulation_steps())

    def set_data_post_process_func(self, post_process_func):
        if self.training_dataloader is not None:
            self.training_dataloader.post_process_func = post_process_func

    # ------------------------------------------------------------------------------------------------------------
    # config accessors
    # ------------------------------------------------------------------------------------------------------------
    def checkpoint_tag_validation_enabled(self):
        return self._config.checkpoint_tag_validation_enabled

    def checkpoint_tag_validation_fail(self):
        return self._config.checkpoint_tag_validation_fail

    def elasticity_enabled(self):
        return bool(self._config.elasticity.get("enabled", False))

    def is_elastic_model_parallel_supported(self):
        if not self.elasticity_enabled():
            return False
        ec = self._config.elasticity
        return int(ec.get("model_parallel_size", 1)) > 1 and float(ec.get("version", 0.1)) >= 0.2

    def pld_enabled(self):
        return bool(self._config.pld_config.get("enabled", False))

    def pld_params(self):
        return self._config.pld_config

    def pld_theta(self):
        return self._config.pld_config.get("theta", 1.0)

    def pld_gamma(self):
        return self._config.pld_config.get("gamma", 0.001)

    def _eig(self, key, default):
        return (self._config.eigenvalue_config or {}).get(key, default)

    def eigenvalue_enabled(self):
        return bool(self._eig("enabled", False))

    def eigenvalue_verbose(self):
        return bool(self._eig("verbose", False))

    def eigenvalue_max_iter(self):
        return int(self._eig("max_iter", 100))

    def eigenvalue_tol(self):
        return float(self._eig("tol", 1e-2))

    def eigenvalue_stability(self):
        return float(self._eig("stability", 1e-6))

    def eigenvalue_gas_boundary_resolution(self):
        return int(self._eig("gas_boundary_resolution", 1))

    def eigenvalue_layer_name(self):
        return self._eig("layer_name", "bert.encoder.layer")

    def eigenvalue_layer_num(self):
        return int(self._eig("layer_num", 0))

    def curriculum_enabled_legacy(self):
        return bool(self._config.curriculum_learning.get("enabled", False))

    def curriculum_params_legacy(self):
        return self._config.curriculum_learning

    def data_efficiency_enabled(self):
        return bool(self._config.data_efficiency.get("enabled", False))

    def data_efficiency_config(self):
        return self._config.data_efficiency

    def data_sampling_enabled(self):
        return bool(_sec(self._config.data_efficiency, "data_sampling", "enabled", default=False))

    def data_sampling_config(self):
        return _sec(self._config.data_efficiency, "data_sampling", default={})

    def curriculum_learning_enabled(self):
        return bool(_sec(self._config.data_efficiency, "data_sampling", "curriculum_learning", "enabled",
                         default=False))

    def curriculum_learning_config(self):
        return _sec(self._config.data_efficiency, "data_sampling", "curriculum_learning", default={})

    def random_ltd_enabled(self):
        return bool(_sec(self._config.data_efficiency, "data_routing", "random_ltd", "enabled", default=False))

    def random_ltd_config(self):
        return _sec(self._config.data_efficiency, "data_routing", "random_ltd", default={})

    def random_ltd_initialize(self):
        """Attach the random-LTD scheduler to the ``RandomLayerTokenDrop`` layers named by ``random_ltd_layer_id``
        (reference engine.py:691): layer ids matched in module-name order; their count must equal
        ``random_ltd_layer_num``."""
        from .data_pipeline.random_ltd import RandomLayerTokenDrop, RandomLTDScheduler
        assert self.random_ltd_enabled(), "random_ltd is not enabled in data_efficiency.data_routing"
        cfg = self.random_ltd_config()
        self.random_ltd_scheduler = RandomLTDScheduler(cfg)
        queue = deque(sorted(cfg.get("random_ltd_layer_id", [])))
        count = 0
        for name, layer in self.module.named_modules():
            if isinstance(layer, RandomLayerTokenDrop) and queue and str(queue[0]) in name:
                layer.scheduler = self.random_ltd_scheduler
                queue.popleft()
                count += 1
        if int(cfg.get("random_ltd_layer_num", count)) != count:
            raise ValueError(f"random_ltd_layer_num {cfg.get('random_ltd_layer_num')} must equal the number of "
                             f"random_ltd_layer_id layers found ({count})")
        return self.random_ltd_scheduler

    def get_sequence_parallel_group(self):
        return self.seq_parallel_group

    def _fp(self, key, default):
        return (self._config.flops_profiler_config or {}).get(key, default)

    def flops_profiler_enabled(self):
        return bool(self._fp("enabled", False)) or self.autotuning_enabled()

    def flops_profiler_recompute_fwd_factor(self):
        return float(self._fp("recompute_fwd_factor", 0.0))

    def flops_profiler_profile_step(self):
        return int(self._fp("profile_step", 1))

    def flops_profiler_module_depth(self):
        return int(self._fp("module_depth", -1))

    def flops_profiler_top_modules(self):
        return int(self._fp("top_modules", 1))

    def flops_profiler_detailed(self):
        return bool(self._fp("detailed", True))

    def flops_profiler_output_file(self):
        return self._fp("output_file", None)

    def memory_breakdown(self):
        return self._config.memory_breakdown

    def autotuning_enabled(self):
        return bool(self._config.autotuning.get("enabled", False))

    def autotuning_start_profile_step(self):
        return int(self._config.autotuning.get("start_profile_step", 3))

    def autotuning_end_profile_step(self):
        return int(self._config.autotuning.get("end_profile_step", 5))

    def autotuning_metric_path(self):
        return self._config.autotuning.get("metric_path") or os.getcwd()

    def autotuning_model_info_path(self):
        return self._config.autotuning.get("model_info_path") or os.getcwd()

    def autotuning_metric(self):
        return self._config.autotuning.get("metric", "throughput")

    def autotuning_profile_model_info(self):
        return bool(self._config.autotuning.get("model_info", {}).get("profile", False)) \
            if self.autotuning_enabled() else False

    def sparse_gradients_enabled(self):
        return self._config.sparse_gradients_enabled

    def optimizer_name(self):
        return self.client_optimizer.__class__.__name__ if self.client_optimizer else self._config.optimizer_name

    def optimizer_params(self):
        return self._config.optimizer_params

    def optimizer_legacy_fusion(self):
        return self._config.optimizer_legacy_fusion

    def scheduler_name(self):
        return self._config.scheduler_name

    def scheduler_params(self):
        return self._config.scheduler_params

    def quantize_training(self):
        """(enabled, quantize_weight_in_forward, target_bits, start_bits, period, type, rounding, verbose, kernel) --
        the reference tuple, from the ``quantize_training`` section."""
        q = self._config.quantize_training or {}
        bits = q.get("quantize_bits", {})
        sch = q.get("quantize_schedule", {})
        return (bool(q.get("enabled", False)), bool(q.get("quantize_weight_in_forward", False)),
                int(bits.get("target_bits", 8)), int(bits.get("start_bits", 16)), int(sch.get("quantize_period", 1000)),
                q.get("quantize_algo", {}).get("q_type", "symmetric"),
                q.get("quantize_algo", {}).get("rounding", "nearest"), bool(q.get("quantize_verbose", False)),
                bool(q.get("use_quantizer_kernel", False)))

    # ---- ZeRO ----------------------------------------------------------------------------------------------------
    def _z(self):
        return self._config.zero_config

    def zero_allow_untested_optimizer(self):
        return self._config.zero_allow_untested_optimizer

    def zero_force_ds_cpu_optimizer(self):
        return self._config.zero_force_ds_cpu_optimizer

    def zero_reduce_scatter(self):
        return self._z().reduce_scatter

    def zero_overlap_comm(self):
        return self._z().overlap_comm

    def zero_offload_optimizer(self):
        oo = self._z().offload_optimizer
        return oo if oo.enabled else None

    def zero_offload_param(self):
        op = self._z().offload_param
        return op if op.enabled else None

    def zero_use_cpu_optimizer(self):
        return self._z().offload_optimizer.device in ("cpu", "nvme")

    def zero_cpu_offload(self):
        return self._z().offload_optimizer.device == "cpu"

    def zero_partial_offload(self):
        return self._z().offload_optimizer.ratio if self.zero_use_cpu_optimizer() else 1.0

    def zero_sub_group_size(self):
        return self._z().sub_group_size

    def mics_shard_size(self):
        return self._z().mics_shard_size

    def zero_reduce_bucket_size(self):
        return self._z().reduce_bucket_size

    def zero_multi_rank_bucket_allreduce(self):
        return self._z().use_multi_rank_bucket_allreduce

    def zero_allgather_bucket_size(self):
        return self._z().allgather_bucket_size

    def zero_optimization_partition_gradients(self):
        return self.zero_optimization_stage() >= 2

    def zero_optimization_partition_weights(self):
        return self.zero_optimization_stage() >= 3

    def is_first_weights_partition_group(self):
        if self.mics_shard_size() > 0:
            return dist.get_rank() < self.mics_shard_size()
        return self.zero_optimization_partition_weights()

    def zero_contiguous_gradients(self):
        return self._z().contiguous_gradients

    def zero_load_from_fp32_weights(self):
        return self._z().load_from_fp32_weights

    def zero_elastic_checkpoint(self):
        return self._z().elastic_checkpoint

    def zero_nvme_offload_optimizer(self):
        return self._z().offload_optimizer.device == "nvme"

    def zero_max_live_parameters(self):
        return self._z().max_live_parameters

    def zero_max_reuse_distance(self):
        return self._z().max_reuse_distance

    def zero_prefetch_bucket_size(self):
        return self._z().prefetch_bucket_size

    def zero_module_granularity_threshold(self):
        return self._z().module_granularity_threshold

    def zero_param_persistence_threshold(self):
        return self._z().param_persistence_threshold

    def zero_model_persistence_threshold(self):
        return self._z().model_persistence_threshold

    def zero_gather_16bit_weights_on_model_save(self):
        z = self._z()
        return bool(z.gather_16bit_weights_on_model_save or z.stage3_gather_fp16_weights_on_model_save)

    def zero_grad_hooks(self):
        return bool((self._config.raw.get("zero_optimization") or {}).get("grad_hooks", True))

    def zero_legacy_stage1(self):
        return self._z().legacy_stage1

    def zero_ignore_unused_parameters(self):
        return self._z().ignore_unused_parameters

    def zero_allgather_partitions(self):
        return self._z().allgather_partitions

    def zero_round_robin_gradients(self):
        return self._z().round_robin_gradients

    def zero_hpz_partition_size(self):
        return self._z().zero_hpz_partition_size

    def zero_quantized_weights(self):
        return self._z().zero_quantized_weights

    def zero_quantized_nontrainable_weights(self):
        return self._z().zero_quantized_nontrainable_weights

    def zero_quantized_gradients(self):
        return self._z().zero_quantized_gradients

    def zeropp_loco_param(self):
        return (self._config.raw.get("zero_optimization") or {}).get("zeropp_loco_param")

    def zero_log_trace_cache_warnings(self):
        return self._z().log_trace_cache_warnings

    # ---- parallelism / precision ------------------------------------------------------------------------------
    def tensor_parallel_config(self):
        return self._config.tensor_parallel

    def autotp_size(self):
        return int(self._config.tensor_parallel.get("autotp_size", 0) or 0)

    def graph_harvesting(self):
        return bool(self._config.raw.get("graph_harvesting", False))

    def fp16_master_weights_and_gradients(self):
        return bool((self._config.raw.get("fp16") or {}).get("fp16_master_weights_and_grads", False))

    def amp_enabled(self):
        return self._config.amp_enabled

    def amp_params(self):
        return {k: v for k, v in (self._config.raw.get("amp") or {}).items() if k != "enabled"}

    def fp16_auto_cast(self):
        return self._config.loss_scale_config.auto_cast

    def loss_scale(self):
        return self._config.loss_scale_config.loss_scale

    def use_node_local_storage(self):
        return self._config.use_node_local_storage

    def load_universal_checkpoint(self):
        return self._config.load_universal_checkpoint

    @property
    def communication_data_type(self):
        """Gradient-collective dtype: the configured one, else the compute dtype's (fp16 / bf16), else fp32."""
        override = getattr(self, "_comm_dtype_override", None)
        if override is not None:
            return override
        name = self._config.communication_data_type
        if name is not None:
            return {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16,
                    "bfp16": torch.bfloat16}.get(str(name).lower(), torch.float32)
        if self.fp16_enabled():
            return torch.float16
        if self.bfloat16_enabled():
            return torch.bfloat16
        return torch.float32

    @communication_data_type.setter
    def communication_data_type(self, value):
        self._comm_dtype_override = value

    def postscale_gradients(self):
        return not self._config.prescale_gradients

    def gradient_predivide_factor(self):
        return self._config.gradient_predivide_factor

    def dump_state(self):
        return self._config.dump_state

    def dynamic_loss_scale(self):
        return self._config.loss_scale_config.loss_scale == 0

    def initial_dynamic_scale(self):
        return 2.0**self._config.loss_scale_config.initial_scale_power

    def dynamic_loss_scale_args(self):
        ls = self._config.loss_scale_config
        if not self.fp16_enabled() or ls.loss_scale != 0:
            return None
        return {"init_scale": 2.0**ls.initial_scale_power, "scale_window": ls.loss_scale_window,
                "delayed_shift": ls.hysteresis, "consecutive_hysteresis": ls.consecutive_hysteresis,
                "min_scale": ls.min_loss_scale}

    def swap_tensor_config(self):
        z = self._z()
        return {"offload_optimizer": z.offload_optimizer, "offload_param": z.offload_param}

    def aio_config(self):
        return self._config.aio_config

    def get_data_types(self):
        """(model dtype, gradient-accumulation dtype) -- reference engine.py get_data_types."""
        model = self.compute_dtype
        ga = self._config.grad_accum_dtype
        grad = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}.get(ga, None) if ga else None
        if grad is None:
            grad = torch.float32 if model == torch.bfloat16 and self.zero_optimization_stage() == 0 else model
        return model, grad

    @staticmethod
    def is_map_style_dataset(obj):
        return hasattr(obj, "__getitem__") and hasattr(obj, "__len__")

    @staticmethod
    def is_iterable_style_dataset(obj):
        return isinstance(obj, torch.utils.data.IterableDataset)

    def dataloader_drop_last(self):
        return bool(self._config.raw.get("dataloader_drop_last", False))

    # ------------------------------------------------------------------------------------------------------------
    # step state
    # ------------------------------------------------------------------------------------------------------------
    def was_step_applied(self) -> bool:
        """False when the last optimizer step was skipped (fp16 overflow, symmetric-memory failure flag)."""
        return bool(getattr(self, "_step_applied", True))

    def print_forward_breakdown(self, fwd_time):
        """Log the forward's breakdown (reference: MoE gate / all-to-all timers; here every engine timer that ran)."""
        names = list(getattr(self.timers, "timers", {}) or {})
        if names:
            self.timers.log(names, reset=False)
        log_dist(f"forward time {fwd_time:.2f} ms", ranks=[0])

    def _get_optimizer_param(self, name):
        if self.optimizer is None:
            return []
        return [g[name] for g in self.optimizer.param_groups if name in g]

    def get_type(self):
        return self._get_optimizer_param("type")

    def get_mom(self):
        if str(self.optimizer_name() or "").lower() in ("sgd", "rmsprop"):
            return self._get_optimizer_param("momentum")
        return self._get_optimizer_param("betas")

    # ------------------------------------------------------------------------------------------------------------
    # gradient reduction
    # ------------------------------------------------------------------------------------------------------------
    def allreduce_gradients(self, bucket_size=None):
        """Reduce the gradients ``backward(allreduce_gradients=False)`` held back (ZeRO-0/1/2: the flat unit
        reductions queue in the optimizer until this call; ZeRO-3 reduces in its backward hooks, as the reference's
        stage-3 optimizer does, so nothing is held there)."""
        z = self.optimizer
        if z is not None and hasattr(z, "release_held_reductions"):
            z.release_held_reductions()
            z.hold_reduction = bool(getattr(self, "_pipe_hold", False))

    def clip_fp32_gradients(self):
        """Clip the gradients to ``gradient_clipping`` now. ZeRO clips inside ``step()`` from the flat store's norm;
        for module gradients outside the store (a client optimizer) torch's clip applies."""
        mx = self.gradient_clipping()
        if mx <= 0:
            return None
        params = [p for p in self.module.parameters() if p.grad is not None]
        if params:
            return torch.nn.utils.clip_grad_norm_(params, mx)
        return None

    def _dp_average(self, t, dp_group):
        if dist.get_world_size(dp_group) == 1:
            return t
        pre = self.gradient_predivide_factor()
        if self.postscale_gradients():
            if pre != 1.0:
                t.mul_(1.0 / pre)
            dist.all_reduce(t, group=dp_group)
            if pre != dist.get_world_size(dp_group):
                t.mul_(pre / dist.get_world_size(dp_group))
        else:
            t.div_(dist.get_world_size(dp_group))
            dist.all_reduce(t, group=dp_group)
        return t

    def allreduce_bucket(self, bucket, dp_group, dp_world_size=None):
        """Flatten ``bucket`` (list of tensors), all-reduce-average it over ``dp_group`` in the communication dtype,
        return the flat result."""
        flat = torch.cat([t.reshape(-1) for t in bucket])
        cdt = self.communication_data_type
        work = flat.to(cdt) if flat.dtype != cdt else flat
        self._dp_average(work, dp_group)
        return work.to(flat.dtype) if work is not flat else work

    def allreduce_and_copy(self, small_bucket, dp_group, dp_world_size=None):
        flat = self.allreduce_bucket(small_bucket, dp_group, dp_world_size)
        off = 0
        for t in small_bucket:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n

    def allreduce_no_retain(self, bucket, dp_group, numel_per_bucket=500000000, dp_world_size=None):
        small, n = [], 0
        for t in bucket:
            small.append(t)
            n += t.numel()
            if n > numel_per_bucket:
                self.allreduce_and_copy(small, dp_group, dp_world_size)
                small, n = [], 0
        if small:
            self.allreduce_and_copy(small, dp_group, dp_world_size)

    def buffered_allreduce_fallback(self, grads=None, elements_per_buffer=500000000):
        """All-reduce-average the module gradients (or ``grads``) over the data-parallel group, bucketed by dtype;
        sparse (row-sparse embedding) gradients go through ``sparse_allreduce_no_retain``."""
        if grads is None:
            grads = [p.grad for p in self.module.parameters() if p.grad is not None]
        dense, sparse = {}, []
        for g in grads:
            if g.is_sparse:
                sparse.append(g)
            else:
                dense.setdefault(g.dtype, []).append(g.data)
        for bucket in dense.values():
            self.allreduce_no_retain(bucket, self.dp_group, numel_per_bucket=elements_per_buffer)
        if sparse:
            self.sparse_allreduce_no_retain(sparse, self.dp_group)

    def sparse_allreduce_no_retain(self, bucket, dp_group, dp_world_size=None):
        out = self.sparse_allreduce_bucket(bucket, dp_group, dp_world_size)
        for t, r in zip(bucket, out):
            if t.is_sparse:
                t.copy_(r.to_coo_tensor())
            else:
                t.copy_(r.to_dense())

    def sparse_allreduce_bucket(self, bucket, dp_group, dp_world_size=None):
        from .sparse_tensor import SparseTensor
        return [self.sparse_allreduce(SparseTensor(t), dp_group, dp_world_size) for t in bucket]

    def sparse_allreduce(self, sparse, dp_group, dp_world_size=None):
        """Average a row-sparse gradient over ``dp_group``: all-gather every rank's (indices, values) and sum the rows
        (duplicates add), divided by the group size."""
        W = dp_world_size or dist.get_world_size(dp_group)
        values = sparse.values.float() / W
        idx, vals = self.sparse_all_gather(sparse.indices, dp_group), self.sparse_all_gather(values, dp_group)
        sparse.indices = torch.cat(idx)
        sparse.values = torch.cat(vals).to(sparse.values.dtype)
        return sparse

    def sparse_all_gather(self, value, dp_group):
        """All-gather tensors whose first dimension differs per rank (padded to the max, trimmed after)."""
        W = dist.get_world_size(dp_group)
        sizes = self.all_gather_scalar(value.size(0), dp_group)
        mx = int(max(sizes))
        pad = value.new_zeros((mx,) + tuple(value.shape[1:]))
        pad[:value.size(0)] = value
        outs = [torch.empty_like(pad) for _ in range(W)]
        dist.all_gather(outs, pad, group=dp_group)
        return [o[:int(n)] for o, n in zip(outs, sizes)]

    def all_gather_scalar(self, value, dp_group):
        W = dist.get_world_size(dp_group)
        dev = self.device if dist.get_backend(dp_group) == "nccl" else torch.device("cpu")
        t = torch.tensor([value], dtype=torch.int64, device=dev)
        outs = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(outs, t, group=dp_group)
        return [int(o.item()) for o in outs]

    # ------------------------------------------------------------------------------------------------------------
    # state dicts / checkpoints
    # ------------------------------------------------------------------------------------------------------------
    def load_module_state_dict(self, checkpoint, strict=True, custom_load_fn=None, fetch_z3_params=False):
        """Load ``checkpoint["module"]`` (or a bare state dict) into the model. Under partitioned ZeRO-3 the values go
        straight into the flat shards (each rank keeps its slice; fp32 master and compute copy both refreshed)."""
        sd = checkpoint["module"] if isinstance(checkpoint, dict) and "module" in checkpoint else checkpoint
        if custom_load_fn is not None:
            custom_load_fn(src=sd, dst=self.module)
            return
        z = self.optimizer
        managed = getattr(z, "param_to_unit", None) if z is not None else None
        if managed:
            # parameters in the flat store: write the fp32 master (each rank its fragment) and the compute copy, so
            # no precision is lost through the bf16 parameter (collective under ZeRO-3 partitioning)
            from ..utils.tensor_fragment import safe_set_full_fp32_param
            names = dict(self.module.named_parameters())
            missing = [n for n in names if n not in sd]
            if strict and missing:
                raise RuntimeError(f"load_module_state_dict: missing keys {missing[:8]}")
            for n, p in names.items():
                if n in sd and id(p) in managed:
                    safe_set_full_fp32_param(p, sd[n].to(torch.float32))
            rest = {k: v for k, v in sd.items() if k not in names or id(names[k]) not in managed}
            if rest:
                self.module.load_state_dict(rest, strict=False)
            return
        self.module.load_state_dict(sd, strict=strict)

    @staticmethod
    def load_moe_state_dict(checkpoint_path, tag, state_dict, old_moe_load=False, model=None, mpu=None,
                            num_experts=1, checkpoint_engine=None):
        """Merge the expert files of an expert-parallel checkpoint into ``state_dict`` (this rank's experts: global
        expert ids ep_rank * local + i, read from ``expert_<id>_mp_rank_XX_model_states.pt`` when present, else from
        the per-EP-rank module files this framework writes)."""
        import glob

        from .checkpointing import _expert_name
        files = sorted(glob.glob(os.path.join(checkpoint_path, str(tag), "expert_*_mp_rank_*_model_states.pt")))
        if files:
            for f in files:
                sd = torch.load(f, map_location="cpu", weights_only=True)
                state_dict.update(sd.get("module", sd))
            return state_dict
        ep = 0
        while True:
            path = _expert_name(checkpoint_path, str(tag), ep)
            if not os.path.exists(path):
                break
            sd = torch.load(path, map_location="cpu", weights_only=True)
            state_dict.update(sd.get("module", sd))
            ep += 1
        return state_dict

    def save_fp16_model(self, save_dir, save_filename="pytorch_model.bin"):
        return self.save_16bit_model(save_dir, save_filename)

    def empty_partition_cache(self):
        """Release every gathered ZeRO-3 unit buffer (the next forward gathers again) and return the cached blocks to
        the device -- e.g. between training and generation."""
        z = self.optimizer
        if z is not None and self.zero_optimization_stage() == 3 and hasattr(z, "release_all"):
            z.release_all()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    # ------------------------------------------------------------------------------------------------------------
    # teardown
    # ------------------------------------------------------------------------------------------------------------
    def destroy(self):
        """Release what the engine holds outside Python's reference counting: ZeRO-3 module hooks and gathered
        units, the startup transports (communicators, symmetric buffers), offloaded-state pinned buffers, the host
        activation cache's hooks and pinned pool. Collective when transports were set up."""
        z = self.optimizer
        if z is not None:
            if hasattr(z, "release_transports"):
                try:
                    z.release_transports()
                except Exception as e:  # noqa: BLE001
                    logger.warning(f"destroy: transport release failed: {e}")
            for h in getattr(z, "_hook_handles", []) or []:
                try:
                    h.remove()
                except Exception:  # noqa: BLE001
                    pass
            if hasattr(z, "_hook_handles"):
                z._hook_handles = []
            so = getattr(z, "state_offload", None)
            if so is not None:
                if hasattr(so, "join"):
                    so.join()  # an async host step still writing parameters
                z.state_offload = None
            if self.zero_optimization_stage() == 3 and hasattr(z, "release_all"):
                try:
                    z.release_all()
                except Exception:  # noqa: BLE001
                    pass
        ac = getattr(self, "_activation_cache", None)
        if ac is not None:
            if hasattr(ac, "detach"):
                ac.detach()
            self._activation_cache = None
        self._destroyed = True
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
