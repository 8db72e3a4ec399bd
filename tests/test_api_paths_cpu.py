"""Every public import path a DeepSpeed user script uses resolves here, the way the
script writes it with ``import hcache_deepspeed_amd as deepspeed`` (reference deepspeed/__init__.py:25-50,
accelerator/real_accelerator.py:51, pipe/__init__.py, moe/layer.py:17, sequence/layer.py:311,
inference/v2/engine_factory.py:69, ops/adam/__init__.py, utils/zero_to_fp32.py)."""
import importlib

import pytest
import torch

PKG = "hcache_deepspeed_amd"

PATHS = [
    ("", ["initialize", "init_inference", "tp_model_init", "add_config_arguments", "init_distributed", "zero",
          "DeepSpeedEngine", "PipelineEngine", "DeepSpeedHybridEngine", "InferenceEngine", "DeepSpeedConfig",
          "DeepSpeedConfigError", "DeepSpeedInferenceConfig", "PipelineModule", "OnDevice", "get_accelerator",
          "add_tuning_arguments", "is_compile_supported", "checkpointing", "DeepSpeedTransformerLayer",
          "DeepSpeedTransformerConfig", "replace_transformer_layer", "revert_transformer_layer", "log_dist",
          "logger", "ops", "comm", "version", "__version__", "default_inference_config"]),
    ("accelerator", ["get_accelerator", "set_accelerator"]),
    ("comm", ["init_distributed", "all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "barrier",
              "get_rank", "get_world_size", "all_to_all_single"]),
    ("runtime.zero", ["Init", "GatheredParameters", "register_external_parameter"]),
    ("pipe", ["PipelineModule", "LayerSpec", "TiedLayerSpec"]),
    ("moe.layer", ["MoE"]),
    ("moe.utils", ["split_params_into_different_moe_groups_for_optimizer", "is_moe_param"]),
    ("sequence.layer", ["DistributedAttention"]),
    ("sequence.cross_entropy", ["vocab_sequence_parallel_cross_entropy"]),
    ("sequence.fpdt_layer", ["FPDT_Attention", "FPDT_FFN", "FPDT_LogitsLoss", "FPDTInputConstruct"]),
    ("ops.adam", ["FusedAdam", "DeepSpeedCPUAdam"]),
    ("ops.lamb", ["FusedLamb"]),
    ("ops.lion", ["FusedLion", "DeepSpeedCPULion"]),
    ("ops.adagrad", ["DeepSpeedCPUAdagrad"]),
    ("ops.fp_quantizer", ["FP_Quantize"]),
    ("ops.sparse_attention", ["SparseSelfAttention", "SparsityConfig", "FixedSparsityConfig"]),
    ("ops.transformer", ["DeepSpeedTransformerLayer", "DeepSpeedTransformerConfig"]),
    ("ops.op_builder", ["AsyncIOBuilder", "CPUAdamBuilder", "FusedAdamBuilder"]),
    ("ops.deepspeed4science", ["DS4Sci_EvoformerAttention"]),
    ("checkpoint", ["ds_to_universal", "get_fp32_state_dict_from_zero_checkpoint", "SubparamShape"]),
    ("checkpoint.ds_to_universal", ["main", "parse_arguments"]),
    ("utils", ["safe_get_full_fp32_param", "safe_get_full_grad", "safe_get_full_optimizer_state",
               "safe_set_full_fp32_param", "OnDevice", "logger", "log_dist", "instrument_w_nvtx",
               "set_z3_leaf_modules"]),
    ("utils.zero_to_fp32", ["get_fp32_state_dict_from_zero_checkpoint",
                            "convert_zero_checkpoint_to_fp32_state_dict", "load_state_dict_from_zero_checkpoint"]),
    ("utils.groups", ["_get_data_parallel_group", "_get_expert_parallel_group"]),
    ("inference.v2.engine_factory", ["build_hf_engine", "build_engine_from_ds_checkpoint"]),
    ("inference.v2", ["InferenceEngineV2", "RaggedInferenceEngineConfig"]),
    ("module_inject", ["replace_transformer_layer", "revert_transformer_layer", "set_autotp_mode", "AutoTP"]),
    ("runtime.lr_schedules", ["WarmupLR", "WarmupDecayLR", "WarmupCosineLR", "OneCycle", "LRRangeTest"]),
    ("runtime.compiler", ["is_compile_supported"]),
    ("runtime.activation_checkpointing.checkpointing", ["checkpoint", "configure"]),
    ("profiling.flops_profiler", ["FlopsProfiler", "get_model_profile"]),
    ("monitor.monitor", ["MonitorMaster"]),
    ("linear", ["OptimizedLinear", "LoRAConfig", "QuantizationConfig"]),
    ("compression.compress", ["init_compression", "redundancy_clean"]),
    ("elasticity", ["compute_elastic_config"]),
]


@pytest.mark.parametrize("mod,names", PATHS, ids=[p[0] or "deepspeed" for p in PATHS])
def test_import_path(mod, names):
    m = importlib.import_module(PKG + ("." + mod if mod else ""))
    missing = [n for n in names if not hasattr(m, n)]
    assert not missing, f"{mod}: missing {missing}"


def test_accelerator_contract():
    import hcache_deepspeed_amd as deepspeed
    acc = deepspeed.get_accelerator()
    assert acc is deepspeed.get_accelerator()
    assert acc.communication_backend_name() == ("nccl" if torch.cuda.is_available() else "gloo")
    assert acc.is_bf16_supported()
    assert acc.device_name() in ("cuda", "cpu")
    ev = acc.Event(enable_timing=True) if acc.is_available() else acc.Event()
    ev.record()
    s = acc.Stream() if acc.is_available() else acc.Stream()
    with acc.stream(s):
        pass
    assert acc.memory_allocated() >= 0
    assert acc.total_memory() > 0
    t = acc.FloatTensor([1.0, 2.0])
    assert t.dtype == torch.float32
    assert acc.on_accelerator(t)
    assert acc.create_op_builder("AsyncIOBuilder").is_compatible()


def test_user_script_style():
    """A typical reference user script runs unchanged with the import swapped."""
    import argparse

    import hcache_deepspeed_amd as deepspeed
    from hcache_deepspeed_amd.ops.adam import FusedAdam  # noqa: F401
    from hcache_deepspeed_amd.pipe import PipelineModule, LayerSpec  # noqa: F401
    parser = deepspeed.add_config_arguments(argparse.ArgumentParser())
    parser = deepspeed.add_tuning_arguments(parser)
    args = parser.parse_args(["--deepspeed", "--lr_schedule", "WarmupLR"])
    assert args.deepspeed and args.lr_schedule == "WarmupLR"
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
    eng, opt, _, _ = deepspeed.initialize(args=args, model=model, model_parameters=model.parameters(),
                                          config={"train_micro_batch_size_per_gpu": 4,
                                                  "optimizer": {"type": "Adam", "params": {"lr": 1e-3}}})
    x = torch.randn(4, 8)
    loss = eng(x).pow(2).mean()
    eng.backward(loss)
    eng.step()
    assert eng.global_steps == 1
