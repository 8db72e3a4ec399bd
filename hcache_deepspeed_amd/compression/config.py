"""``compression_training`` config section (same JSON schema as the reference).

Reference parity: compression/constants.py (key names and defaults) and compression/config.py
(``get_compression_config``: per-technique ``shared_parameters`` + ``different_groups`` with ``params``,
``modules``, ``related_modules``; ``layer_reduction``).
"""
import copy

COMPRESSION_TRAINING = "compression_training"
SHARED_PARAMETERS = "shared_parameters"
DIFFERENT_GROUPS = "different_groups"
PARAMS = "params"
MODULES = "modules"
RELATED_MODULES = "related_modules"

LAYER_REDUCTION = "layer_reduction"
WEIGHT_QUANTIZATION = "weight_quantization"
ACTIVATION_QUANTIZATION = "activation_quantization"
SPARSE_PRUNING = "sparse_pruning"
ROW_PRUNING = "row_pruning"
HEAD_PRUNING = "head_pruning"
CHANNEL_PRUNING = "channel_pruning"

TECHNIQUES = (WEIGHT_QUANTIZATION, ACTIVATION_QUANTIZATION, SPARSE_PRUNING, ROW_PRUNING, HEAD_PRUNING,
              CHANNEL_PRUNING)

_SHARED_DEFAULTS = {
    WEIGHT_QUANTIZATION: {
        "enabled": False, "quantizer_kernel": False, "schedule_offset": 0, "quantize_groups": 1,
        "quantize_verbose": False, "quantization_type": "symmetric", "quantize_weight_in_forward": False,
        "rounding": "nearest", "fp16_mixed_quantize": {"enabled": False, "quantize_change_ratio": 0.001},
    },
    ACTIVATION_QUANTIZATION: {
        "enabled": False, "quantization_type": "symmetric", "range_calibration": "dynamic", "schedule_offset": 1000,
    },
    SPARSE_PRUNING: {
        "enabled": False, "method": "l1", "block_pattern": "4x1", "schedule_offset_stride": 1,
        "schedule_offset": 1000, "schedule_offset_end": None, "excluded_modules": [],
    },
    ROW_PRUNING: {"enabled": False, "method": "l1", "schedule_offset": 1000},
    HEAD_PRUNING: {"enabled": False, "method": "topk", "schedule_offset": 1000, "num_heads": None},
    CHANNEL_PRUNING: {"enabled": False, "method": "l1", "schedule_offset": 1000},
}

_PARAM_DEFAULTS = {
    WEIGHT_QUANTIZATION: {"start_bits": 8, "target_bits": 8, "quantization_period": 1},
    ACTIVATION_QUANTIZATION: {"bits": 8},
    SPARSE_PRUNING: {"dense_ratio": 0.1},
    ROW_PRUNING: {"dense_ratio": 1.0},
    HEAD_PRUNING: {"dense_ratio": 1.0},
    CHANNEL_PRUNING: {"dense_ratio": 1.0},
}

_LAYER_REDUCTION_DEFAULTS = {"enabled": False, "keep_number_layer": None, "module_name_prefix": "",
                             "teacher_layer": [], "other_module_name": []}


def get_compression_config(ds_config):
    """Normalise ``ds_config['compression_training']`` (missing keys -> reference defaults)."""
    section = copy.deepcopy((ds_config or {}).get(COMPRESSION_TRAINING, {}))
    out = {LAYER_REDUCTION: {**_LAYER_REDUCTION_DEFAULTS, **section.get(LAYER_REDUCTION, {})}}
    for tech in TECHNIQUES:
        sub = section.get(tech, {})
        shared = copy.deepcopy(_SHARED_DEFAULTS[tech])
        for k, v in sub.get(SHARED_PARAMETERS, {}).items():
            if isinstance(v, dict) and isinstance(shared.get(k), dict):
                shared[k].update(v)
            else:
                shared[k] = v
        if tech == SPARSE_PRUNING and shared["schedule_offset_end"] is None:
            shared["schedule_offset_end"] = shared["schedule_offset"]
        groups = {}
        for name, g in sub.get(DIFFERENT_GROUPS, {}).items():
            groups[name] = {
                PARAMS: {**_PARAM_DEFAULTS[tech], **g.get(PARAMS, {})},
                MODULES: list(g.get(MODULES, ["*"])),
                RELATED_MODULES: g.get(RELATED_MODULES),
            }
        if shared["enabled"]:
            assert groups, f"compression technique {tech} is enabled but has no different_groups"
        out[tech] = {SHARED_PARAMETERS: shared, DIFFERENT_GROUPS: groups}
    return out
