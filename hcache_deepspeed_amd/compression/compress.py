"""``init_compression`` / ``redundancy_clean`` / layer-reduction student init and the compression scheduler.

Reference parity: compression/compress.py (``init_compression`` :100, ``redundancy_clean`` :148,
``student_initialization`` :192, ``get_module_name`` / ``get_compress_methods`` :30-97),
compression/helper.py (``module_replacement``, ``compression_preparation``, ``fix_compression``,
``recursive_getattr``/``setattr``, ``is_module_compressible``) and compression/scheduler.py
(``compression_scheduler`` :12 -- switches techniques on at their ``schedule_offset``).

``snip_momentum`` sparse pruning needs Intel neural_compressor in the reference; it is not importable here
and raises a clear error (the l1 / topk methods cover the native path).
"""
import json
import os
import re

import torch.nn as nn

from ..utils.logging import logger
from . import config as C
from .layers import (BNLayer_Compress, ColumnParallelLinear_Compress, Conv2dLayer_Compress, Embedding_Compress,
                     LinearLayer_Compress, RowParallelLinear_Compress)


def recursive_getattr(model, module_name):
    out = model
    for name in module_name.split("."):
        out = getattr(out, name)
    return out


def recursive_setattr(model, module_name, module):
    parts = module_name.split(".")
    parent = recursive_getattr(model, ".".join(parts[:-1])) if len(parts) > 1 else model
    setattr(parent, parts[-1], module)


def _load_config(cfg):
    if isinstance(cfg, dict):
        return cfg
    if hasattr(cfg, "raw"):
        return cfg.raw
    if isinstance(cfg, str) and os.path.exists(cfg):
        with open(cfg) as f:
            return json.load(f)
    raise ValueError(f"expected a deepspeed config dict or path, got {cfg!r}")


def _tp_classes():
    from ..parallel.tp import LinearAllreduce, LinearLayer
    return LinearLayer, LinearAllreduce


def is_module_compressible(module, mpu=None):
    col, row = _tp_classes()
    return isinstance(module, (nn.Linear, nn.Conv2d, nn.Embedding, nn.BatchNorm2d, col, row,
                               ColumnParallelLinear_Compress, RowParallelLinear_Compress))


def _convert(old):
    """Compression-aware replacement of a compressible module (weights shared, not copied)."""
    col, row = _tp_classes()
    if isinstance(old, (LinearLayer_Compress, Conv2dLayer_Compress, Embedding_Compress, BNLayer_Compress,
                        ColumnParallelLinear_Compress, RowParallelLinear_Compress)):
        return old
    if isinstance(old, nn.Linear):
        new = LinearLayer_Compress(old.in_features, old.out_features, bias=old.bias is not None, device="meta")
    elif isinstance(old, nn.Conv2d):
        new = Conv2dLayer_Compress(old.in_channels, old.out_channels, old.kernel_size, old.stride, old.padding,
                                   old.dilation, old.groups, old.bias is not None, old.padding_mode, device="meta")
    elif isinstance(old, nn.Embedding):
        new = Embedding_Compress(old.num_embeddings, old.embedding_dim, old.padding_idx, old.max_norm,
                                 old.norm_type, old.scale_grad_by_freq, old.sparse, device="meta")
    elif isinstance(old, nn.BatchNorm2d):
        new = BNLayer_Compress(old.num_features, old.eps, old.momentum, old.affine, old.track_running_stats,
                               device="meta")
        new.running_mean, new.running_var = old.running_mean, old.running_var
        new.num_batches_tracked = old.num_batches_tracked
    elif isinstance(old, col):
        return ColumnParallelLinear_Compress(old)
    elif isinstance(old, row):
        return RowParallelLinear_Compress(old)
    else:
        return None
    new.weight = old.weight
    if getattr(old, "bias", None) is not None:
        new.bias = old.bias
    if hasattr(new, "_init_compression"):
        new._init_compression()
    new.train(old.training)
    return new


def module_replacement(model, module_name, compression_technique=None, mpu=None):
    old = recursive_getattr(model, module_name)
    new = _convert(old)
    if new is None:
        return
    for k, v in (compression_technique or {}).items():
        if not v.get("enabled", False):
            continue
        if k == C.SPARSE_PRUNING:
            new.enable_sparse_pruning(v["dense_ratio"], v["method"])
        elif k == C.ROW_PRUNING:
            new.enable_row_pruning(v["dense_ratio"], v["method"])
        elif k == C.HEAD_PRUNING:
            new.enable_head_pruning(v["dense_ratio"], v["method"], v["num_heads"])
        elif k == C.ACTIVATION_QUANTIZATION:
            new.enable_activation_quantization(v["bits"], v["quantization_type"], v["range_calibration"])
        elif k == C.WEIGHT_QUANTIZATION:
            new.enable_weight_quantization(v["start_bits"], v["target_bits"], v["quantization_period"],
                                           v["quantize_weight_in_forward"], v["quantization_type"],
                                           v["quantize_groups"])
        elif k == C.CHANNEL_PRUNING:
            new.enable_channel_pruning(v["dense_ratio"], v["method"])
        else:
            raise NotImplementedError(f"compression technique {k}")
    recursive_setattr(model, module_name, new)


def get_module_name(group_name, model, key_word, exist_module_name, mpu=None, verbose=True):
    """Names of compressible modules matching ``key_word`` (regex search; ``"*"`` = every module)."""
    found = []
    for name, module in model.named_modules():
        if not name or not is_module_compressible(module, mpu):
            continue
        if key_word != "*" and re.search(key_word, name) is None:
            continue
        if name in exist_module_name:
            if verbose:
                raise ValueError(f"{name} is already added to compression, check the config of {group_name}")
            continue
        exist_module_name.add(name)
        found.append(name)
    return found, exist_module_name


def get_compress_methods(model, compress_methods, mpu=None):
    items = []
    for method, content in compress_methods.items():
        if method == C.LAYER_REDUCTION:
            continue
        seen = set()
        shared = content[C.SHARED_PARAMETERS]
        for group_name, g in content[C.DIFFERENT_GROUPS].items():
            names, related = [], []
            if g[C.RELATED_MODULES]:
                for kw, rkws in zip(g[C.MODULES], g[C.RELATED_MODULES]):
                    n, seen = get_module_name(group_name, model, kw, seen, mpu=mpu)
                    names.append(n)
                    related.append([get_module_name(group_name, model, rk, set(), mpu=mpu)[0] for rk in rkws])
            else:
                for kw in g[C.MODULES]:
                    n, seen = get_module_name(group_name, model, kw, seen, mpu=mpu)
                    names.append(n)
            if any(names):
                items.append([names, related, {method: {**g[C.PARAMS], **shared}}])
    return items


def compression_preparation(model, compression_technique_list, mpu):
    for name, module in list(model.named_modules()):
        if name and is_module_compressible(module, mpu):
            module_replacement(model, name, mpu=mpu)
    for names_lists, _, technique in compression_technique_list:
        for names in names_lists:
            for name in names:
                module_replacement(model, name, technique, mpu=mpu)
    return model


def fix_compression(model, module_name, compression_technique, mask=None, dim_reduction=False):
    module = recursive_getattr(model, module_name)
    for k, v in compression_technique.items():
        if k == C.WEIGHT_QUANTIZATION and v.get("enabled") and module.weight_quantization_enabled_in_forward:
            return module.fix_weight_quantization()
        if k == C.SPARSE_PRUNING and v.get("enabled"):
            return module.fix_sparse_pruning_helper()
        if k == C.ROW_PRUNING and (v.get("enabled") or mask is not None):
            return module.fix_row_col_pruning_helper(mask, dim_reduction=dim_reduction)
        if k == C.HEAD_PRUNING and (v.get("enabled") or mask is not None):
            return module.fix_head_pruning_helper(mask, v["num_heads"], dim_reduction=dim_reduction)
        if k == C.CHANNEL_PRUNING and (v.get("enabled") or mask is not None):
            return module.fix_channel_pruning_helper(mask, dim_reduction=dim_reduction)
    return None


def init_compression(model, deepspeed_config, teacher_model=None, mpu=None):
    """Replace compressible modules with compression-aware ones per ``compression_training`` (reference :100)."""
    methods = C.get_compression_config(_load_config(deepspeed_config))
    c_model = model.module if hasattr(model, "module") else model
    if methods[C.LAYER_REDUCTION]["enabled"]:
        assert teacher_model is not None, "teacher model is required for layer reduction"
        student_initialization(c_model, teacher_model, deepspeed_config)
    sp = methods[C.SPARSE_PRUNING][C.SHARED_PARAMETERS]
    if sp["enabled"] and sp["method"] == "snip_momentum":
        raise NotImplementedError("snip_momentum sparse pruning requires Intel neural_compressor (not available); "
                                  "use method 'l1' or 'topk'")
    compression_preparation(c_model, get_compress_methods(c_model, methods, mpu=mpu), mpu)
    return model


def redundancy_clean(model, deepspeed_config, mpu=None):
    """Make compression permanent; row/head/channel pruning with related modules shrinks the dims (reference :148)."""
    methods = C.get_compression_config(_load_config(deepspeed_config))
    c_model = model.module if hasattr(model, "module") else model
    order = [C.WEIGHT_QUANTIZATION, C.SPARSE_PRUNING, C.ROW_PRUNING, C.HEAD_PRUNING, C.CHANNEL_PRUNING,
             C.ACTIVATION_QUANTIZATION]
    items = sorted(get_compress_methods(c_model, methods, mpu=mpu), key=lambda x: order.index(list(x[2])[0]))
    for names_lists, related_lists, technique in items:
        need_mask = bool(related_lists)
        for i, names in enumerate(names_lists):
            masks = []
            for name in names:
                m = fix_compression(c_model, name, technique, dim_reduction=need_mask)
                if need_mask:
                    masks.append(m)
            if need_mask:
                for rnames in related_lists[i]:
                    for j, name in enumerate(rnames):
                        fix_compression(c_model, name, technique, mask=masks[j], dim_reduction=True)
    return model


def student_initialization(student_model, teacher_model, deepspeed_config):
    """Layer reduction: copy the chosen teacher layers (and other modules) into the shallower student."""
    cfg = C.get_compression_config(_load_config(deepspeed_config))[C.LAYER_REDUCTION]
    prefix, teacher_layer, other = cfg["module_name_prefix"], cfg["teacher_layer"], cfg["other_module_name"]
    for s_idx, t_idx in enumerate(teacher_layer):
        s_mod = recursive_getattr(student_model, f"{prefix}.{s_idx}")
        t_mod = recursive_getattr(teacher_model, f"{prefix}.{t_idx}")
        for sp, tp in zip(s_mod.parameters(), t_mod.parameters()):
            sp.data.copy_(tp.data)
    for name in other:
        s_mod, t_mod = recursive_getattr(student_model, name), recursive_getattr(teacher_model, name)
        for sp, tp in zip(s_mod.parameters(), t_mod.parameters()):
            sp.data.copy_(tp.data)


class compression_scheduler:
    """Turns each technique on for its modules once ``training_steps`` reaches the technique's schedule offset
    (sparse pruning: inside [schedule_offset, schedule_offset_end])."""

    _FLAGS = {
        C.WEIGHT_QUANTIZATION: "weight_quantization_enabled",
        C.ACTIVATION_QUANTIZATION: "activation_quantization_enabled",
        C.SPARSE_PRUNING: "sparse_pruning_enabled",
        C.HEAD_PRUNING: "head_pruning_enabled",
        C.ROW_PRUNING: "row_pruning_enabled",
        C.CHANNEL_PRUNING: "channel_pruning_enabled",
    }

    def __init__(self, model, compression_config):
        self.model = model
        self.compression_config = compression_config
        self.training_steps = 0
        self.weight_quantization_enabled = False
        self.verbose = {k: False for k in self._FLAGS}
        self.methods = {}
        for method, content in compression_config.items():
            if method == C.LAYER_REDUCTION:
                continue
            seen, groups = set(), []
            for gname, g in content[C.DIFFERENT_GROUPS].items():
                names = []
                for kw in g[C.MODULES]:
                    n, seen = get_module_name(gname, model, kw, seen, verbose=False)
                    names.extend(n)
                if names:
                    groups.append([gname, names, dict(g[C.PARAMS])])
            self.methods[method] = {"enabled": content[C.SHARED_PARAMETERS]["enabled"],
                                    "shared": content[C.SHARED_PARAMETERS], "groups": groups}

    def _check(self, method):
        m = self.methods.get(method)
        if not m or not m["enabled"]:
            return
        sh = m["shared"]
        active = self.training_steps >= sh["schedule_offset"]
        if method == C.SPARSE_PRUNING:
            active = sh["schedule_offset"] <= self.training_steps <= sh["schedule_offset_end"]
        if not active:
            return
        for _, names, _ in m["groups"]:
            for name in names:
                setattr(recursive_getattr(self.model, name), self._FLAGS[method], True)
        if not self.verbose[method]:
            logger.info(f"{method} is enabled at step {self.training_steps}")
            self.verbose[method] = True
            if method == C.WEIGHT_QUANTIZATION:
                self.weight_quantization_enabled = True

    def check_all_modules(self):
        for method in self._FLAGS:
            self._check(method)

    def step(self, step_zero_check=False):
        if not step_zero_check:
            self.training_steps += 1
        self.check_all_modules()
