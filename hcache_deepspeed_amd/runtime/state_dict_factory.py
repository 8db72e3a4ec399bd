"""Model-parallel checkpoint resharding loader (Megatron layout).

Reference parity: runtime/state_dict_factory.py (``SDLoaderFactory`` :21 -- ``get_sd_loader_json`` /
``get_sd_loader``; ``SDLoaderBase.load(mp_world_size, mp_rank, ...)`` :57 picks load / merge / split by comparing
the number of checkpoint files with the target model-parallel size; ``MegatronSDLoader`` :190 with the three
historical fused-QKV layouts).

Resharding rules (key substring -> how a TP shard relates to the full tensor):
  * row-parallel weights (``attention.dense.weight``, ``mlp.dense_4h_to_h.weight``): concatenated along dim 1;
  * column-parallel tensors (``mlp.dense_h_to_4h.*``, ``word_embeddings.weight``, ``final_linear.weight``): dim 0;
  * fused ``attention.query_key_value.*``: version 0 stores ``[3, np*hn]`` blocks (q|k|v of every shard must be
    regrouped), versions 1.0 / 2.0 store per-shard ``[np*hn*3]`` / ``[np*3*hn]`` (plain dim-0 concatenation);
  * everything else is replicated.
Files are loaded through the checkpoint engine (weights-only ``torch.load``).
"""
import collections
import copy
import json
import os

import torch

from ..utils.logging import logger
from .checkpoint_engine import TorchCheckpointEngine
from .weight_quantizer import WeightQuantization

AUTO_MODULE_KEY = "auto"

_DIM1 = ("attention.dense.weight", "mlp.dense_4h_to_h.weight")
_DIM0 = ("mlp.dense_h_to_4h.weight", "mlp.dense_h_to_4h.bias", "word_embeddings.weight", "final_linear.weight")
_QKV = "attention.query_key_value"


def _rule(key):
    if any(s in key for s in _DIM1):
        return "dim1"
    if _QKV in key:
        return "qkv"
    if any(s in key for s in _DIM0):
        return "dim0"
    return "replicated"


class SDLoaderFactory:

    @staticmethod
    def get_sd_loader_json(json_file, checkpoint_engine):
        if isinstance(json_file, str):
            with open(json_file) as f:
                data = json.load(f)
        else:
            assert isinstance(json_file, dict)
            data = json_file
        sd_type = data["type"]
        if sd_type.lower() in ("bloom", "ds_model"):
            return data
        return SDLoaderFactory.get_sd_loader(data["checkpoints"], checkpoint_engine, sd_type, data["version"])

    @staticmethod
    def get_sd_loader(ckpt_list, checkpoint_engine, sd_type="Megatron", version=None):
        if sd_type == "Megatron":
            return MegatronSDLoader(ckpt_list, version, checkpoint_engine)
        raise AssertionError(f"{sd_type} checkpoint type is not supported")


class SDLoaderBase:

    def __init__(self, ckpt_list, version, checkpoint_engine):
        self.module_key = None
        self.ckpt_list = ckpt_list
        self.version = version
        self.checkpoint_engine = checkpoint_engine if checkpoint_engine is not None else TorchCheckpointEngine()
        self.check_ckpt_list()

    def _load(self, path):
        return self.checkpoint_engine.load(path, map_location="cpu")

    def load(self, mp_world_size, mp_rank, module_key=AUTO_MODULE_KEY, is_pipe_parallel=False, quantize=False,
             quantize_bits=8, quantize_groups=64, mlp_extra_grouping=True):
        """Returns ``(load_path, state_dict, (scales, merge_count))`` for ``mp_rank`` of ``mp_world_size``."""
        self.module_key = module_key
        n = len(self.ckpt_list)
        idx = mp_rank * n // mp_world_size
        if is_pipe_parallel and module_key is not None and mp_world_size != n:
            mp_world_size, idx = n, 0
        path = self.ckpt_list[idx]
        q = (quantize_bits, quantize_groups, mlp_extra_grouping) if quantize else None
        if n == mp_world_size:
            assert os.path.exists(path), path
            sd = self._load(path)
            scales = None
            if q is not None:  # int8 weights + per-group scales (reference state_dict_factory.py:62-64)
                wq = WeightQuantization(mlp_extra_grouping=mlp_extra_grouping, mp_size=mp_world_size)
                module, scales = wq.sd_quantize_megatron(self.get_module(sd), quantize_bits, quantize_groups)
                self.set_module(sd, module)
            return path, sd, (scales, 1)
        if n > mp_world_size:
            sd, scales, count = self.merge_state_dict(mp_world_size, mp_rank, q)
            return path, sd, (scales, count)
        sd, scales = self.split_state_dict(mp_world_size, mp_rank, q)
        return path, sd, (scales, 1)

    def get_merge_state_dicts(self, mp_world_size, mp_rank):
        n = len(self.ckpt_list)
        assert n % mp_world_size == 0, "Invalid checkpoints and world size for sd merge"
        per = n // mp_world_size
        files = self.ckpt_list[per * mp_rank:per * (mp_rank + 1)]
        logger.info(f"mp_rank: {mp_rank}, ckpt_list: {files}")
        return [self._load(f) for f in files]

    def get_split_state_dict(self, mp_world_size, mp_rank):
        n = len(self.ckpt_list)
        assert mp_world_size % n == 0, "Invalid checkpoints and world size for sd split"
        per = mp_world_size // n
        return self._load(self.ckpt_list[mp_rank // per]), per, mp_rank % per

    def _choose_module_key(self, sd):
        assert not ("module" in sd and "model" in sd), "checkpoint has both 'model' and 'module' keys"
        assert "module" in sd or "model" in sd, "checkpoint contains neither 'model' nor 'module' keys"
        return "module" if "module" in sd else "model"

    def get_module(self, sd):
        if self.module_key is None:
            return sd
        if self.module_key == AUTO_MODULE_KEY:
            return sd[self._choose_module_key(sd)]
        return sd[self.module_key]

    def set_module(self, sd, module):
        if self.module_key is None:
            return module
        key = self._choose_module_key(sd) if self.module_key == AUTO_MODULE_KEY else self.module_key
        sd[key] = module
        return sd

    def check_ckpt_list(self):
        assert len(self.ckpt_list) > 0
        sd = self._load(self.ckpt_list[0])
        if "mp_world_size" in sd:
            assert len(self.ckpt_list) == sd["mp_world_size"], \
                f"checkpoint count {len(self.ckpt_list)} differs from saved mp_world_size {sd['mp_world_size']}"

    def merge_state_dict(self, mp_world_size, mp_rank, *args, **kwargs):
        raise NotImplementedError

    def split_state_dict(self, mp_world_size, mp_rank, *args, **kwargs):
        raise NotImplementedError

    def sanity_check(self, ckpt_file_name):
        raise NotImplementedError


class MegatronSDLoader(SDLoaderBase):

    def merge_query_key_value(self, param_list, ckpt_ver):
        if ckpt_ver == 0:  # each shard [3 * np*hn, h]: regroup q | k | v across shards
            parts = [torch.chunk(p, 3, dim=0) for p in param_list]
            return torch.cat([torch.cat([pp[i] for pp in parts], 0) for i in range(3)], 0)
        if ckpt_ver in (1.0, 2.0):
            return torch.cat(param_list, 0)
        raise AssertionError(f"checkpoint version: {ckpt_ver} is not supported")

    def split_query_key_value(self, param, num_to_split, offset, ckpt_ver):
        if ckpt_ver == 0:
            q, k, v = torch.chunk(param, 3, dim=0)
            assert q.shape[0] % num_to_split == 0
            return torch.cat([torch.chunk(t, num_to_split, 0)[offset] for t in (q, k, v)], 0)
        if ckpt_ver in (1.0, 2.0):
            assert param.shape[0] % num_to_split == 0
            return torch.chunk(param, num_to_split, 0)[offset]
        raise AssertionError(f"checkpoint version: {ckpt_ver} is not supported")

    def merge_state_dict(self, mp_world_size, mp_rank, quantize=None, *args, **kwargs):
        """``quantize`` = (bits, groups, mlp_extra_grouping) or None: each shard of the four projection weights is
        quantized with its own group scales BEFORE the int8 shards are merged (reference :100)."""
        self.sanity_check(self.ckpt_list[0])
        sd_list = self.get_merge_state_dicts(mp_world_size, mp_rank)
        ds_sd = copy.deepcopy(sd_list[0])
        modules = [self.get_module(sd) for sd in sd_list]
        ver = self.get_checkpoint_version(ds_sd)
        wq = WeightQuantization(mlp_extra_grouping=quantize[2], mp_size=mp_world_size) if quantize else None
        out = collections.OrderedDict()
        for key in modules[0].keys():
            vals = [m[key] for m in modules]
            rule = _rule(key)
            if wq is not None and key.endswith(".weight") and rule in ("dim0", "dim1", "qkv") and \
                    any(k in key for k in ("attention.dense", "mlp.dense_4h_to_h", "mlp.dense_h_to_4h", _QKV)):
                vals = wq.Quantize(vals, quantize[0], quantize[1], key=key, merge_dim=1 if rule == "dim1" else 0)
            if rule == "dim1":
                out[key] = torch.cat(vals, 1)
            elif rule == "qkv":
                out[key] = self.merge_query_key_value(vals, ver)
            elif rule == "dim0":
                out[key] = torch.cat(vals, 0)
            else:
                out[key] = vals[0]
        return self.set_module(ds_sd, out), (wq.merge_scales() if wq is not None else None), len(modules)

    def split_state_dict(self, mp_world_size, mp_rank, quantize=None, *args, **kwargs):
        """``quantize``: the whole tensor is quantized first, then split; each target gets its slice of the group
        scales (reference merge_scales_split)."""
        sd, per, off = self.get_split_state_dict(mp_world_size, mp_rank)
        ds_sd = copy.deepcopy(sd)
        ver = self.get_checkpoint_version(ds_sd)
        wq = WeightQuantization(mlp_extra_grouping=quantize[2], mp_size=mp_world_size) if quantize else None
        out = collections.OrderedDict()
        for key, val in self.get_module(sd).items():
            rule = _rule(key)
            if wq is not None and key.endswith(".weight") and rule in ("dim0", "dim1", "qkv") and \
                    any(k in key for k in ("attention.dense", "mlp.dense_4h_to_h", "mlp.dense_h_to_4h", _QKV)):
                val = wq.Quantize([val], quantize[0], quantize[1], key=key)[0]
            if rule == "dim1":
                assert val.shape[1] % per == 0
                out[key] = torch.chunk(val, per, 1)[off]
            elif rule == "qkv":
                out[key] = self.split_query_key_value(val, per, off, ver)
            elif rule == "dim0":
                assert val.shape[0] % per == 0
                out[key] = torch.chunk(val, per, 0)[off]
            else:
                out[key] = val
        scales = wq.merge_scales_split(per)[off] if wq is not None and wq.qkv_scales else None
        return self.set_module(ds_sd, out), scales

    def sanity_check(self, ckpt_file_name):
        need = ("attention.dense.weight", "mlp.dense_4h_to_h.weight", _QKV, "mlp.dense_h_to_4h.weight",
                "mlp.dense_h_to_4h.bias")
        keys = list(self.get_module(self._load(ckpt_file_name)).keys())
        for n in need:
            assert any(n in k for k in keys), f"key: {n} is not found in the checkpoint {ckpt_file_name}"

    def get_checkpoint_version(self, state_dict):
        return self.version if self.version is not None else state_dict.get("checkpoint_version", 0)
