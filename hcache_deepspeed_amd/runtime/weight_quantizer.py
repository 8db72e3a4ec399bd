"""Grouped symmetric int8/int4 weight quantization of Megatron checkpoints while they are loaded / resharded.

Reference: runtime/weight_quantizer.py ``WeightQuantization`` (``quantize_data``, ``Quantize``, ``merge_scales``,
``merge_scales_split``, ``sd_quantize_megatron``), used by runtime/state_dict_factory.py:62-64,100 when
``SDLoaderBase.load(..., quantize=True)``.

Per tensor: the flattened values are cut into ``groups`` equal groups (twice as many for the MLP projections with
``mlp_extra_grouping``), each group gets the scale 2^bits / (2 max|w| + 1e-5), and the values become
round(w * scale) clamped to the signed ``bits`` range, stored as int8. The per-layer scale record is the inverse
scales of the four quantized projections in the order [qkv, attention dense, h->4h, 4h->h], zero-padded to one
width: the layout the inference kernels' dequantization reads (ops/quantizer.py).
"""
import torch

_QUANT_KEYS = ("attention.query_key_value.weight", "attention.dense.weight", "mlp.dense_h_to_4h.weight",
               "mlp.dense_4h_to_h.weight")


def _kind(key):
    for i, k in enumerate(_QUANT_KEYS):
        if k in key:
            return i
    return None


class WeightQuantization:

    def __init__(self, mlp_extra_grouping=True, mp_size=1):
        self.mlp_extra_grouping = bool(mlp_extra_grouping)
        self.mp_size = int(mp_size)
        self._scales = {i: [] for i in range(len(_QUANT_KEYS))}  # kind -> [per layer inverse scales [1, g]]

    # reference attribute names of the four scale lists
    @property
    def qkv_scales(self):
        return self._scales[0]

    @property
    def dense_scales(self):
        return self._scales[1]

    @property
    def mlph4h_scales(self):
        return self._scales[2]

    @property
    def mlp4hh_scales(self):
        return self._scales[3]

    def quantize_data(self, data, quantize_bits, groups, key=None):
        """(int8 tensor of ``data``'s shape, scales [groups, 1]) -- scale = 2^bits / (2 max|w| + 1e-5) per group."""
        flat = data.detach().float().reshape(groups, -1)
        amax = flat.abs().amax(dim=1, keepdim=True)
        scale = float(1 << quantize_bits) / (2 * amax + 1e-5)
        lo, hi = -(1 << (quantize_bits - 1)), (1 << (quantize_bits - 1)) - 1
        q = (flat * scale).round_().clamp_(lo, hi).to(torch.int8).reshape(data.shape)
        return q, scale

    def is_mlp(self, data, merge_count=1):
        r0, r1 = data.shape[0], data.shape[1]
        return self.mp_size * r0 * merge_count / r1 == 4 or self.mp_size * r1 * merge_count / r0 == 4

    def is_qkv(self, data):
        r0, r1 = data.shape[0], data.shape[1]
        return self.mp_size * r0 / r1 == 3 or self.mp_size * r1 / r0 == 3

    def Quantize(self, value_list, quantize_bits, groups, key, merge_dim=0):  # noqa: N802 (reference name)
        """Quantize every shard of one tensor (``value_list``: the shards about to be merged, or one tensor) in place
        of the list; record the inverse scales of this layer under the tensor's kind."""
        if self.mlp_extra_grouping and self.is_mlp(value_list[0], merge_count=len(value_list)):
            groups *= 2
        inv = []
        for i, v in enumerate(value_list):
            q, s = self.quantize_data(v, quantize_bits, groups, key)
            value_list[i] = q
            inv.append(s)
        rec = (1.0 / torch.cat(inv, dim=merge_dim)).reshape(1, -1)
        k = _kind(key)
        self._scales[1 if k is None else k].append(rec)
        return value_list

    @staticmethod
    def merge_layer_scales(layer_scales):
        width = max(s.shape[-1] for s in layer_scales)
        padded = [torch.nn.functional.pad(s, (0, width - s.shape[-1])) for s in layer_scales]
        return torch.cat(padded).unsqueeze(0)

    def merge_scales(self):
        """[layers, 4, width]: per layer [qkv, dense, h->4h, 4h->h] inverse scales."""
        layers = zip(self.qkv_scales, self.dense_scales, self.mlph4h_scales, self.mlp4hh_scales)
        return torch.cat([self.merge_layer_scales(list(ls)) for ls in layers]) if self.qkv_scales else None

    def merge_scales_split(self, split_count):
        """The same, per split target: each layer's scales cut into ``split_count`` equal parts (the column / row
        groups of each model-parallel slice); the qkv / dense parts are zero-padded to twice their width (the
        reference layout: those two have half the groups of the MLP projections)."""
        out = [[] for _ in range(split_count)]
        for qkv, dense, h4h, hh4 in zip(self.qkv_scales, self.dense_scales, self.mlph4h_scales, self.mlp4hh_scales):
            parts = [torch.chunk(t, split_count, dim=1) for t in (qkv, dense, h4h, hh4)]
            for s in range(split_count):
                q, d, a, b = (p[s] for p in parts)
                out[s].append(self.merge_layer_scales([torch.cat((q, torch.zeros_like(q)), 1),
                                                       torch.cat((d, torch.zeros_like(d)), 1), a, b]))
        return [torch.cat(o) if o else None for o in out]

    def sd_quantize_megatron(self, sd, quantize_bits, groups):
        """Quantize the four projection weights of every layer of ``sd`` in place; returns (sd, merged scales)."""
        for key in list(sd.keys()):
            if _kind(key) is not None:
                sd[key] = self.Quantize([sd[key]], quantize_bits, groups, key=key)[0]
        return sd, self.merge_scales()
