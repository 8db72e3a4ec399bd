"""Compression-aware layers: QAT weight / activation fake-quantization and sparse / row / head / channel pruning.

Reference parity: compression/basic_layer.py (``LinearLayer_Compress`` :121, ``Embedding_Compress``,
``Conv2dLayer_Compress``, ``BNLayer_Compress``, ``ColumnParallelLinear_Compress``,
``RowParallelLinear_Compress``; ``TopKBinarizer``, ``SymQuantizer``/``AsymQuantizer``/``TernaryQuantizer``/
``BinaryQuantizer``, ``QuantAct``) and compression/utils.py.

Design: one mixin carries every technique's state and mask logic; the concrete layers only differ in how the
effective weight is applied (linear / conv / embedding / TP linears). Fake quantization of 4- and 8-bit groups
runs through the HIP group-quant kernel (ops/quantizer.fake_quantize) on GPU, with a straight-through
estimator for the gradient. Masks are plain tensors multiplied into the weight -- no module surgery until
``fix_*`` (``redundancy_clean``) physically shrinks rows / heads / channels.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.quantizer import fake_quantize


# ---------------------------------------------------------------------------------------------
# straight-through quantizers and binarizers
# ---------------------------------------------------------------------------------------------
def _group_size(x, groups):
    n = x.numel()
    groups = groups if groups and n % groups == 0 else 1
    return n // groups


class _STEQuantize(torch.autograd.Function):
    """Symmetric / asymmetric group fake-quant, identity gradient (reference SymQuantizer / AsymQuantizer)."""

    @staticmethod
    def forward(ctx, x, bits, groups, symmetric):
        gs = _group_size(x, groups)
        return fake_quantize(x.contiguous().view(-1), gs, int(bits), bool(symmetric)).view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None


class _STETernary(torch.autograd.Function):
    """2-bit ternary {-a, 0, a} per group with threshold 0.7 * mean|w| (reference TernaryQuantizer)."""

    @staticmethod
    def forward(ctx, x, groups):
        g = x.float().reshape(x.numel() // _group_size(x, groups), -1)
        thr = 0.7 * g.abs().mean(1, keepdim=True)
        pos, neg = (g > thr).float(), (g < -thr).float()
        mask = pos + neg
        alpha = (g.abs() * mask).sum(1, keepdim=True) / mask.sum(1, keepdim=True).clamp_min(1.0)
        return (alpha * (pos - neg)).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _STEBinary(torch.autograd.Function):
    """1-bit sign * mean|w| per group (reference BinaryQuantizer)."""

    @staticmethod
    def forward(ctx, x, groups):
        g = x.float().reshape(x.numel() // _group_size(x, groups), -1)
        alpha = g.abs().mean(1, keepdim=True)
        return (torch.sign(g) * alpha).reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None


def quantize_weight(w, bits, groups=1, symmetric=True):
    if bits >= 3:
        return _STEQuantize.apply(w, bits, groups, symmetric)
    if bits == 2:
        return _STETernary.apply(w, groups)
    return _STEBinary.apply(w, groups)


class TopKBinarizer(torch.autograd.Function):
    """Mask keeping the top ``ratio`` fraction of ``scores``; straight-through gradient to the scores."""

    @staticmethod
    def forward(ctx, scores, ratio, sigmoid=False):
        s = torch.sigmoid(scores) if sigmoid else scores
        keep = max(1, int(math.ceil(ratio * s.numel())))
        mask = torch.zeros_like(s)
        idx = torch.topk(s.reshape(-1), keep, sorted=False).indices
        mask.view(-1)[idx] = 1.0
        return mask

    @staticmethod
    def backward(ctx, g):
        return g, None, None


class QuantAct(nn.Module):
    """Static-range activation fake-quant: EMA of the batch min/max (reference QuantAct, momentum 0.95)."""

    def __init__(self, act_range_momentum=0.95, quant_mode="symmetric"):
        super().__init__()
        self.momentum = act_range_momentum
        self.symmetric = quant_mode == "symmetric"
        self.register_buffer("x_min_max", torch.zeros(2))

    def forward(self, x, bits, *args):
        if self.training:
            lo, hi = x.detach().min().float(), x.detach().max().float()
            if self.x_min_max.abs().sum() == 0:
                self.x_min_max[0], self.x_min_max[1] = lo, hi
            else:
                self.x_min_max[0] = self.x_min_max[0] * self.momentum + lo * (1 - self.momentum)
                self.x_min_max[1] = self.x_min_max[1] * self.momentum + hi * (1 - self.momentum)
        lo, hi = self.x_min_max[0], self.x_min_max[1]
        xf = x.float()
        if self.symmetric:
            qmax = 2**(bits - 1) - 1
            sc = torch.maximum(lo.abs(), hi.abs()).clamp_min(1e-8) / qmax
            y = torch.clamp(torch.round(xf / sc), -qmax - 1, qmax) * sc
        else:
            sc = (hi - lo).clamp_min(1e-8) / (2**bits - 1)
            y = torch.clamp(torch.round((xf - lo) / sc), 0, 2**bits - 1) * sc + lo
        return x + (y.to(x.dtype) - x).detach()  # straight-through


# ---------------------------------------------------------------------------------------------
# technique state shared by all compressible layers
# ---------------------------------------------------------------------------------------------
def _copy_q_attrs(src, dst):
    for a in ("start_bits", "target_bits", "q_period"):
        setattr(dst, a, getattr(src, a, None))


class CompressionMixin:
    """Adds the reference ``enable_*`` / ``get_mask`` / ``fix_*`` API to a module with a ``weight``."""

    def _init_compression(self):
        self.sparse_pruning_method = None
        self.row_pruning_method = None
        self.head_pruning_method = None
        self.channel_pruning_method = None
        self.activation_quantization_method = None
        self.weight.start_bits = None
        self.weight.target_bits = None
        self.weight.q_period = None
        self.weight_quantization_enabled_in_forward = False
        self.weight_quantization_enabled = False
        self.sparse_pruning_enabled = False
        self.row_pruning_enabled = False
        self.head_pruning_enabled = False
        self.channel_pruning_enabled = False
        self.activation_quantization_enabled = False
        self.weight_quantize_num_groups = 1
        self.weight_quantization_type = "symmetric"

    # ---- enable ------------------------------------------------------------------------------
    def enable_weight_quantization(self, start_bits, target_bits, quantization_period,
                                   weight_quantization_enabled_in_forward, quantization_type, num_groups):
        self.weight.start_bits = start_bits
        self.weight.target_bits = target_bits
        self.weight.q_period = quantization_period
        self.weight_quantization_enabled_in_forward = weight_quantization_enabled_in_forward
        self.weight_quantization_type = quantization_type
        self.weight_quantize_num_groups = num_groups
        if target_bits <= 2:
            assert quantization_type == "symmetric", "ternary / binary weight quantization is symmetric only"

    def enable_activation_quantization(self, bits, quantization_type, range_calibration):
        assert bits in (4, 8), "only 4/8-bit activation quantization is supported"
        self.activation_quantization_bits = bits
        self.activation_quantization_method = f"{quantization_type}_{range_calibration}"
        self.activation_symmetric = quantization_type == "symmetric"
        self.activation_quantizer = QuantAct(quant_mode=quantization_type) if range_calibration == "static" else None

    def enable_sparse_pruning(self, ratio, method):
        self.sparse_pruning_ratio = ratio
        self.sparse_pruning_method = method
        if method == "l1":
            mask = TopKBinarizer.apply(self.weight.data.abs().float(), ratio).to(self.weight.device)
            self.register_buffer("sparse_pruning_mask", mask.view_as(self.weight))
        elif method == "topk":
            self.sparse_mask_scores = nn.Parameter(torch.empty(self.weight.shape, device=self.weight.device))
            nn.init.kaiming_uniform_(self.sparse_mask_scores, a=math.sqrt(5))
            self.register_buffer("sparse_pruning_mask", None)
        else:
            raise NotImplementedError(f"sparse pruning method {method}")

    def enable_row_pruning(self, ratio, method):
        self.row_pruning_ratio = ratio
        self.row_pruning_method = method
        rows = self.weight.shape[0]
        if method == "l1":
            norms = self.weight.data.float().reshape(rows, -1).abs().sum(1)
            self.register_buffer("row_pruning_mask", TopKBinarizer.apply(norms, ratio).view(-1, 1))
        elif method == "topk":
            self.row_mask_scores = nn.Parameter(torch.empty(rows, 1, device=self.weight.device))
            nn.init.kaiming_uniform_(self.row_mask_scores, a=math.sqrt(5))
            self.register_buffer("row_pruning_mask", None)
        else:
            raise NotImplementedError(f"row pruning method {method}")

    def enable_head_pruning(self, ratio, method, num_heads):
        if method != "topk":
            raise NotImplementedError("head pruning supports method 'topk' only")
        self.num_heads = num_heads
        self.head_pruning_ratio = ratio
        self.head_pruning_method = method
        self.head_pruning_scores = nn.Parameter(torch.empty(1, num_heads, device=self.weight.device))
        nn.init.kaiming_uniform_(self.head_pruning_scores, a=math.sqrt(5))

    def enable_channel_pruning(self, ratio, method):
        self.channel_pruning_ratio = ratio
        self.channel_pruning_method = method
        ch = self.weight.shape[0]
        shape = (ch, ) + (1, ) * (self.weight.dim() - 1)
        if method == "l1":
            norms = self.weight.data.float().reshape(ch, -1).abs().sum(1)
            self.register_buffer("channel_pruning_mask", TopKBinarizer.apply(norms, ratio).view(shape))
        elif method == "topk":
            self.channel_mask_scores = nn.Parameter(torch.empty(shape, device=self.weight.device))
            nn.init.kaiming_uniform_(self.channel_mask_scores.data.view(ch, -1), a=math.sqrt(5))
            self.register_buffer("channel_pruning_mask", None)
        else:
            raise NotImplementedError(f"channel pruning method {method}")

    # ---- masks -------------------------------------------------------------------------------
    def get_mask(self, pruning_type="row"):
        if pruning_type == "sparse":
            if self.sparse_pruning_method == "l1":
                return self.sparse_pruning_mask
            return TopKBinarizer.apply(self.sparse_mask_scores, self.sparse_pruning_ratio, False)
        if pruning_type == "row":
            if self.row_pruning_method == "l1":
                return self.row_pruning_mask
            return TopKBinarizer.apply(self.row_mask_scores, self.row_pruning_ratio, False)
        if pruning_type == "head":
            return TopKBinarizer.apply(self.head_pruning_scores, self.head_pruning_ratio, False)
        if pruning_type == "channel":
            if self.channel_pruning_method == "l1":
                return self.channel_pruning_mask
            return TopKBinarizer.apply(self.channel_mask_scores, self.channel_pruning_ratio, False)
        raise NotImplementedError(pruning_type)

    def _head_mask_cols(self, w, mask):
        out, inp = w.shape[0], w.shape[1]
        return (w.view(out, self.num_heads, inp // self.num_heads) * mask.view(1, -1, 1).to(w.dtype)).view(out, inp)

    def effective_weight(self):
        w = self.weight
        if self.weight_quantization_enabled and self.weight_quantization_enabled_in_forward:
            w = quantize_weight(w, w.target_bits, self.weight_quantize_num_groups,
                                self.weight_quantization_type == "symmetric")
        if self.sparse_pruning_enabled and self.sparse_pruning_method:
            w = w * self.get_mask("sparse").view_as(w).to(w.dtype)
        if self.row_pruning_enabled and self.row_pruning_method:
            w = w * self.get_mask("row").to(w.dtype)
        if self.head_pruning_enabled and self.head_pruning_method:
            w = self._head_mask_cols(w, self.get_mask("head"))
        if self.channel_pruning_enabled and self.channel_pruning_method:
            w = w * self.get_mask("channel").to(w.dtype)
        return w

    def effective_bias(self):
        b = getattr(self, "bias", None)
        if b is None:
            return None
        if self.row_pruning_enabled and self.row_pruning_method:
            b = b * self.get_mask("row").view(-1).to(b.dtype)
        if self.channel_pruning_enabled and self.channel_pruning_method:
            b = b * self.get_mask("channel").view(-1).to(b.dtype)
        return b

    def quantize_input(self, x):
        if not (self.activation_quantization_enabled and self.activation_quantization_method):
            return x
        if self.activation_quantizer is not None:
            return self.activation_quantizer(x, self.activation_quantization_bits)
        flat = x.reshape(-1, x.shape[-1]) if x.dim() > 1 else x.reshape(1, -1)
        # dynamic range: one group per token row
        return _STEQuantize.apply(flat, self.activation_quantization_bits, flat.shape[0],
                                  self.activation_symmetric).view_as(x)

    # ---- fix (physically apply, optionally shrink) -------------------------------------------
    def _replace_weight(self, data):
        old = self.weight
        self.weight = nn.Parameter(data.contiguous())
        _copy_q_attrs(old, self.weight)

    def fix_weight_quantization(self):
        w = self.weight
        self.weight.data = quantize_weight(w.data, w.target_bits, self.weight_quantize_num_groups,
                                           self.weight_quantization_type == "symmetric")
        self.weight_quantization_enabled_in_forward = False
        return None

    def fix_sparse_pruning_helper(self):
        self.weight.data = self.weight.data * self.get_mask("sparse").detach().view_as(self.weight).to(
            self.weight.dtype)
        if self.sparse_pruning_method == "topk":
            del self.sparse_mask_scores
        self.sparse_pruning_mask = None
        self.sparse_pruning_method = None
        self.sparse_pruning_enabled = False
        return None

    def fix_row_col_pruning_helper(self, mask=None, dim_reduction=False):
        """No mask: prune this layer's OUTPUT rows (returns the row mask for the next layer). With a mask:
        drop the matching INPUT columns (the consumer of a row-pruned producer)."""
        if mask is None:
            mask = self.get_mask("row").detach().bool().view(-1)
            if dim_reduction:
                self._replace_weight(self.weight.data[mask])
                if getattr(self, "bias", None) is not None:
                    self.bias = nn.Parameter(self.bias.data[mask])
                if hasattr(self, "out_features"):
                    self.out_features = self.weight.shape[0]
            else:
                self.weight.data = self.weight.data * mask.view(-1, 1).to(self.weight.dtype)
                if getattr(self, "bias", None) is not None:
                    self.bias.data = self.bias.data * mask.to(self.bias.dtype)
            if self.row_pruning_method == "topk":
                del self.row_mask_scores
            self.row_pruning_mask = None
            self.row_pruning_method = None
        else:
            self._replace_weight(self.weight.data[:, mask.view(-1).bool()])
            if hasattr(self, "in_features"):
                self.in_features = self.weight.shape[1]
            mask = None
        self.row_pruning_enabled = False
        return mask

    def fix_head_pruning_helper(self, mask=None, num_heads=None, dim_reduction=False):
        """No mask: this is the attention OUTPUT projection -- prune its head-grouped input columns and return
        the head mask. With a mask: this is a Q/K/V projection -- drop the matching head-grouped output rows."""
        num_heads = num_heads or self.num_heads
        if mask is None:
            mask = self.get_mask("head").detach().bool().view(-1)
            out, inp = self.weight.shape
            hd = inp // num_heads
            if dim_reduction:
                self._replace_weight(self.weight.data.view(out, num_heads, hd)[:, mask].reshape(out, -1))
                if hasattr(self, "in_features"):
                    self.in_features = self.weight.shape[1]
            else:
                self.weight.data = self._head_mask_cols(self.weight.data, mask)
            del self.head_pruning_scores
            self.head_pruning_method = None
        else:
            out, inp = self.weight.shape
            self._replace_weight(self.weight.data.view(num_heads, out // num_heads, inp)[mask.view(-1)].reshape(-1, inp))
            if getattr(self, "bias", None) is not None:
                self.bias = nn.Parameter(self.bias.data.view(num_heads, -1)[mask.view(-1)].reshape(-1))
            if hasattr(self, "out_features"):
                self.out_features = self.weight.shape[0]
        self.head_pruning_enabled = False
        return mask

    def fix_channel_pruning_helper(self, mask=None, dim_reduction=False):
        if mask is None:
            mask = self.get_mask("channel").detach().bool().view(-1)
            if dim_reduction:
                self._replace_weight(self.weight.data[mask])
                if getattr(self, "bias", None) is not None:
                    self.bias = nn.Parameter(self.bias.data[mask])
                if hasattr(self, "out_channels"):
                    self.out_channels = self.weight.shape[0]
            else:
                shape = (-1, ) + (1, ) * (self.weight.dim() - 1)
                self.weight.data = self.weight.data * mask.view(shape).to(self.weight.dtype)
                if getattr(self, "bias", None) is not None:
                    self.bias.data = self.bias.data * mask.to(self.bias.dtype)
            if self.channel_pruning_method == "topk":
                del self.channel_mask_scores
            self.channel_pruning_mask = None
            self.channel_pruning_method = None
        else:
            self._replace_weight(self.weight.data[:, mask.view(-1).bool()])
            if hasattr(self, "in_channels"):
                self.in_channels = self.weight.shape[1]
            mask = None
        self.channel_pruning_enabled = False
        return mask


# ---------------------------------------------------------------------------------------------
# concrete layers
# ---------------------------------------------------------------------------------------------
class LinearLayer_Compress(CompressionMixin, nn.Linear):

    def __init__(self, *args, bias=True, **kwargs):
        super().__init__(*args, bias=bias, **kwargs)
        self._init_compression()

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}, "
                f"sparse pruning={self.sparse_pruning_method is not None}, "
                f"row pruning={self.row_pruning_method is not None}, "
                f"head pruning={self.head_pruning_method is not None}, "
                f"activation quantization={self.activation_quantization_method is not None}, "
                f"weight_quantization={self.weight.target_bits}")

    def forward(self, x, skip_bias_add=False):
        x = self.quantize_input(x)
        w, b = self.effective_weight(), self.effective_bias()
        if skip_bias_add:
            return F.linear(x, w), b
        return F.linear(x, w, b)


class Conv2dLayer_Compress(CompressionMixin, nn.Conv2d):

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._init_compression()

    def forward(self, x):
        if self.activation_quantization_enabled and self.activation_quantization_method:
            x = self.quantize_input(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
        return self._conv_forward(x, self.effective_weight(), self.effective_bias())


class BNLayer_Compress(nn.BatchNorm2d):
    """BatchNorm that follows a channel-pruned conv (reference BNLayer_Compress)."""

    def fix_channel_pruning_helper(self, mask, dim_reduction=True):
        m = mask.view(-1).bool()
        self.weight = nn.Parameter(self.weight.data[m])
        self.bias = nn.Parameter(self.bias.data[m])
        self.running_mean = self.running_mean[m]
        self.running_var = self.running_var[m]
        self.num_features = int(m.sum())


class Embedding_Compress(CompressionMixin, nn.Embedding):

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._init_compression()

    def extra_repr(self):
        return f"{self.num_embeddings}, {self.embedding_dim}, weight_quantization={self.weight.target_bits}"

    def forward(self, ids):
        return F.embedding(ids, self.effective_weight(), self.padding_idx, self.max_norm, self.norm_type,
                           self.scale_grad_by_freq, self.sparse)


class ColumnParallelLinear_Compress(CompressionMixin, nn.Module):
    """Compression-aware wrapper of the column-parallel linear (parallel/tp.LinearLayer)."""

    def __init__(self, tp_linear):
        nn.Module.__init__(self)
        self.weight = tp_linear.weight
        self.bias = tp_linear.bias
        self.tp_group = tp_linear.tp_group
        self._init_compression()

    def forward(self, x):
        from ..parallel.tp import _ColumnParallelFn
        return _ColumnParallelFn.apply(self.quantize_input(x), self.effective_weight(), self.effective_bias(),
                                       self.tp_group)


class RowParallelLinear_Compress(CompressionMixin, nn.Module):
    """Compression-aware wrapper of the row-parallel linear (parallel/tp.LinearAllreduce)."""

    def __init__(self, tp_linear):
        nn.Module.__init__(self)
        self.weight = tp_linear.weight
        self.bias = tp_linear.bias
        self.tp_group = tp_linear.tp_group
        self._init_compression()

    def forward(self, x):
        from ..parallel.tp import _AllReduceFwd
        y = _AllReduceFwd.apply(F.linear(self.quantize_input(x), self.effective_weight()), self.tp_group)
        b = self.effective_bias()
        return y + b if b is not None else y
