"""TiledLinear: split one huge linear into in x out tiles so ZeRO-3 fetches and frees it piecewise.

Reference parity: runtime/zero/tiling.py (``TiledLinear`` :32, ``TiledLinearReturnBias`` :259,
``split_tensor_along_last_dim``). Each tile is its own ``nn.Linear`` inside an ``nn.ModuleList`` so the flat
ZeRO-3 discovers every tile as a separate fetch unit; input splits are summed, output splits concatenated.
"""
import torch
import torch.nn as nn


def split_tensor_along_last_dim(tensor, partitions, contiguous_split_chunks=False):
    if isinstance(partitions, int):
        n = tensor.shape[-1]
        base, rem = divmod(n, partitions)
        partitions = [base + (1 if i < rem else 0) for i in range(partitions)]
    parts = torch.split(tensor, partitions, dim=-1)
    return tuple(p.contiguous() for p in parts) if contiguous_split_chunks else parts


def _sizes(n, k):
    base, rem = divmod(n, k)
    return [base + (1 if i < rem else 0) for i in range(k)]


class TiledLinear(nn.Module):

    def __init__(self, in_features, out_features, bias=True, in_splits=1, out_splits=1, input_is_already_split=False,
                 combine_out_splits=True, linear_cls=nn.Linear, init_linear=None, **kwargs):
        super().__init__()
        assert 1 <= in_splits <= in_features and 1 <= out_splits <= out_features
        self.in_features, self.out_features = in_features, out_features
        self.in_splits, self.out_splits = in_splits, out_splits
        self.use_bias = bias
        self.input_is_already_split = input_is_already_split
        self.combine_out_splits = combine_out_splits
        self.in_parts = _sizes(in_features, in_splits)
        self.out_parts = _sizes(out_features, out_splits)
        self.linears = nn.ModuleList()
        for o, osz in enumerate(self.out_parts):
            row = nn.ModuleList()
            for i, isz in enumerate(self.in_parts):
                # only the last input tile carries the bias (summed once)
                row.append(linear_cls(isz, osz, bias=bias and i == in_splits - 1, **kwargs))
            self.linears.append(row)
        if init_linear is not None:
            self.copy_params_from(init_linear)

    def forward(self, x):
        xs = x if self.input_is_already_split else split_tensor_along_last_dim(x, self.in_parts)
        outs = []
        for row in self.linears:
            acc = None
            for lin, xi in zip(row, xs):
                y = lin(xi)
                acc = y if acc is None else acc + y
            outs.append(acc)
        return torch.cat(outs, dim=-1) if self.combine_out_splits else outs

    @torch.no_grad()
    def copy_params_from(self, other):
        w = other.weight
        o0 = 0
        for o, osz in enumerate(self.out_parts):
            i0 = 0
            for i, isz in enumerate(self.in_parts):
                self.linears[o][i].weight.copy_(w[o0:o0 + osz, i0:i0 + isz])
                i0 += isz
            if self.use_bias and other.bias is not None:
                self.linears[o][-1].bias.copy_(other.bias[o0:o0 + osz])
            o0 += osz


class TiledLinearReturnBias(TiledLinear):
    """Variant for layers returning (output, bias) like Megatron's RowParallelLinear."""

    def forward(self, x):
        out = super().forward(x)
        return out, None
