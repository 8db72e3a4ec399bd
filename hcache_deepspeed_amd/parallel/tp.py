"""Tensor parallelism: column/row-parallel linears, AutoTP sharding, training manager, Domino-style overlap.

Reference parity: module_inject/layers.py (``LinearLayer`` column-parallel, ``LinearAllreduce`` row-parallel,
training-mode ColumnParallel/RowParallel autograd :51-140, ``AsyncColumnParallel`` :83-109), module_inject/
auto_tp.py (``AutoTP`` :193 -- policy-free discovery of which linears to split), runtime/tensor_parallel/
tp_manager.py (``TpTrainingManager`` :12) and runtime/domino (overlap of the TP all-reduce with compute).

On one 8x MI355X node every GPU pair has a dedicated xGMI link, so the [tokens, hidden] all-reduce of a
row-parallel layer is latency/bandwidth cheap for TP<=8; the backward all-reduce of a column-parallel
input gradient is issued asynchronously and overlapped with the weight-gradient GEMM (Domino idea).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist


def _ws(group):
    return dist.get_world_size(group)


class _ColumnParallelFn(torch.autograd.Function):
    """y = x @ W_shard^T (+b_shard). fwd: identity on x; bwd: all-reduce dx (async, overlapped with dW)."""

    @staticmethod
    def forward(ctx, x, w, b, group):
        ctx.save_for_backward(x, w)
        ctx.group, ctx.has_b = group, b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w
        work = dist.all_reduce(dx, group=ctx.group, async_op=True) if _ws(ctx.group) > 1 else None
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = dy2.t() @ x.reshape(-1, x.shape[-1]) if ctx.needs_input_grad[1] else None
        db = dy2.sum(0) if ctx.has_b else None
        if work is not None:
            work.wait()
        return dx, dw, db, None


class _AllReduceFwd(torch.autograd.Function):
    """fwd: all-reduce (row-parallel output); bwd: identity."""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) > 1:
            from ..comm.symmetric import small_all_reduce
            x = small_all_reduce(x.contiguous(), group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _CopyToTP(torch.autograd.Function):
    """fwd: identity; bwd: all-reduce (used where a replicated activation feeds sharded compute)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class LinearLayer(nn.Module):
    """Column-parallel linear: weight rows sharded, output stays sharded (reference LinearLayer)."""

    def __init__(self, weight, bias=None, group=None):
        super().__init__()
        self.weight = weight if isinstance(weight, nn.Parameter) else nn.Parameter(weight)
        self.bias = bias if (bias is None or isinstance(bias, nn.Parameter)) else nn.Parameter(bias)
        self.tp_group = group

    def forward(self, x):
        return _ColumnParallelFn.apply(x, self.weight, self.bias, self.tp_group)


class LinearAllreduce(nn.Module):
    """Row-parallel linear: weight columns sharded, partial outputs all-reduced (reference LinearAllreduce)."""

    def __init__(self, weight, bias=None, group=None):
        super().__init__()
        self.weight = weight if isinstance(weight, nn.Parameter) else nn.Parameter(weight)
        self.bias = bias if (bias is None or isinstance(bias, nn.Parameter)) else nn.Parameter(bias)
        self.tp_group = group

    def forward(self, x):
        y = _AllReduceFwd.apply(F.linear(x, self.weight), self.tp_group)
        return y + self.bias if self.bias is not None else y


def _rows(w, r, n):
    s = w.shape[0] // n
    return w[r * s:(r + 1) * s]


def _cols(w, r, n):
    s = w.shape[1] // n
    return w[:, r * s:(r + 1) * s]


def get_shard_size(total, n, rank):
    """Uneven shard sizes (reference tp_shard.get_shard_size): first ``total % n`` ranks get one extra."""
    return total // n + (1 if rank < total % n else 0)


def get_shard_size_list(total, n):
    return [get_shard_size(total, n, r) for r in range(n)]


# ---------------------------------------------------------------------------------------------
# AutoTP
# ---------------------------------------------------------------------------------------------
ROW_NAMES = ("o_proj", "down_proj", "out_proj", "dense_4h_to_h", "fc2", "c_proj", "wo", "w2")
COLUMN_NAMES = ("q_proj", "k_proj", "v_proj", "qkv_proj", "gate_proj", "up_proj", "gate_up_proj", "dense_h_to_4h",
                "fc1", "c_fc", "query_key_value", "wq", "wk", "wv", "w1", "w3")


class AutoTP:
    """Shard a model's linears in place over ``group`` (policy-free, by module role names)."""

    def __init__(self, model, group, tp_size=None):
        self.model = model
        self.group = group
        self.n = tp_size or _ws(group)
        self.r = dist.get_rank(group) if group is not None else 0

    def _shard_llama_attention(self, attn):
        D, nq, nkv = attn.d, attn.n_q, attn.n_kv
        assert nq % self.n == 0 and nkv % self.n == 0, "heads must divide the TP size"
        w = attn.qkv_proj.weight.data
        q, k, v = w.split([nq * D, nkv * D, nkv * D], 0)
        lq, lkv = nq // self.n, nkv // self.n
        r = self.r
        nw = torch.cat([q[r * lq * D:(r + 1) * lq * D], k[r * lkv * D:(r + 1) * lkv * D],
                        v[r * lkv * D:(r + 1) * lkv * D]], 0).clone()
        attn.qkv_proj = LinearLayer(nw, None, self.group)
        attn.qkv_proj.weight.ds_tp_sub_params = (nq * D, nkv * D, nkv * D)  # q/k/v sliced independently
        attn.o_proj = LinearAllreduce(_cols(attn.o_proj.weight.data, r, self.n).clone(), None, self.group)
        attn.n_q, attn.n_kv = lq, lkv

    def _shard_llama_mlp(self, mlp):
        w = mlp.gate_up_proj.weight.data
        I = w.shape[0] // 2
        g, u = w.split([I, I], 0)
        nw = torch.cat([_rows(g, self.r, self.n), _rows(u, self.r, self.n)], 0).clone()
        mlp.gate_up_proj = LinearLayer(nw, None, self.group)
        mlp.gate_up_proj.weight.ds_tp_sub_params = (I, I)
        mlp.down_proj = LinearAllreduce(_cols(mlp.down_proj.weight.data, self.r, self.n).clone(), None, self.group)

    def shard(self):
        from ..models.llama import LlamaAttention, LlamaMLP
        for name, m in list(self.model.named_modules()):
            if isinstance(m, LlamaAttention):
                self._shard_llama_attention(m)
            elif isinstance(m, LlamaMLP):
                self._shard_llama_mlp(m)
        # generic nn.Linear children by role name (HF-style models)
        for name, m in list(self.model.named_modules()):
            for cname, child in list(m.named_children()):
                if not isinstance(child, nn.Linear) or isinstance(child, (LinearLayer, LinearAllreduce)):
                    continue
                if cname in ROW_NAMES:
                    b = child.bias.data.clone() if child.bias is not None else None
                    setattr(m, cname, LinearAllreduce(_cols(child.weight.data, self.r, self.n).clone(), b, self.group))
                elif cname in COLUMN_NAMES:
                    b = _rows(child.bias.data[:, None], self.r, self.n)[:, 0].clone() if child.bias is not None \
                        else None
                    setattr(m, cname, LinearLayer(_rows(child.weight.data, self.r, self.n).clone(), b, self.group))
        for p in self.model.parameters():
            p.ds_tensor_model_parallel = False
        for m in self.model.modules():
            if isinstance(m, (LinearLayer, LinearAllreduce)):
                m.weight.ds_tensor_model_parallel = True
                # checkpoint metadata: the dim the TP slices concatenate along (universal_checkpoint_info)
                m.weight.ds_tp_cat_dim = 1 if isinstance(m, LinearAllreduce) else 0
                if m.bias is not None and isinstance(m, LinearLayer):
                    m.bias.ds_tensor_model_parallel = True
                    m.bias.ds_tp_cat_dim = 0
        return self.model


class TpTrainingManager:
    """``deepspeed.tp_model_init`` backend (reference runtime/tensor_parallel/tp_manager.py:12)."""

    def __init__(self, model, tp_size, dtype, group=None):
        from ..utils import groups
        if group is None:
            if groups._State.topo is None or groups.get_tensor_model_parallel_world_size() != tp_size:
                dist.init_distributed(verbose=False)
                groups.reset()
                groups.initialize(tp=tp_size)
            group = groups._get_model_parallel_group()
        self.module = AutoTP(model, group, tp_size).shard().to(dtype)
        self.module._hds_tp_size = tp_size


def copy_to_tensor_parallel_region(x, group):
    return _CopyToTP.apply(x, group)


def reduce_from_tensor_parallel_region(x, group):
    return _AllReduceFwd.apply(x, group)
