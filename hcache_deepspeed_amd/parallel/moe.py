"""Mixture of Experts with expert parallelism (EP all-to-all over xGMI).

Reference parity: moe/layer.py (``MoE`` :17-132), moe/sharded_moe.py (``TopKGate`` :183-447, ``MOELayer``
:449-677, ``_AllToAll``), moe/experts.py (``Experts`` :13), moe/utils.py (``split_params_into_different_moe_groups_for_optimizer`` :155, ``is_moe_param``), utils/groups.py expert groups (E+D layout :236-428).

Dispatch is capacity based: tokens are permuted into an expert-major [E, C, H] tensor by the HIP dispatch
kernel, ONE ``all_to_all_single`` with equal splits moves each expert's slots to its owner (on the full
xGMI mesh this uses every link of every GPU at once), the local experts run as per-expert 2-D hipBLASLt GEMMs
over [E_local, ep*C, H] slices (``expert_linear``), one all-to-all returns the results and the
combine kernel un-permutes with the gate weights. No dense [T, E, C] dispatch masks are ever built.

Expert tensor parallelism (``enable_expert_tensor_parallelism`` under a TP dense model, reference moe/layer.py:52-58,
moe/mappings.py:105-113): each TP rank sends only its 1/tp of the capacity slots through the expert all-to-all,
all-gathers its experts' slots from the TP peers, runs column/row-sharded experts and folds the partial sums and
the token drop into ONE reduce-scatter before the return all-to-all.
"""
import copy
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import comm as dist
from ..ops.activations import glu
from ..ops.moe import moe_combine, moe_dispatch, topk_route
from ..utils import groups

# MOELayer: run the grouped experts over the occupied capacity slots only (HDS_MOE_EXACT_ROWS=0: every slot)
_EXACT_ROWS = os.environ.get("HDS_MOE_EXACT_ROWS", "1") != "0"


class _AllToAll(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        if dist.get_world_size(group) == 1:
            return x
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return _AllToAll.apply(g, ctx.group), None


# ---------------------------------------------------------------------------------------------------------------
# tensor-parallel token mappings (reference moe/mappings.py:105-113 drop_tokens / gather_tokens). Tokens are
# duplicated across the TP ranks of a tensor-parallel dense model; each rank keeps 1/tp of the capacity slots
# across the expert all-to-all (1/tp of its bytes on xGMI). Every mapping works on a dim moved to the front so the
# collective is one flat all_gather_into_tensor / reduce_scatter_tensor.
# ---------------------------------------------------------------------------------------------------------------
def _tp():
    if groups._State.topo is None:
        return None, 1, 0
    n = groups.get_tensor_model_parallel_world_size()
    return (groups._get_model_parallel_group() if n > 1 else None), n, groups.get_tensor_model_parallel_rank()


def _tp_gather(x, dim):
    grp, n, _ = _tp()
    xt = x.movedim(dim, 0).contiguous()
    out = xt.new_empty((n * xt.shape[0], ) + tuple(xt.shape[1:]))
    dist.all_gather_into_tensor(out, xt, group=grp)
    return out.movedim(0, dim)


def _tp_reduce_scatter(x, dim):
    grp, n, _ = _tp()
    xt = x.movedim(dim, 0).contiguous()
    out = xt.new_empty((xt.shape[0] // n, ) + tuple(xt.shape[1:]))
    dist.reduce_scatter_tensor(out, xt, group=grp)
    return out.movedim(0, dim)


def _tp_narrow(x, dim):
    _, n, r = _tp()
    c = x.shape[dim] // n
    return x.narrow(dim, r * c, c)


class _DropTokens(torch.autograd.Function):
    """fwd: this TP rank's 1/tp slice of ``dim`` (the inputs are replicated); bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, dim):
        ctx.dim = dim
        return _tp_narrow(x, dim).contiguous()

    @staticmethod
    def backward(ctx, g):
        return _tp_gather(g, ctx.dim), None


class _GatherTokens(torch.autograd.Function):
    """fwd: all-gather ``dim`` over TP; bwd: this rank's slice (the consumer's gradient is replicated) or, with
    ``partial_grad`` (the consumer is a TP-sharded expert whose input gradient is a partial sum), reduce-scatter."""

    @staticmethod
    def forward(ctx, x, dim, partial_grad):
        ctx.dim, ctx.partial = dim, partial_grad
        return _tp_gather(x, dim)

    @staticmethod
    def backward(ctx, g):
        return (_tp_reduce_scatter(g, ctx.dim) if ctx.partial else _tp_narrow(g, ctx.dim).contiguous()), None, None


class _ReduceScatterTokens(torch.autograd.Function):
    """fwd: sum the TP ranks' partial expert outputs and keep this rank's slice of ``dim`` (all-reduce + drop in
    one reduce-scatter); bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, dim):
        ctx.dim = dim
        return _tp_reduce_scatter(x, dim)

    @staticmethod
    def backward(ctx, g):
        return _tp_gather(g.contiguous(), ctx.dim), None


def drop_tokens(x, dim=0):
    return x if _tp()[1] == 1 else _DropTokens.apply(x, dim)


def gather_tokens(x, dim=0, partial_grad=False):
    return x if _tp()[1] == 1 else _GatherTokens.apply(x, dim, partial_grad)


class TopKGate(nn.Module):

    def __init__(self, model_dim, num_experts, k=1, capacity_factor=1.0, eval_capacity_factor=1.0, min_capacity=8,
                 noisy_gate_policy=None, drop_tokens=True, use_rts=True, ep_group=None,
                 top2_2nd_expert_sampling=True):
        super().__init__()
        self.wg = nn.Linear(model_dim, num_experts, bias=False)
        self.k = k
        self.capacity_factor, self.eval_capacity_factor = capacity_factor, eval_capacity_factor
        self.min_capacity = min_capacity
        self.noisy_gate_policy = noisy_gate_policy
        self.drop_tokens = drop_tokens
        self.use_rts = use_rts
        self.ep_group = ep_group
        self.num_experts = num_experts

    def forward(self, x):
        logits = F.linear(x.float(), self.wg.weight.float())
        cf = self.capacity_factor if self.training else self.eval_capacity_factor
        expert, pos, w, C, l_aux, counts = topk_route(logits, self.k, cf, self.min_capacity, self.drop_tokens,
                                                      self.use_rts, True, self.noisy_gate_policy, self.training)
        if not self.drop_tokens and self.ep_group is not None and dist.get_world_size(self.ep_group) > 1:
            c = torch.tensor([C], device=x.device)
            dist.all_reduce(c, op=dist.ReduceOp.MAX, group=self.ep_group)
            C = int(c.item())
        return expert, pos, w, C, l_aux, counts


class Experts(nn.Module):
    """``num_local_experts`` copies of ``expert`` (reference moe/experts.py). Params are tagged as MoE params."""

    def __init__(self, expert, num_local_experts=1, expert_group_name=None):
        super().__init__()
        self.deepspeed_experts = nn.ModuleList([copy.deepcopy(expert) for _ in range(num_local_experts)])
        self.num_local_experts = num_local_experts
        self._hds_expert_group = expert_group_name
        for e in self.deepspeed_experts:
            for p in e.parameters():
                p.allreduce = False
                p.group_name = expert_group_name
                p._hds_expert_stacked = False
                p._hds_num_local = num_local_experts

    def forward(self, x):
        # x: [E_local, N, H]
        outs = [e(x[i]) for i, e in enumerate(self.deepspeed_experts)]
        return torch.stack(outs, 0)


class _ExpertLinear(torch.autograd.Function):
    """y[e] = x[e] @ w[e]^T for stacked experts x [E, C, K], w [E, N, K], as E plain 2-D GEMMs written into slices
    of one output (and, in backward, of one dX and one dW). Batched ``torch.bmm`` with the transposed stacked weight
    hits a hipBLASLt failure on MI355X at Mixtral-8x7B shapes (HIPBLAS_STATUS_INTERNAL_ERROR for the strided batched
    TN problem m 4096 n 1280 k 14336, then an illegal access in the rocBLAS fallback); the 2-D forms are the
    projection GEMMs the dense model runs every step (NT forward, layout-timed dgrad / wgrad from ops/gemm.py).

    ``segs`` (host ints): per expert, the (start, rows) row ranges that hold tokens -- dispatch fills each expert's
    capacity slots densely from 0 and zeroes the rest, so an expert's tokens are one prefix per source rank (one
    segment at EP 1, one per EP rank behind the all-to-all). The GEMMs run over those rows only and every other row
    of each output is zeroed -- exactly what the full GEMMs give for zero slots. With capacity factor 1.25 a fifth of
    the expert GEMM rows were empty."""

    @staticmethod
    def forward(ctx, x, w, segs=None):
        E, C, K = x.shape
        y = x.new_empty(E, C, w.shape[1])
        segs = tuple(((0, C), ) for _ in range(E)) if segs is None else segs
        for e in range(E):
            for s0, m in segs[e]:
                torch.mm(x[e, s0:s0 + m], w[e].t(), out=y[e, s0:s0 + m])
            for a, b in _gaps(segs[e], C):
                y[e, a:b].zero_()
        # like runtime/zero/linear.py: keep the Parameter object, not its (ZeRO-3 gathered) data, for backward
        ctx.save_for_backward(x)
        ctx.weight = w
        ctx.segs = segs
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..ops.gemm import dgrad, wgrad
        from ..runtime.zero.linear import write_weight_grad
        (x, ) = ctx.saved_tensors
        w, segs = ctx.weight, ctx.segs
        C = x.shape[1]
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            for e in range(x.shape[0]):
                for s0, m in segs[e]:
                    dgrad(dy[e, s0:s0 + m], w[e], out=dx[e, s0:s0 + m])
                for a, b in _gaps(segs[e], C):
                    dx[e, a:b].zero_()
        if ctx.needs_input_grad[1]:

            def gemm(out, accumulate):  # straight into the ZeRO gradient buffer (no AccumulateGrad add)
                for e in range(x.shape[0]):
                    acc = accumulate
                    for s0, m in segs[e]:
                        wgrad(dy[e, s0:s0 + m], x[e, s0:s0 + m], out[e], acc)
                        acc = True
                    if not acc:
                        out[e].zero_()  # no token reached this expert: its gradient is zero

            if not write_weight_grad(w, gemm):
                dw = torch.empty_like(w)
                gemm(dw, False)
        return dx, dw, None


def _gaps(segs, C):
    """[a, b) row ranges of [0, C) outside the sorted, disjoint segments."""
    out, pos = [], 0
    for s0, m in segs:
        if s0 > pos:
            out.append((pos, s0))
        pos = max(pos, s0 + m)
    if pos < C:
        out.append((pos, C))
    return out


def occupied_segments(counts, C, blocks=1, granule=128):
    """Per local expert, the (start, rows) ranges holding tokens. ``counts``: [blocks][E_local] token counts (one row
    per source rank behind the EP all-to-all); block r of an expert occupies rows [r*C, r*C + min(count, C)), rounded
    up to ``granule`` rows (few distinct GEMM shapes) and capped at the block."""
    n_local = len(counts[0])
    segs = []
    for j in range(n_local):
        s = []
        for r in range(blocks):
            m = min(C, -(-min(int(counts[r][j]), C) // granule) * granule)
            if m > 0:
                s.append((r * C, m))
        segs.append(tuple(s))
    return tuple(segs)


def expert_linear(x, w, segs=None):
    if torch.is_grad_enabled() or x.is_cuda:  # the same Function on CPU, so gloo tests exercise the GPU path's logic
        return _ExpertLinear.apply(x.contiguous(), w, segs)
    return torch.bmm(x, w.transpose(1, 2))


class GroupedSwiGLUExperts(nn.Module):
    """E_local SwiGLU experts stored stacked ([E, 2I, H], [E, H, I]) and run as batched GEMMs."""

    def __init__(self, hidden, inter, num_local_experts, expert_group_name=None, std=0.02, act="silu", tp_size=1):
        super().__init__()
        assert inter % tp_size == 0, f"expert intermediate size {inter} not divisible by expert TP size {tp_size}"
        # expert tensor parallelism: this rank holds gate/up rows [r*I/tp, (r+1)*I/tp) (column parallel) and the
        # matching w2 columns (row parallel); the partial outputs are summed by the MoE layer's reduce-scatter
        self.tp_size = tp_size
        inter = inter // tp_size
        self.w13 = nn.Parameter(torch.empty(num_local_experts, 2 * inter, hidden))
        self.w2 = nn.Parameter(torch.empty(num_local_experts, hidden, inter))
        self._std = std
        self.act = act
        self.num_local_experts = num_local_experts
        self._hds_expert_group = expert_group_name
        for p in (self.w13, self.w2):
            p.allreduce = False
            p.group_name = expert_group_name
            p._hds_expert_stacked = True  # dim 0 = local expert index
            p._hds_num_local = num_local_experts
            p.tensor_model_parallel = tp_size > 1
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.normal_(self.w13, std=self._std)
        nn.init.normal_(self.w2, std=self._std)

    @torch.no_grad()
    def load_full(self, w13, w2, tp_rank=0):
        """Copy this TP rank's shard of full (unsharded) stacked weights w13 [E, 2I, H] (gate | up) and w2
        [E, H, I]."""
        i_full = w2.shape[-1]
        i = i_full // self.tp_size
        lo = tp_rank * i
        self.w13.copy_(torch.cat([w13[:, lo:lo + i], w13[:, i_full + lo:i_full + lo + i]], 1))
        self.w2.copy_(w2[:, :, lo:lo + i])

    def forward(self, x, segs=None):
        h = expert_linear(x, self.w13, segs)
        return expert_linear(glu(h, self.act), self.w2, segs)


class MOELayer(nn.Module):

    def __init__(self, gate, experts, ep_group_name, ep_size, num_local_experts, expert_tp=False):
        super().__init__()
        self.expert_tp = expert_tp
        self.gate = gate
        self.experts = experts
        self.ep_group_name = ep_group_name
        self.ep_size = ep_size
        self.num_local_experts = num_local_experts
        self.l_aux = None
        self.exp_counts = None

    @property
    def ep_group(self):
        return groups._State.expert_groups.get(self.ep_group_name) if self.ep_size > 1 else None

    def forward(self, x):
        shape = x.shape
        H = shape[-1]
        x2 = x.reshape(-1, H)
        E = self.num_local_experts * self.ep_size
        expert, pos, w, C, l_aux, counts = self.gate(x2)
        tp = _tp()[1]
        # expert TP: the TP ranks split the slots over the all-to-all. Without it the (replicated) experts run the
        # same slots on every TP rank, so their gradients need no reduction over TP.
        sharded = self.expert_tp and tp > 1
        if sharded and C % tp:
            # slots split evenly over the TP ranks: pad the buffer, keep every dropped assignment dropped
            Cp = -(-C // tp) * tp
            pos = torch.where(pos >= C, torch.full_like(pos, Cp), pos)
            C = Cp
        disp = moe_dispatch(x2, expert, pos, E, C).view(E, C, H)  # expert-major
        # tokens are replicated over a TP dense model's ranks: each sends only its 1/tp of the slots
        if sharded:
            disp = drop_tokens(disp, 1)
        Cl = disp.shape[1]
        if self.ep_size > 1:
            disp = _AllToAll.apply(disp.contiguous(), self.ep_group)  # now [ep(src), E_local, Cl, H]
            local = disp.view(self.ep_size, self.num_local_experts, Cl, H).transpose(0, 1)
        else:
            local = disp.view(1, E, Cl, H).transpose(0, 1)  # [E_local, 1, Cl, H]
        if sharded:  # TP-sharded experts see every slot of their experts (gathered over the TP ranks)
            local = gather_tokens(local, 2, partial_grad=isinstance(self.experts, GroupedSwiGLUExperts))
        Cx = local.shape[2]
        xe = local.reshape(self.num_local_experts, self.ep_size * Cx, H)
        if not sharded and isinstance(self.experts, GroupedSwiGLUExperts) and _EXACT_ROWS:
            # the experts' GEMMs skip the empty capacity slots: each expert's tokens from one source rank sit in the
            # first min(count, C) slots of that rank's block (one host read of the counts per layer -- behind the EP
            # all-to-all, of every source rank's counts, all-gathered; rounded up to 128 rows so the GEMM shapes and
            # the per-shape layout timings of ops/gemm.py stay few)
            if self.ep_size > 1:
                allc = torch.empty(self.ep_size * E, dtype=counts.dtype, device=counts.device)
                dist.all_gather_into_tensor(allc, counts.contiguous().view(-1), group=self.ep_group)
                allc = allc.view(self.ep_size, E)
                r0 = dist.get_rank(self.ep_group) * self.num_local_experts
                cnt = allc[:, r0:r0 + self.num_local_experts].tolist()
            else:
                cnt = [counts.tolist()]
            y = self.experts(xe, segs=occupied_segments(cnt, Cx, self.ep_size))
        else:
            y = self.experts(xe)
        y = y.view(self.num_local_experts, self.ep_size, Cx, H)
        if sharded:
            if isinstance(self.experts, GroupedSwiGLUExperts):
                y = _ReduceScatterTokens.apply(y, 2)  # partial sums -> this rank's summed slots
            else:  # a TP-aware user expert reduced internally: keep this rank's slots
                y = drop_tokens(y, 2)
        y = y.transpose(0, 1).contiguous()  # [ep, E_local, Cl, H]
        if self.ep_size > 1:
            y = _AllToAll.apply(y, self.ep_group)
        y = y.view(E, Cl, H)
        if sharded:
            y = gather_tokens(y, 1)
        y = y.reshape(E * C, H)
        out = moe_combine(y, expert, pos, w, C)
        self.l_aux, self.exp_counts = l_aux, counts
        return out.view(shape)


class MoE(nn.Module):
    """Reference-compatible MoE block: returns (output, l_aux, exp_counts)."""

    def __init__(self, hidden_size, expert=None, num_experts=1, ep_size=1, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, min_capacity=4, use_residual=False, noisy_gate_policy=None,
                 drop_tokens=True, use_rts=True, use_tutel=False, enable_expert_tensor_parallelism=False,
                 top2_2nd_expert_sampling=True, expert_intermediate_size=None):
        super().__init__()
        assert num_experts % ep_size == 0, f"num_experts ({num_experts}) must be divisible by ep_size ({ep_size})"
        self.ep_size = ep_size
        self.num_experts = num_experts
        self.num_local_experts = num_experts // ep_size
        self.expert_group_name = f"ep_size_{ep_size}"
        if ep_size > 1 and self.expert_group_name not in groups._State.expert_groups:
            if groups._State.topo is None:
                groups.initialize()
            groups._create_expert_and_data_parallel(ep_size)
        # expert tensor parallelism (reference moe/layer.py:52-58, sharded_moe.py:609-660): with a TP dense model
        # the EP groups already pair ranks of equal TP coordinate (utils/groups.py), so each TP rank's all-to-all
        # carries 1/tp of the slots and the experts are sharded over the same TP group
        tp = _tp()[1]
        self.enable_expert_tensor_parallelism = bool(enable_expert_tensor_parallelism) and tp > 1
        if expert is None:
            experts = GroupedSwiGLUExperts(hidden_size, expert_intermediate_size or 4 * hidden_size,
                                           self.num_local_experts, self.expert_group_name,
                                           tp_size=tp if self.enable_expert_tensor_parallelism else 1)
        else:
            # a user expert under expert TP must be TP-aware itself (a Megatron-style MLP that all-reduces its
            # output), exactly as in the reference
            experts = Experts(expert, self.num_local_experts, self.expert_group_name)
        gate = TopKGate(hidden_size, num_experts, k, capacity_factor, eval_capacity_factor, min_capacity,
                        noisy_gate_policy, drop_tokens, use_rts, None, top2_2nd_expert_sampling)
        self.deepspeed_moe = MOELayer(gate, experts, self.expert_group_name, ep_size, self.num_local_experts,
                                      expert_tp=self.enable_expert_tensor_parallelism)
        gate.ep_group = self.deepspeed_moe.ep_group
        self.use_residual = use_residual
        if use_residual:
            self.mlp = copy.deepcopy(expert)
            self.coefficient = nn.Linear(hidden_size, 2)

    def forward(self, hidden_states, used_token=None):
        out = self.deepspeed_moe(hidden_states)
        if self.use_residual:
            mo = self.mlp(hidden_states)
            coef = torch.softmax(self.coefficient(hidden_states), dim=-1)
            out = out * coef[..., 0:1] + mo * coef[..., 1:]
        return out, self.deepspeed_moe.l_aux, self.deepspeed_moe.exp_counts


def is_moe_param(p):
    return hasattr(p, "allreduce") and not p.allreduce


def split_params_into_different_moe_groups_for_optimizer(param_groups, max_group_size=178956971):
    """Split each optimizer group into dense + one group per expert group (reference moe/utils.py:155)."""
    if isinstance(param_groups, dict):
        param_groups = [param_groups]
    out = []
    for g in param_groups:
        dense = {k: v for k, v in g.items() if k != "params"}
        dense["params"] = [p for p in g["params"] if not is_moe_param(p)]
        out.append(dense)
        by = {}
        for p in g["params"]:
            if is_moe_param(p):
                by.setdefault(p.group_name, []).append(p)
        for name, ps in by.items():
            ng = {k: v for k, v in g.items() if k != "params"}
            ng.update(params=ps, moe=True, name=name)
            out.append(ng)
    return out
