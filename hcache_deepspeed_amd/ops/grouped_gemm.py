"""Grouped (MoE) GEMM over expert-contiguous ragged rows, and the dropless top-k MoE FFN built on it.

Reference parity: the grouped MoE GEMM of inference/v2/kernels/cutlass_ops/moe_gemm (SURVEY.md §2.10 N15,
§2.11 K37) used by the v2 Mixtral / Qwen2-MoE implementations, and moe_scatter / moe_gather (K35/K36).

``grouped_gemm(x, w, offs)``: ``y[offs[e]:offs[e+1]] = x[offs[e]:offs[e+1]] @ w[e].T`` for ``w [E, N, K]``. On the
GPU this is ONE launch of the HIP kernel in csrc/kernels/grouped_gemm.hip (MFMA 32x32x16 bf16, LDS-DMA staged,
device-side tile plan): the routing counts never travel to the host and no capacity padding is computed. The
backward computes dX with the same kernel on the transposed weights; dW is one GEMM per expert.

``moe_ffn_dropless``: permutes the (token, choice) pairs into expert-contiguous rows with device index ops, runs the
gated expert FFN as two grouped GEMMs, and combines with the gate weights — no ``.item()`` in the whole path,
unlike the capacity/bmm formulation whose dropless capacity is ``max(count)`` (a host sync plus padding waste).
"""
import torch

from . import native


def _eligible(x, w):
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[1] % 128 == 0
            and w.shape[2] % 128 == 0 and x.shape[1] == w.shape[2])


def _ref_grouped(x, w, offs):
    y = x.new_empty(x.shape[0], w.shape[1])
    o = offs.tolist()
    for e in range(w.shape[0]):
        if o[e + 1] > o[e]:
            y[o[e]:o[e + 1]] = (x[o[e]:o[e + 1]].float() @ w[e].float().t()).to(x.dtype)
    return y


_VARIANT = int(__import__("os").environ.get("HDS_GG_VARIANT", "0"))  # 0 auto, 1 = 128^2 tiles, 2 = 256^2 tiles


def _grouped_fwd(x, w, offs, variant=None):
    T, K = x.shape
    E, N, _ = w.shape
    if native.use_native(x, w) and _eligible(x, w):
        x = x.contiguous()
        w = w.contiguous()
        offs = offs.to(device=x.device, dtype=torch.int32).contiguous()
        assert offs.numel() == E + 1, "offs must be the [E+1] exclusive prefix of the per-expert row counts"
        y = torch.empty(T, N, dtype=x.dtype, device=x.device)
        if T == 0:
            return y
        lib = native.kernels()
        work = torch.empty(2 * lib.hds_grouped_gemm_max_tiles(T, E) + 1, dtype=torch.int32, device=x.device)
        native.check(lib.hds_grouped_gemm(x.data_ptr(), w.data_ptr(), y.data_ptr(), offs.data_ptr(), work.data_ptr(),
                                          T, N, K, E, N, _VARIANT if variant is None else variant,
                                          native.stream()), "grouped_gemm")
        return y
    return _ref_grouped(x, w, offs)


class _GroupedGemm(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, w, offs):
        ctx.save_for_backward(x, w, offs)
        return _grouped_fwd(x, w, offs)

    @staticmethod
    def backward(ctx, dy):
        x, w, offs = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = _grouped_fwd(dy.contiguous(), w.transpose(1, 2).contiguous(), offs)
        if ctx.needs_input_grad[1]:
            dw = torch.zeros_like(w)
            o = offs.tolist()
            for e in range(w.shape[0]):
                if o[e + 1] > o[e]:
                    dw[e] = (dy[o[e]:o[e + 1]].t() @ x[o[e]:o[e + 1]]).to(w.dtype)
        return dx, dw, None


def grouped_gemm(x, w, offs, variant=None):
    """x [T, K] (rows sorted by expert), w [E, N, K], offs [E+1] int (exclusive prefix, offs[E] == T) -> [T, N].
    ``variant`` (GPU tile shape): None/0 = auto, 1 = 128x128 tiles (small experts / decode), 2 = 256x256 tiles."""
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
        return _GroupedGemm.apply(x, w, offs)
    return _grouped_fwd(x, w, offs, variant)


def expert_offsets(counts):
    """[E] counts -> [E+1] int32 exclusive prefix (device, no sync)."""
    offs = torch.zeros(counts.numel() + 1, dtype=torch.int32, device=counts.device)
    offs[1:] = torch.cumsum(counts.to(torch.int32), 0)
    return offs


def permute_rows(expert, pos, offs):
    """Row of every (token, choice) in the expert-contiguous layout: offs[expert] + pos, shape [T, k]."""
    return offs[:-1].long()[expert.long()] + pos.long()


def moe_ffn_dropless(x, expert, pos, gate_w, counts, w13, w2, act_fn):
    """Dropless top-k gated-expert FFN. x [T, H]; expert/pos/gate_w [T, k] from ``topk_route``; counts [E];
    w13 [E, 2I, H] (gate|up), w2 [E, H, I]; ``act_fn`` maps [rows, 2I] -> [rows, I] (e.g. ops.activations.glu)."""
    T, H = x.shape
    k = expert.shape[1]
    offs = expert_offsets(counts)
    rows = permute_rows(expert, pos, offs).reshape(-1)  # [T*k]
    xs = x.new_empty(T * k, H)
    xs[rows] = x.unsqueeze(1).expand(T, k, H).reshape(T * k, H)
    h = grouped_gemm(xs, w13, offs)
    ys = grouped_gemm(act_fn(h), w2, offs)
    out = (ys[rows].view(T, k, H).float() * gate_w.view(T, k, 1).float()).sum(1)
    return out.to(x.dtype)
