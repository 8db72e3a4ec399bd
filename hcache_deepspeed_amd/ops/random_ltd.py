"""Random-LTD token ops: sort sampled indices, gather / scatter token rows, slice attention masks.

Reference parity: ops/random_ltd/dropping_utils.py (``gpt_sample_tokens``, ``bert_sample_tokens``,
``GatherTokens``, ``ScatterTokens``) over csrc/random_ltd. GPU tensors run the HIP kernels of
csrc/kernels/token_ops.hip; CPU tensors run the torch reference below (also the numerics reference of the tests).
Layout: activations [B, S, H] (``batch_first``) or [S, B, H]; indices [B, R] int, sorted per row.
"""
import torch

from . import native


def token_sort_(keys):
    """Sort every row of an int32 [..., n] tensor ascending, in place (n <= 16384 on GPU)."""
    if native.use_native(keys):
        assert keys.dtype == torch.int32 and keys.is_contiguous() and keys.shape[-1] <= 16384
        n = keys.shape[-1]
        native.check(native.kernels().hds_token_sort(keys.data_ptr(), keys.numel() // n, n, native.stream()),
                     "token_sort")
        return keys
    keys.copy_(keys.sort(dim=-1).values)
    return keys


def _gather_ref(x, idx):
    B, S, H = x.shape
    flat = (idx.long() + torch.arange(B, device=x.device)[:, None] * S).reshape(-1)
    return x.reshape(B * S, H).index_select(0, flat).view(B, -1, H)


def _scatter_ref(full, part, idx):
    B, S, H = full.shape
    flat = (idx.long() + torch.arange(B, device=full.device)[:, None] * S).reshape(-1)
    return full.reshape(B * S, H).index_copy(0, flat, part.reshape(-1, H)).view(B, S, H)


def _native_ok(x):
    return native.use_native(x) and x.shape[-1] % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16,
                                                                         torch.float16)


def gather_rows(x, idx):
    """[B, S, H], [B, R] -> [B, R, H] (no autograd)."""
    if not _native_ok(x):
        return _gather_ref(x, idx)
    x = x.contiguous()
    idx = idx.to(torch.int32).contiguous()
    B, S, H = x.shape
    R = idx.shape[1]
    assert idx.shape[0] == B
    out = torch.empty(B, R, H, dtype=x.dtype, device=x.device)
    native.check(native.kernels().hds_token_gather(native.dt(x), x.data_ptr(), idx.data_ptr(), out.data_ptr(), B, S,
                                                    R, H, native.stream()), "token_gather")
    return out


def scatter_rows(full, part, idx):
    """Copy of ``full`` [B, S, H] with rows ``idx`` replaced by ``part`` [B, R, H] (no autograd)."""
    if not _native_ok(full):
        return _scatter_ref(full, part, idx)
    out = full.contiguous().clone()
    part = part.to(full.dtype).contiguous()
    idx = idx.to(torch.int32).contiguous()
    B, S, H = out.shape
    R = idx.shape[1]
    assert part.shape == (B, R, H)
    native.check(native.kernels().hds_token_scatter(native.dt(out), part.data_ptr(), idx.data_ptr(), out.data_ptr(),
                                                     B, S, R, H, native.stream()), "token_scatter")
    return out


class GatherTokens(torch.autograd.Function):
    """(activations, sorted_indices, batch_first) -> (activations, gathered); backward scatters the gathered grad."""

    @staticmethod
    def forward(ctx, activations, sorted_indices, batch_first=True):
        x = activations if batch_first else activations.transpose(0, 1)
        ctx.save_for_backward(sorted_indices)
        ctx.batch_first = batch_first
        ctx.S = x.shape[1]
        g = gather_rows(x, sorted_indices)
        return activations, (g if batch_first else g.transpose(0, 1).contiguous())

    @staticmethod
    def backward(ctx, g_act, g_gathered):
        idx, = ctx.saved_tensors
        if g_gathered is None:
            return g_act, None, None
        gg = g_gathered if ctx.batch_first else g_gathered.transpose(0, 1)
        base = g_act if g_act is not None else gg.new_zeros(gg.shape[0], ctx.S, gg.shape[2]) if ctx.batch_first \
            else gg.new_zeros(ctx.S, gg.shape[0], gg.shape[2])
        b = base if ctx.batch_first else base.transpose(0, 1)
        # accumulate: rows at idx get base + gathered grad
        add = gather_rows(b, idx) + gg
        out = scatter_rows(b, add, idx)
        return (out if ctx.batch_first else out.transpose(0, 1)), None, None


class ScatterTokens(torch.autograd.Function):
    """(all_activations, layer_activations, sorted_indices, batch_first) -> scattered."""

    @staticmethod
    def forward(ctx, all_activations, layer_activations, sorted_indices, batch_first=True):
        full = all_activations if batch_first else all_activations.transpose(0, 1)
        part = layer_activations if batch_first else layer_activations.transpose(0, 1)
        ctx.save_for_backward(sorted_indices)
        ctx.batch_first = batch_first
        out = scatter_rows(full, part, sorted_indices)
        return out if batch_first else out.transpose(0, 1).contiguous()

    @staticmethod
    def backward(ctx, g):
        idx, = ctx.saved_tensors
        gb = g if ctx.batch_first else g.transpose(0, 1)
        g_part = gather_rows(gb, idx)
        g_full = scatter_rows(gb, torch.zeros_like(g_part), idx)
        if not ctx.batch_first:
            g_part, g_full = g_part.transpose(0, 1), g_full.transpose(0, 1)
        return g_full, g_part, None, None


def slice_attention_mask(mask, idx):
    """mask [Bm, 1 or none, S, S] (Bm in {1, B}), idx [L, B, R] or [B, R] -> [L, B, 1, R, R] / [B, 1, R, R]."""
    squeeze_l = idx.dim() == 2
    if squeeze_l:
        idx = idx[None]
    L, B, R = idx.shape
    m = mask.reshape(-1, mask.shape[-2], mask.shape[-1])
    Bm, S = m.shape[0], m.shape[-1]
    if native.use_native(m) and m.dtype in (torch.float32, torch.bfloat16, torch.float16):
        m = m.contiguous()
        ix = idx.to(torch.int32).contiguous()
        out = torch.empty(L, B, R, R, dtype=m.dtype, device=m.device)
        native.check(native.kernels().hds_slice_mask(native.dt(m), m.data_ptr(), ix.data_ptr(), out.data_ptr(), L,
                                                      B, Bm, S, R, native.stream()), "slice_mask")
    else:
        il = idx.long()
        bsel = torch.arange(B, device=m.device) if Bm == B else torch.zeros(B, dtype=torch.long, device=m.device)
        out = m[bsel[None, :, None, None], il[:, :, :, None], il[:, :, None, :]]
    out = out.unsqueeze(2)
    return out[0] if squeeze_l else out


def slice_gpt_mask(mask, reserved_length):
    """Causal masks stay causal over sorted indices: the reserved mask is the top-left [R, R] block."""
    return mask[..., :reserved_length, :reserved_length].contiguous()


def bert_sample_tokens(reserved_length, seq_length, batch_size, layers=1, device="cpu", attn_mask=None,
                       generator=None):
    """Sorted random token indices [layers, B, R] plus the per-layer sliced padding masks."""
    scores = torch.rand(layers * batch_size, seq_length, device=device, generator=generator)
    idx = scores.topk(reserved_length, dim=1).indices.to(torch.int32).contiguous()
    token_sort_(idx)
    idx = idx.view(layers, batch_size, reserved_length)
    masks = None
    if attn_mask is not None:
        masks = slice_attention_mask(attn_mask, idx)
    return idx, masks
