"""Rotary embeddings: host-built cos/sin tables + in-place HIP rotation (fwd and inverse).

Reference parity: ``apply_rotary_pos_emb`` (csrc/transformer/inference/csrc/apply_rotary_pos_emb.cu,
ops/transformer/inference/op_binding) and the rotary part of ``kv_rotary_pos_kernel``
(inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary). Supports Llama-3 frequency scaling
(rope_type="llama3") and linear scaling.
"""
import math

import torch

from . import native

_CACHE = {}


def rope_inv_freq(rot_dim, base=10000.0, scaling=None):
    inv = 1.0 / (base**(torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
    if scaling:
        kind = scaling.get("rope_type", scaling.get("type", "default"))
        if kind == "linear":
            inv = inv / float(scaling["factor"])
        elif kind == "llama3":
            factor = float(scaling.get("factor", 8.0))
            lo = float(scaling.get("low_freq_factor", 1.0))
            hi = float(scaling.get("high_freq_factor", 4.0))
            old = float(scaling.get("original_max_position_embeddings", 8192))
            lo_wl, hi_wl = old / lo, old / hi
            wl = 2 * math.pi / inv
            smooth = (old / wl - lo) / (hi - lo)
            scaled = torch.where(wl > lo_wl, inv / factor, inv)
            mid = (wl <= lo_wl) & (wl >= hi_wl)
            inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    return inv


def rope_tables(max_pos, rot_dim, base=10000.0, scaling=None, device="cpu"):
    """fp32 cos/sin tables [max_pos, rot_dim // 2] (cached per device/config)."""
    key = (int(max_pos), int(rot_dim), float(base), repr(sorted((scaling or {}).items())), str(device))
    t = _CACHE.get(key)
    if t is None:
        inv = rope_inv_freq(rot_dim, base, scaling)
        pos = torch.arange(max_pos, dtype=torch.float64)
        ang = torch.outer(pos, inv)
        t = (ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device))
        _CACHE[key] = t
    return t


def _ref_rope_(x, cos, sin, n_rot, rot_dim, pos, sign, interleaved):
    # x: [T, nh, D] view (modified in place)
    half = rot_dim // 2
    c = cos[pos][:, None, :]
    s = sin[pos][:, None, :] * sign
    xr = x[:, :n_rot, :rot_dim].float()
    if not interleaved:
        a, b = xr[..., :half], xr[..., half:]
        out = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    else:
        a, b = xr[..., 0::2], xr[..., 1::2]
        out = torch.stack([a * c - b * s, b * c + a * s], dim=-1).flatten(-2)
    x[:, :n_rot, :rot_dim] = out.to(x.dtype)


def rope_(x, cos, sin, n_rot_heads, seq_len=None, pos_ids=None, rot_dim=None, sign=1.0, interleaved=False,
          pos_offset=0):
    """Rotate the first ``n_rot_heads`` heads of ``x`` ([T, n_heads, D], head dim contiguous) in place.

    Positions: ``pos_ids`` (int32 [T]) or ``t % seq_len + pos_offset``. ``sign=-1`` applies the inverse
    rotation (used by backward).
    """
    T, nh, D = x.shape
    rot_dim = rot_dim or D
    assert x.stride(2) == 1 and x.stride(1) == D, "rope_: head dim must be contiguous"
    if seq_len is None:
        seq_len = T
    if native.use_native(x):
        lib = native.kernels()
        pid = pos_ids.to(torch.int32).contiguous() if pos_ids is not None else None
        native.check(
            lib.hds_rope(native.dt(x), int(interleaved), x.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                         native.ptr(pid), T, n_rot_heads, D, rot_dim, x.stride(0), int(seq_len), int(pos_offset),
                         float(sign), native.stream()), "rope")
    else:
        if pos_ids is not None:
            pos = pos_ids.long()
        else:
            pos = torch.arange(T, device=x.device) % seq_len + pos_offset
        _ref_rope_(x, cos, sin, n_rot_heads, rot_dim, pos, sign, interleaved)
    return x


class _RopeFn(torch.autograd.Function):

    @staticmethod
    def forward(ctx, x, cos, sin, seq_len, pos_ids, interleaved):
        y = x.contiguous().clone()
        rope_(y, cos, sin, y.shape[1], seq_len, pos_ids, sign=1.0, interleaved=interleaved)
        ctx.save_for_backward(cos, sin, pos_ids)
        ctx.seq_len, ctx.interleaved = seq_len, interleaved
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin, pos_ids = ctx.saved_tensors
        dx = dy.contiguous().clone()
        rope_(dx, cos, sin, dx.shape[1], ctx.seq_len, pos_ids, sign=-1.0, interleaved=ctx.interleaved)
        return dx, None, None, None, None, None


def apply_rotary(x, cos, sin, seq_len=None, pos_ids=None, interleaved=False):
    """Out-of-place autograd RoPE on [T, nh, D]."""
    return _RopeFn.apply(x, cos, sin, seq_len if seq_len is not None else x.shape[0], pos_ids, interleaved)
