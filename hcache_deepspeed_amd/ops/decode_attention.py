"""Decode (single new token) attention over HF-style KV caches ``[B, Hkv, S, D]``
(csrc/kernels/decode_attn.hip; reference ds_softmax_context / KV-cache attention).

GQA is served without ``repeat_interleave`` copies; an additive per-key bias (padding masks) and ALiBi slopes
(BLOOM-style models) are applied in the kernel. CPU tensors / unsupported head dims use the torch reference.
"""
import math

import torch
import torch.nn.functional as F

from . import native


def decode_attention_ref(q, k, v, scale, bias=None, alibi=None):
    """q [B, H, D], k/v [B, Hkv, S, D], bias [B, S] additive, alibi [H] -> o [B, H, D] (fp32 math)."""
    B, H, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    G = H // Hkv
    kk = k.float().repeat_interleave(G, 1)
    vv = v.float().repeat_interleave(G, 1)
    s = torch.einsum("bhd,bhsd->bhs", q.float(), kk) * scale
    if bias is not None:
        s = s + bias.float()[:, None, :]
    if alibi is not None:
        s = s + alibi.float()[None, :, None] * (torch.arange(S, device=q.device) - (S - 1)).float()[None, None, :]
    return torch.einsum("bhs,bhsd->bhd", torch.softmax(s, -1), vv).to(q.dtype)


def decode_supported(q, k):
    if not (native.use_native(q) and q.dtype == torch.bfloat16 and k.dtype == torch.bfloat16):
        return False
    B, H, D = q.shape
    return bool(native.kernels().hds_decode_attn_supported(D, H // k.shape[1])) and H % k.shape[1] == 0


def decode_attention(q, k, v, scale=None, bias=None, alibi=None, lens=None, window=0):
    """q [B, H, D] (any head/batch strides, last dim contiguous), k/v [B, Hkv, S, D] (last dim contiguous).

    ``lens`` (int32 [B] on the device): only the first lens[b] cache slots are keys (and, with ``window`` > 0,
    only the last ``window`` of those). The launch shape then depends on the buffer size S alone, so a decode
    step that calls this can be captured once in a HIP graph and replayed for every token."""
    B, H, D = q.shape
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if not decode_supported(q, k) or q.stride(2) != 1 or k.stride(3) != 1 or v.stride(3) != 1:
        if lens is not None:  # reference path: mask the slots past each sequence's length (and outside the window)
            j = torch.arange(k.shape[2], device=q.device)[None, :]
            n = lens.to(torch.long)[:, None]
            off = (j >= n) | ((j < n - window) if window > 0 else torch.zeros_like(j, dtype=torch.bool))
            extra = torch.zeros(off.shape, device=q.device, dtype=torch.float32).masked_fill_(off, float("-inf"))
            bias = extra if bias is None else bias.float() + extra
        return decode_attention_ref(q, k, v, scale, bias, alibi)
    Hkv, S = k.shape[1], k.shape[2]
    kern = native.kernels()
    splits = kern.hds_decode_attn_splits(B, Hkv, S)
    o = torch.empty(B, H, D, device=q.device, dtype=q.dtype)
    part_o = part_ml = None
    if splits > 1:
        part_o = torch.empty(B, H, splits, D, device=q.device, dtype=torch.float32)
        part_ml = torch.empty(B, H, splits, 2, device=q.device, dtype=torch.float32)
    if bias is not None:
        bias = bias.float()
        if bias.stride(-1) != 1:
            bias = bias.contiguous()
    if alibi is not None:
        alibi = alibi.float().contiguous()
    if lens is not None:
        assert lens.dtype == torch.int32 and lens.numel() == B and lens.is_contiguous()
    native.check(kern.hds_decode_attn_len(q.data_ptr(), q.stride(0), q.stride(1), k.data_ptr(), k.stride(0), k.stride(1),
                                      k.stride(2), v.data_ptr(), v.stride(0), v.stride(1), v.stride(2),
                                      bias.data_ptr() if bias is not None else None,
                                      bias.stride(0) if bias is not None else 0,
                                      alibi.data_ptr() if alibi is not None else None, o.data_ptr(),
                                      part_o.data_ptr() if part_o is not None else None,
                                      part_ml.data_ptr() if part_ml is not None else None, B, H, Hkv, S, D, splits,
                                      float(scale), lens.data_ptr() if lens is not None else None, int(window),
                                      native.stream()), "decode_attn")
    return o


def sdpa_gqa(q, k, v, mask=None, is_causal=False, scale=None):
    """[B, H, Sq, D] x [B, Hkv, Skv, D] attention without materialising repeated K/V."""
    return F.scaled_dot_product_attention(q, k, v, attn_mask=mask, is_causal=is_causal, scale=scale,
                                          enable_gqa=k.shape[1] != q.shape[1])


def kv_append(k, v, kc, vc, cur_idx):
    """kc[:, :, cur] = k ; vc[:, :, cur] = v for k/v [B, Hkv, D] (last dim contiguous) and caches [B, Hkv, S, D], with
    the slot ``cur_idx`` (int64 [1]) read on the device: one HIP launch, capturable in the decode graph."""
    B, H, D = k.shape
    if not (native.use_native(k) and k.dtype == torch.bfloat16 and kc.dtype == torch.bfloat16 and D % 8 == 0
            and k.stride(2) == 1 and v.stride(2) == 1 and kc.stride(3) == 1 and vc.stride(3) == 1
            and cur_idx.dtype == torch.int64 and k.data_ptr() % 16 == 0 and v.data_ptr() % 16 == 0
            and all(st % 8 == 0 for st in (k.stride(0), k.stride(1), v.stride(0), v.stride(1)))):
        kc.index_copy_(2, cur_idx, k.reshape(B, H, 1, D))
        vc.index_copy_(2, cur_idx, v.reshape(B, H, 1, D))
        return
    native.check(native.kernels().hds_kv_append(k.data_ptr(), k.stride(0), k.stride(1), v.data_ptr(), v.stride(0),
                                                v.stride(1), kc.data_ptr(), kc.stride(0), kc.stride(1), kc.stride(2),
                                                vc.data_ptr(), vc.stride(0), vc.stride(1), vc.stride(2),
                                                cur_idx.data_ptr(), B, H, D, native.stream()), "kv_append")
