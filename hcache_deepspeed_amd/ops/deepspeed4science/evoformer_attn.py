"""Evoformer attention with pair bias (AlphaFold / OpenFold MSA row- and triangle-attention).

Reference parity: ops/deepspeed4science/evoformer_attn.py (``DS4Sci_EvoformerAttention(Q, K, V, biases)`` :88,
``EvoformerFusedAttention`` autograd :59 with bias gradients) backed there by CUTLASS memory-efficient attention
(csrc/deepspeed4science/evoformer_attn, 14.9k LoC).

Shapes: Q/K/V ``[B, N, L, H, D]``; ``bias1 = [B, N, 1, 1, L]`` (MSA mask, broadcast over heads and queries);
``bias2 = [B, 1, H, L, L]`` (pair bias, broadcast over the N rows). Output ``[B, N, L, H, D]``.

Forward on the GPU (bf16, head_dim 32/64/128): the HIP kernel csrc/kernels/evoformer.hip (MFMA 32x32x16 flash
attention with both biases fused, emits the LSE). Backward on the GPU: the FlashAttention dK/dV and dQ kernels
(csrc/kernels/flash_attn.hip, ``EVO`` instantiations) with the biases folded into the recomputed P and the bias
gradients reduced by fp32 atomics. Elsewhere: a memory-efficient flash-style
decomposition -- the forward keeps only the fp32 log-sum-exp per
query, the backward recomputes the probabilities one query chunk at a time, so peak memory is O(chunk x L)
instead of O(L^2) per (B, N, H). The per-chunk products run as batched GEMMs on the matrix cores; head_dim is
arbitrary (Evoformer uses 16-64, below the 128 the FlashAttention HIP kernel is tiled for). Bias gradients
are reduced exactly as the reference (dB2 summed over N, dB1 over heads and queries).
"""
import math

import torch

_CHUNK_BYTES = 256 << 20


def _chunk_rows(B, N, H, L):
    per_row = max(1, B * N * H * L * 4)
    return max(16, min(L, _CHUNK_BYTES // per_row))


def _scores(q, k, b1, b2, i0, i1, scale):
    s = torch.matmul(q[..., i0:i1, :], k.transpose(-1, -2)).float() * scale  # [B, N, H, c, L]
    if b1 is not None:
        s = s + b1.float()  # [B, N, 1, 1, L]
    if b2 is not None:
        s = s + b2[..., i0:i1, :].float()  # [B, 1, H, c, L]
    return s


def _hip_eligible(q, k, v, b1, b2):
    from .. import native
    if not native.use_native(q):
        return False
    ok_b = all(b is None or (b.dtype in (torch.bfloat16, torch.float32) and b.is_contiguous()) for b in (b1, b2))
    same_b = b1 is None or b2 is None or b1.dtype == b2.dtype
    return (q.dtype == k.dtype == v.dtype == torch.bfloat16 and q.shape[-1] in (32, 64, 128) and ok_b and same_b
            and all(x.is_contiguous() for x in (q, k, v)))


def _hip_forward(q, k, v, b1, b2, scale):
    """HIP forward (csrc/kernels/evoformer.hip): O [B, N, L, H, D] and the natural-log LSE [B, N, H, L]."""
    from .. import native
    B, N, L, H, D = q.shape
    o = torch.empty_like(q)
    lse = torch.empty(B, N, H, L, dtype=torch.float32, device=q.device)
    bdt = (b1 if b1 is not None else b2)
    bdt = native.dt(bdt) if bdt is not None else 1
    native.check(native.kernels().hds_evoformer_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), native.ptr(b1),
                                                    native.ptr(b2), bdt, o.data_ptr(), lse.data_ptr(), B, N, L, H,
                                                    D, float(scale), native.stream()), "evoformer_fwd")
    return o, lse


def _hip_backward(ctx, do, qh, kh, vh, oh, lse, bias1, bias2, scale):
    """HIP backward: the FlashAttention dK/dV and dQ kernels with both biases folded into P (flash_attn.hip
    ``hds_evoformer_bwd``); dB2 is summed over the N rows and dB1 over heads/queries by fp32 atomics."""
    from .. import native
    B, N, H, L, D = qh.shape
    q, k, v, o = (x.transpose(-2, -3) for x in (qh, kh, vh, oh))  # back to the contiguous [B, N, L, H, D]
    do = do.contiguous()
    lse_t = lse.permute(2, 0, 1, 3).reshape(H, B * N * L).contiguous()  # [H][tokens]
    delta = torch.empty(H, B * N * L, dtype=torch.float32, device=q.device)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    want_b1 = bias1 is not None and ctx.needs_input_grad[3]
    want_b2 = bias2 is not None and ctx.needs_input_grad[4]
    db1 = torch.zeros(B * N, L, dtype=torch.float32, device=q.device) if want_b1 else None
    db2 = torch.zeros(B, H, L, L, dtype=torch.float32, device=q.device) if want_b2 else None
    bias_f32 = int((bias1 if bias1 is not None else bias2) is not None and
                   (bias1 if bias1 is not None else bias2).dtype == torch.float32)
    native.check(native.kernels().hds_evoformer_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                                    lse_t.data_ptr(), do.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                                    dv.data_ptr(), delta.data_ptr(), native.ptr(bias1),
                                                    native.ptr(bias2), bias_f32, native.ptr(db1), native.ptr(db2), B,
                                                    N, L, H, D, float(scale), native.stream()), "evoformer_bwd")
    g1 = db1.view(B, N, 1, 1, L).to(bias1.dtype) if want_b1 else None
    g2 = db2.view(B, 1, H, L, L).to(bias2.dtype) if want_b2 else None
    return dq, dk, dv, g1, g2


class EvoformerFusedAttention(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, bias1=None, bias2=None):
        # [B, N, L, H, D] -> [B, N, H, L, D]
        qh, kh, vh = (x.transpose(-2, -3) for x in (q, k, v))
        B, N, H, L, D = qh.shape
        scale = 1.0 / math.sqrt(D)
        if _hip_eligible(q, k, v, bias1, bias2):
            o, lse = _hip_forward(q, k, v, bias1, bias2, scale)
            ctx.save_for_backward(qh, kh, vh, o.transpose(-2, -3), lse, bias1, bias2)
            ctx.scale = scale
            ctx.hip = True
            return o
        o = torch.empty(qh.shape, dtype=q.dtype, device=q.device)
        lse = torch.empty(B, N, H, L, dtype=torch.float32, device=q.device)
        c = _chunk_rows(B, N, H, L)
        for i0 in range(0, L, c):
            i1 = min(L, i0 + c)
            s = _scores(qh, kh, bias1, bias2, i0, i1, scale)
            m = torch.logsumexp(s, -1)
            lse[..., i0:i1] = m
            p = torch.exp(s - m[..., None])
            o[..., i0:i1, :] = torch.matmul(p.to(v.dtype), vh)
        ctx.save_for_backward(qh, kh, vh, o, lse, bias1, bias2)
        ctx.scale = scale
        return o.transpose(-2, -3)

    @staticmethod
    def backward(ctx, do):
        qh, kh, vh, o, lse, bias1, bias2 = ctx.saved_tensors
        scale = ctx.scale
        B, N, H, L, D = qh.shape
        if getattr(ctx, "hip", False):
            return _hip_backward(ctx, do, qh, kh, vh, o, lse, bias1, bias2, scale)
        doh = do.transpose(-2, -3)
        delta = (doh.float() * o.float()).sum(-1)  # [B, N, H, L]
        dq = torch.empty(qh.shape, dtype=torch.float32, device=qh.device)
        dk = torch.zeros(kh.shape, dtype=torch.float32, device=qh.device)
        dv = torch.zeros(vh.shape, dtype=torch.float32, device=qh.device)
        want_b1 = bias1 is not None and ctx.needs_input_grad[3]
        want_b2 = bias2 is not None and ctx.needs_input_grad[4]
        db1 = torch.zeros(bias1.shape, dtype=torch.float32, device=qh.device) if want_b1 else None
        db2 = torch.zeros(bias2.shape, dtype=torch.float32, device=qh.device) if want_b2 else None
        c = _chunk_rows(B, N, H, L)
        for i0 in range(0, L, c):
            i1 = min(L, i0 + c)
            p = torch.exp(_scores(qh, kh, bias1, bias2, i0, i1, scale) - lse[..., i0:i1, None])  # [B,N,H,c,L]
            dob = doh[..., i0:i1, :]
            dv += torch.matmul(p.transpose(-1, -2).to(vh.dtype), dob).float()
            dp = torch.matmul(dob, vh.transpose(-1, -2)).float()
            ds = p * (dp - delta[..., i0:i1, None])  # gradient wrt the biased scores
            if want_b2:
                db2[..., i0:i1, :] += ds.sum(1, keepdim=True)
            if want_b1:
                db1 += ds.sum((2, 3), keepdim=True)
            dsq = ds.to(qh.dtype)
            dq[..., i0:i1, :] = torch.matmul(dsq, kh).float() * scale
            dk += torch.matmul(dsq.transpose(-1, -2), qh[..., i0:i1, :]).float() * scale
        out = [x.to(qh.dtype).transpose(-2, -3) for x in (dq, dk, dv)]
        return (out[0], out[1], out[2], db1.to(bias1.dtype) if want_b1 else None,
                db2.to(bias2.dtype) if want_b2 else None)


def DS4Sci_EvoformerAttention(Q, K, V, biases):
    """Q/K/V ``[B, N, L, H, D]``; ``biases``: up to two of ``[B, N, 1, 1, L]`` and ``[B, 1, H, L, L]``."""
    biases = list(biases)
    assert len(biases) <= 2
    while len(biases) < 2:
        biases.append(None)
    if biases[0] is not None:
        assert biases[0].shape == (Q.shape[0], Q.shape[1], 1, 1, Q.shape[2]), "bias1 shape is incorrect"
    if biases[1] is not None:
        assert biases[1].shape == (Q.shape[0], 1, Q.shape[3], Q.shape[2], Q.shape[2]), "bias2 shape is incorrect"
    return EvoformerFusedAttention.apply(Q, K, V, biases[0], biases[1])
