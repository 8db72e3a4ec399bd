"""Batched gradient collectives: one reduce-scatter for a list of tensors, and hierarchical quantized
reduce-scatter (ZeRO++ qgZ) with optional LoCo error feedback.

Reference parity: deepspeed/runtime/comm/coalesced_collectives.py — ``reduce_scatter_coalesced`` (:158-218),
``all_to_all_quant_reduce`` (:31-76), ``all_to_all_loco_quant_reduce`` (:81-153). Semantics kept: every function
returns, per input tensor, THIS rank's 1/world partition of the AVERAGE over ranks (flattened, ceil-partitioned
for ``reduce_scatter_coalesced``).

MI355X design (not a translation):
* ``reduce_scatter_coalesced`` packs all tensors into ONE rank-major ``[world, sum(padded_chunk)]`` buffer with a
  single allocation and one strided copy per tensor (no per-chunk ``torch.cat`` list), then issues ONE
  ``reduce_scatter_tensor`` — one RCCL ring over xGMI instead of one launch per tensor.
* qgZ is two all-to-alls: intra-node over the 8 xGMI-connected GPUs with int4 payloads, then inter-node between
  the GPUs that share a local index. The "swizzle" is a view permutation ``[N, L, c] -> [L, N, c]`` of the
  destination-major chunk layout; the intra-node reduction is the fused HIP dequant-reduce kernel
  (``ops/quantizer.dequant_reduce``, csrc/kernels/quant.hip) which sums the L received int4 copies straight into
  fp32 — no per-peer dequantized temporaries.
* On a single node the inter-node stage disappears (one all-to-all); groups are created by
  :func:`create_qgz_groups`.
"""
import math
from typing import Dict, List, Optional

import torch

from ... import comm as dist
from ...utils.logging import logger


def _quant_group(n):
    for g in (2048, 1024, 512, 256, 128, 64, 32, 16, 8):
        if n % g == 0:
            return g
    return 0


@torch.no_grad()
def reduce_scatter_coalesced(tensors: List[torch.Tensor], group=None) -> List[torch.Tensor]:
    """Average-reduce-scatter a list of tensors with one collective. Returns views of this rank's partition of
    each (flattened) tensor; the last rank's partition of a tensor whose numel is not divisible by world is
    shorter (its padding is dropped)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    chunks = [math.ceil(t.numel() / world) for t in tensors]
    if len(tensors) == 1 and tensors[0].numel() % world == 0 and tensors[0].is_contiguous():
        buf = tensors[0].detach().view(world, chunks[0]).clone()
    else:
        dtype = tensors[0].dtype
        buf = torch.zeros(world, sum(chunks), dtype=dtype, device=tensors[0].device)
        off = 0
        for t, c in zip(tensors, chunks):
            flat = t.detach().reshape(-1)
            full = flat.numel() // c
            if full:
                buf[:full, off:off + c].copy_(flat[:full * c].view(full, c))
            rem = flat.numel() - full * c
            if rem:
                buf[full, off:off + rem].copy_(flat[full * c:])
            off += c
    buf.div_(world)
    out = torch.empty(buf.shape[1], dtype=buf.dtype, device=buf.device)
    dist.reduce_scatter_tensor(out, buf.view(-1), group=group)
    res, off = [], 0
    for t, c in zip(tensors, chunks):
        valid = max(0, min(c, t.numel() - rank * c))
        res.append(out.narrow(0, off, valid))
        off += c
    return res


def create_qgz_groups(local_world_size: Optional[int] = None) -> Dict[str, object]:
    """Process groups for hierarchical qgZ: ``local_{node}`` (the GPUs of one node) and ``global_{local_idx}``
    (one GPU per node with the same local index). Collective over all ranks (every rank creates every group)."""
    world = dist.get_world_size()
    L = local_world_size or int(__import__("os").environ.get("LOCAL_WORLD_SIZE", world))
    L = max(1, min(L, world))
    assert world % L == 0, f"world {world} not divisible by local world {L}"
    N = world // L
    groups = {}
    for node in range(N):
        groups[f"local_{node}"] = dist.new_group(list(range(node * L, (node + 1) * L)))
    for li in range(L):
        groups[f"global_{li}"] = dist.new_group([node * L + li for node in range(N)])
    groups["_L"], groups["_N"] = L, N
    return groups


def _a2a_quant_stage(payload: torch.Tensor, peers: int, group, bits: int, G: int) -> torch.Tensor:
    """payload [peers, c] (destination-major, fp32) -> sum over senders of what they sent to this rank, [c]."""
    from ...ops import quantizer as Q
    c = payload.shape[1]
    if peers == 1:
        return payload.reshape(c).clone()
    q, sc, _ = Q.quantize(payload.reshape(-1), G, bits, True)
    qr, sr = torch.empty_like(q), torch.empty_like(sc)
    dist.all_to_all_single(qr, q, group=group)
    dist.all_to_all_single(sr, sc, group=group)
    return Q.dequant_reduce(qr, sr, peers, c, G, bits, dtype=torch.float32)


def _layout(groups, world):
    if groups and "_L" in groups:
        L, N = groups["_L"], groups["_N"]
    else:
        L, N = world, 1
    rank = dist.get_rank()
    node, li = rank // L, rank % L
    lg = groups.get(f"local_{node}") if groups else None
    gg = groups.get(f"global_{li}") if groups else None
    return L, N, lg, gg


@torch.no_grad()
def all_to_all_quant_reduce(tensors: List[torch.Tensor], groups: Optional[Dict[str, object]] = None,
                            bits: int = 4) -> List[torch.Tensor]:
    """qgZ: per tensor, this rank's 1/world partition of the rank-average, communicated as int4 (or int8).
    Tensors whose per-rank chunk cannot be grouped for the quantizer (or 1-D tensors, as in the reference) fall
    back to :func:`reduce_scatter_coalesced`."""
    world = dist.get_world_size()
    L, N, lg, gg = _layout(groups, world)
    out = []
    for t in tensors:
        n = t.numel()
        c = n // world if n % world == 0 else 0
        G = _quant_group(c) if c else 0
        if t.dim() == 1 or not G or world == 1:
            if t.dim() != 1 and world > 1:
                logger.warning(f"qgZ falls back to reduce_scatter: numel {n} does not split into quantizer groups "
                               f"over world {world}")
            out.append(reduce_scatter_coalesced([t])[0])
            continue
        # destination-major chunks [N, L, c]; intra-node stage sends [L, N, c] (peer j gets chunks (*, j))
        x = t.detach().reshape(N, L, c).float()
        part = _a2a_quant_stage(x.transpose(0, 1).contiguous().view(L, N * c), L, lg, bits, _quant_group(N * c))
        # part [N*c]: node-local sum of chunks (node', my_li); inter-node stage sends chunk node' to node'
        tot = _a2a_quant_stage(part.view(N, c), N, gg, bits, G)
        out.append(tot.div_(world).to(t.dtype))
    return out


@torch.no_grad()
def all_to_all_loco_quant_reduce(params: List[torch.Tensor], groups: Optional[Dict[str, object]] = None,
                                 loco_param: Optional[dict] = None, bits: int = 4) -> List[torch.Tensor]:
    """qgZ with LoCo error feedback (reference :81-153): each stage quantizes ``x + beta * err`` and keeps the
    compression residual as the next step's error (stored int8-quantized on the parameter, as the reference does,
    so the feedback state costs 1 byte/element). ``reset_T`` steps after a reset the errors restart from zero."""
    from ...ops import quantizer as Q
    loco_param = loco_param or {}
    beta = float(loco_param.get("err_beta", 0.8))
    reset_T = int(loco_param.get("reset_T", 1024))
    world = dist.get_world_size()
    L, N, lg, gg = _layout(groups, world)
    out = []
    for p in params:
        t = p.grad
        n = t.numel()
        c = n // world if n % world == 0 else 0
        G = _quant_group(c) if c else 0
        if t.dim() == 1 or not G or world == 1:
            out.append(reduce_scatter_coalesced([t])[0])
            continue
        G1 = _quant_group(N * c)
        step = getattr(p, "_loco_step", reset_T + 1)
        if step > reset_T or not hasattr(p, "_loco_intra"):
            intra_err = torch.zeros(n, dtype=torch.float32, device=t.device)
            inter_err = torch.zeros(N * c, dtype=torch.float32, device=t.device)
            step = 0
        else:
            intra_err = Q.dequantize(*p._loco_intra, group_size=G1, bits=8, dtype=torch.float32)
            inter_err = Q.dequantize(*p._loco_inter, group_size=G, bits=8, dtype=torch.float32)
        x = t.detach().reshape(N, L, c).float().transpose(0, 1).reshape(-1) + beta * intra_err
        if L > 1:
            q, sc, _ = Q.quantize(x, G1, bits, True)
            intra_err = x - Q.dequantize(q, sc, None, G1, bits, True, torch.float32)
            qr, sr = torch.empty_like(q), torch.empty_like(sc)
            dist.all_to_all_single(qr, q, group=lg)
            dist.all_to_all_single(sr, sc, group=lg)
            part = Q.dequant_reduce(qr, sr, L, N * c, G1, bits, dtype=torch.float32)
        else:
            intra_err = torch.zeros_like(x)
            part = x.clone()
        part = part + beta * inter_err
        if N > 1:
            q, sc, _ = Q.quantize(part, G, bits, True)
            inter_err = part - Q.dequantize(q, sc, None, G, bits, True, torch.float32)
            qr, sr = torch.empty_like(q), torch.empty_like(sc)
            dist.all_to_all_single(qr, q, group=gg)
            dist.all_to_all_single(sr, sc, group=gg)
            tot = Q.dequant_reduce(qr, sr, N, c, G, bits, dtype=torch.float32)
        else:
            inter_err = torch.zeros_like(part)
            tot = part
        qi, si, _ = Q.quantize(intra_err, G1, 8, True)
        qe, se, _ = Q.quantize(inter_err, G, 8, True)
        p._loco_intra, p._loco_inter = (qi, si), (qe, se)
        p._loco_step = step + 1
        out.append(tot.div_(world).to(t.dtype))
    return out
