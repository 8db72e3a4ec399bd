"""Error-compensated 1-bit all-reduce (sign + scale) for 1-bit Adam / 0-1 Adam / 1-bit LAMB.

Reference parity: runtime/comm/nccl.py ``NcclBackend.compressed_allreduce`` (:16-166), runtime/comm/compressed.py
(packbits), runtime/comm/mpi.py. Two-phase scheme: every rank sends the packed signs of chunk r of its
(error-compensated) buffer to rank r in ONE all-to-all (1/32 of the fp32 bytes), rank r averages the
``world`` scaled sign chunks into its server chunk (with server error feedback), and one all-gather
returns every server chunk's packed signs + scale. Worker and server errors carry the compression
residual into the next step, so the time-average is unbiased.
"""
import math

import torch

from ... import comm as dist

_BITS = None


def _bit_weights(device):
    global _BITS
    if _BITS is None or _BITS.device != device:
        _BITS = (2**torch.arange(8, device=device, dtype=torch.int32)).to(torch.uint8)
    return _BITS


def pack_signs(x):
    """bool/float tensor (numel % 8 == 0) -> uint8 [numel/8] with bit i = (x[8k+i] >= 0)."""
    b = (x >= 0) if x.dtype != torch.bool else x
    b = b.view(-1, 8).to(torch.uint8)
    return (b * _bit_weights(b.device)).sum(1, dtype=torch.int32).to(torch.uint8)


def unpack_signs(p, dtype=torch.float32):
    """uint8 [n] -> +-1 tensor [8n]."""
    bits = (p.view(-1, 1).to(torch.int32) >> torch.arange(8, device=p.device, dtype=torch.int32)) & 1
    return (bits.to(dtype) * 2 - 1).view(-1)


def padded_size(numel, world):
    return int(math.ceil(numel / (8 * world))) * 8 * world


def compressed_allreduce(buf, worker_error, server_error, group=None):
    """In place: ``buf`` (fp32, numel = padded_size) <- approx. mean over ranks of ``buf``.
    ``worker_error`` [numel], ``server_error`` [numel / world] are updated (error feedback)."""
    world = dist.get_world_size(group)
    n = buf.numel()
    assert n % (8 * world) == 0, "pad the buffer with padded_size()"
    chunk = n // world
    buf.add_(worker_error)
    wscale = buf.norm() / math.sqrt(n)
    sign = buf >= 0
    worker_error.copy_(buf - wscale * (sign.to(buf.dtype) * 2 - 1))
    if world == 1:
        # single rank: the "server" stage still applies (keeps the algorithm identical)
        srv = wscale * (sign.to(buf.dtype) * 2 - 1) + server_error
        sscale = srv.norm() / math.sqrt(n)
        ssign = srv >= 0
        server_error.copy_(srv - sscale * (ssign.to(buf.dtype) * 2 - 1))
        buf.copy_(sscale * (ssign.to(buf.dtype) * 2 - 1))
        return buf
    packed = pack_signs(sign)  # [n/8], chunk r at [r*chunk/8, (r+1)*chunk/8)
    recv = torch.empty_like(packed)
    dist.all_to_all_single(recv, packed, group=group)
    scales = torch.empty(world, dtype=buf.dtype, device=buf.device)
    dist.all_gather_into_tensor(scales, wscale.reshape(1).to(buf.dtype), group=group)
    signs = unpack_signs(recv, buf.dtype).view(world, chunk)
    srv = (signs * scales.view(world, 1)).mean(0) + server_error
    sscale = srv.norm() / math.sqrt(chunk)
    ssign = srv >= 0
    server_error.copy_(srv - sscale * (ssign.to(buf.dtype) * 2 - 1))
    spacked = pack_signs(ssign)
    all_packed = torch.empty(world * spacked.numel(), dtype=torch.uint8, device=buf.device)
    dist.all_gather_into_tensor(all_packed, spacked, group=group)
    sscales = torch.empty(world, dtype=buf.dtype, device=buf.device)
    dist.all_gather_into_tensor(sscales, sscale.reshape(1).to(buf.dtype), group=group)
    out = unpack_signs(all_packed, buf.dtype).view(world, chunk) * sscales.view(world, 1)
    buf.copy_(out.view(-1))
    return buf


class CompressedBackend:
    """Reference-style backend object (``NcclBackend``/``MpiBackend``): holds the group."""

    def __init__(self, group=None):
        self.group = group
        self.size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def compressed_allreduce(self, buffer_m, worker_error, server_error, local_rank=None):
        return compressed_allreduce(buffer_m, worker_error, server_error, self.group)
