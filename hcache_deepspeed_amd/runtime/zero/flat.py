"""Flat-shard building blocks shared by every ZeRO stage.

A :class:`FlatUnit` is a set of parameters laid out back to back in ONE flat buffer of
``padded`` elements, ``padded = world * shard`` (``shard`` a multiple of ``ALIGN``). The buffer is
rank-major: rank r owns elements ``[r*shard, (r+1)*shard)``. Consequences:

* parameter gather = one ``all_gather_into_tensor(full, my_shard)``; every parameter is then a
  *view* into ``full`` -- no per-parameter unshuffle copy (reference partition_parameters.py:695-714);
* gradient reduction = one ``reduce_scatter_tensor(my_grad_shard, grad_full)`` where the parameters'
  ``.grad`` are views into ``grad_full`` -- no interleave/pad copy (coalesced_collectives.py:186-199);
* the optimizer sees each rank's shards of ALL units concatenated in one flat fp32 buffer
  (:class:`ShardStore`), so the whole Adam step is a handful of fused kernel launches.

Unit granularity: ZeRO-3 uses one unit per transformer block (every element of an
``nn.ModuleList``) plus one root unit for the remaining parameters; ZeRO-0/1/2 use fixed-size buckets
in registration order (size tuned for xGMI: several MB per peer per collective).
"""
import math

import torch

ALIGN = 64  # elements per rank shard alignment (128 B for bf16, 256 B for fp32 master)

NOT_AVAILABLE, INFLIGHT, AVAILABLE = 0, 1, 2


class ZeroParamStatus:
    NOT_AVAILABLE = NOT_AVAILABLE
    INFLIGHT = INFLIGHT
    AVAILABLE = AVAILABLE


def _round_up(x, m):
    return (x + m - 1) // m * m


class Segment:
    """A contiguous range of one rank's shard owned by a single optimizer param group."""
    __slots__ = ("group", "store_off", "numel")

    def __init__(self, group, store_off, numel):
        self.group, self.store_off, self.numel = group, store_off, numel


class FlatUnit:

    def __init__(self, uid, params, groups, world, rank, name=""):
        self.uid = uid
        self.name = name
        # order parameters by optimizer group so each rank's shard crosses few group boundaries
        order = sorted(range(len(params)), key=lambda i: groups[i])
        self.params = [params[i] for i in order]
        self.param_groups = [groups[i] for i in order]
        self.shapes = [p.ds_shape if hasattr(p, "ds_shape") else p.shape for p in self.params]
        self.numels = [int(math.prod(s)) for s in self.shapes]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += _round_up(n, 8)  # 16-byte aligned parameter starts (vector loads in kernels)
        self.numel = off
        self.world, self.rank = world, rank
        self.shard = _round_up(max(1, math.ceil(self.numel / world)), ALIGN)
        self.padded = self.shard * world
        self.store_off = None  # offset of this rank's shard inside the ShardStore
        self.full = None  # gathered parameter buffer [padded]
        self.grad_full = None  # gradient buffer [padded] (params' .grad are views)
        self.status = NOT_AVAILABLE
        self.work = None
        self.persistent = False  # never released (root unit during a step, or ZeRO-0/1/2)
        self.pending = 0  # params whose grad has not been accumulated yet in this backward
        self.grads_reduced = False
        self.requires_grad_count = sum(1 for p in self.params if p.requires_grad)
        self.segments = []
        self.module = None

    # group segments of MY shard: which [lo, hi) ranges of my shard belong to which group
    def my_group_ranges(self):
        lo = self.rank * self.shard
        hi = lo + self.shard
        ranges = []
        for p_off, n, g in zip(self.offsets, self.numels, self.param_groups):
            a, b = max(lo, p_off), min(hi, p_off + _round_up(n, 8))
            if a < b:
                if ranges and ranges[-1][2] == g and ranges[-1][1] == a - lo:
                    ranges[-1][1] = b - lo
                else:
                    ranges.append([a - lo, b - lo, g])
        if not ranges:
            ranges.append([0, self.shard, self.param_groups[0] if self.param_groups else 0])
        # extend first/last range over padding gaps so the whole shard is covered
        ranges[0][0] = 0
        for i in range(1, len(ranges)):
            ranges[i][0] = ranges[i - 1][1]
        ranges[-1][1] = self.shard
        return ranges

    def param_view(self, buf, i):
        return buf[self.offsets[i]:self.offsets[i] + self.numels[i]].view(self.shapes[i])

    def bind_params(self, full):
        for i, p in enumerate(self.params):
            p.data = self.param_view(full, i)

    def bind_grads(self, grad_full):
        for i, p in enumerate(self.params):
            if p.requires_grad:
                p.grad = self.param_view(grad_full, i)

    def unbind_params(self, empty):
        for p in self.params:
            p.data = empty

    def unbind_grads(self):
        for p in self.params:
            p.grad = None

    def copy_params_into(self, full):
        """Pack the current (materialised) parameter values into a full flat buffer."""
        full.zero_()
        for i, p in enumerate(self.params):
            full[self.offsets[i]:self.offsets[i] + self.numels[i]].copy_(p.data.reshape(-1))


class ShardStore:
    """Concatenation of this rank's shards of every unit: lp (compute dtype), fp32 master, grads, states."""

    def __init__(self, units, dtype, device, grad_dtype, master=True, lp_host=False):
        total = 0
        for u in units:
            u.store_off = total
            total += u.shard
        self.numel = total
        self.device = device
        if lp_host == "nvme":
            # ZeRO-Infinity NVMe tier: the shard lives in the parameter swap file (runtime/swap_tensor)
            self.lp = torch.empty(0, dtype=dtype)
        elif lp_host:
            # ZeRO-Infinity parameter offload: the compute-dtype shard lives in pinned host memory
            pin = torch.cuda.is_available()
            self.lp = torch.zeros(total, dtype=dtype, device="cpu", pin_memory=pin)
        else:
            self.lp = torch.zeros(total, dtype=dtype, device=device)
        self.grad = torch.zeros(total, dtype=grad_dtype, device=device)
        self.master = None
        self.states = {}
        self.segments = []  # merged Segments over the whole store
        for u in units:
            for lo, hi, g in u.my_group_ranges():
                so = u.store_off + lo
                if self.segments and self.segments[-1].group == g and \
                        self.segments[-1].store_off + self.segments[-1].numel == so:
                    self.segments[-1].numel += hi - lo
                else:
                    self.segments.append(Segment(g, so, hi - lo))

    def lp_slice(self, u):
        return self.lp[u.store_off:u.store_off + u.shard]

    def grad_slice(self, u):
        return self.grad[u.store_off:u.store_off + u.shard]

    def seg(self, buf, s):
        return buf[s.store_off:s.store_off + s.numel]
