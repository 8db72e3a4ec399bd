"""Shared-memory all-reduce among the ranks of one host (CPU tensors).

Reference parity: csrc/cpu/comm/shm.cpp / shm_interface.cpp and comm/torch.py:160-165 (``inference_all_reduce``
routed to ``torch.ops.deepspeed.inference_all_reduce_`` when the SHM op is built). Backed here by
csrc/host/shm_comm.cpp; :func:`hcache_deepspeed_amd.comm.inference_all_reduce` uses it for CPU fp32 / bf16
tensors when every rank of the group is on this host, and falls back to the process-group all-reduce otherwise.
"""
import os

import torch
import torch.distributed as tdist

from ..ops import native

_DT = {torch.float32: 0, torch.bfloat16: 1}
_comms = {}


class ShmAllReduce:

    def __init__(self, group=None, slot_bytes=16 << 20):
        self.group = group
        self.rank = tdist.get_rank(group)
        self.world = tdist.get_world_size(group)
        gid = "w" if group is None else "g" + "_".join(str(r) for r in tdist.get_process_group_ranks(group))
        port = os.environ.get("MASTER_PORT", "0")
        # unique per job (master port + rank-0 pid) and per group
        tag = torch.tensor([os.getpid() if self.rank == 0 else 0], dtype=torch.int64)
        tdist.broadcast(tag, tdist.get_global_rank(group, 0) if group is not None else 0, group=group)
        self.name = f"/hds_shm_{port}_{int(tag.item())}_{gid}"
        lib = native.host_lib()
        self._lib = lib
        self.h = lib.hds_shm_open(self.name.encode(), self.rank, self.world, int(slot_bytes), 1) \
            if self.rank == 0 else None
        tdist.barrier(group=group)
        if self.rank != 0:
            self.h = lib.hds_shm_open(self.name.encode(), self.rank, self.world, int(slot_bytes), 0)
        ok = torch.tensor([1 if self.h else 0])
        tdist.all_reduce(ok, group=group)
        if int(ok.item()) != self.world:
            raise RuntimeError(f"shared-memory segment {self.name} could not be opened on every rank")
        self.slot_bytes = int(lib.hds_shm_slot_bytes(self.h))
        tdist.barrier(group=group)
        if self.rank == 0:  # every rank has it mapped: the name can go, the mapping stays valid
            import ctypes
            ctypes.CDLL(None).shm_unlink(self.name.encode())

    def all_reduce_(self, t):
        """In-place SUM of a contiguous CPU fp32 / bf16 tensor (chunked through the segment)."""
        assert t.device.type == "cpu" and t.is_contiguous() and t.dtype in _DT
        es = t.element_size()
        per = self.slot_bytes // es
        flat = t.view(-1)
        for i in range(0, flat.numel(), per):
            chunk = flat[i:i + per]
            if self._lib.hds_shm_allreduce(self.h, chunk.data_ptr(), chunk.numel(), _DT[t.dtype]) != 0:
                raise RuntimeError("shared-memory all-reduce failed")
        return t

    def close(self):
        if self.h:
            self._lib.hds_shm_close(self.h, 0)
            self.h = None


def _same_host(group):
    local = int(os.environ.get("LOCAL_SIZE", os.environ.get("LOCAL_WORLD_SIZE", "0")) or 0)
    world = tdist.get_world_size()
    return local == world and world > 1


def get_shm_comm(group=None):
    key = id(group) if group is not None else None
    if key not in _comms:
        _comms[key] = ShmAllReduce(group)
    return _comms[key]


def shm_eligible(t, group=None):
    return (t.device.type == "cpu" and t.dtype in _DT and t.is_contiguous() and tdist.is_initialized()
            and tdist.get_world_size(group) > 1 and _same_host(group)
            and os.environ.get("HDS_SHM_ALLREDUCE", "1") == "1")
