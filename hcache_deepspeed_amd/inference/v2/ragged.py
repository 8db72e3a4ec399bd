"""Ragged-batch state for serving: block allocator, sequence descriptors, paged KV cache, batch builder.

Reference parity: inference/v2/ragged/ -- ``BlockedAllocator`` (blocked_allocator.py:11),
``DSSequenceDescriptor`` (sequence_descriptor.py:59), ``BlockedKVCache`` (kv_cache.py:60, shape
(num_layers, num_blocks, block_size, 2, n_kv_heads, head_size) :134, sized from free memory with a MIN
all-reduce over TP :83-122), ``DSStateManager`` (ragged_manager.py:55), ``RaggedBatchWrapper``
(ragged_wrapper.py:31; host shadows flushed with non_blocking copies in ``finalize`` :184-218).

MI355X sizing: the KV pool is carved out of the 288 GB HBM after weights (``memory_config.mode``
"reserve" keeps ``size`` bytes free, "allocate" takes exactly ``size`` bytes). Host metadata lives in
pinned buffers so ``finalize`` is one async H2D copy.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ... import comm as dist


# -----------------------------------------------------------------------------------------------
# config
# -----------------------------------------------------------------------------------------------
@dataclass
class MemoryConfig:
    mode: str = "reserve"  # reserve | allocate
    size: int = 1_000_000_000  # bytes kept free (reserve) or used for KV (allocate)


@dataclass
class DSStateManagerConfig:
    max_tracked_sequences: int = 2048
    max_ragged_batch_size: int = 768
    max_ragged_sequence_count: int = 512
    max_context: int = 8192
    memory_config: MemoryConfig = field(default_factory=MemoryConfig)
    offload: bool = False
    kv_block_size: int = 64

    @staticmethod
    def from_dict(d):
        d = dict(d or {})
        mc = d.pop("memory_config", None)
        cfg = DSStateManagerConfig(**{k: v for k, v in d.items() if k in DSStateManagerConfig.__dataclass_fields__})
        if mc is not None:
            cfg.memory_config = mc if isinstance(mc, MemoryConfig) else MemoryConfig(**mc)
        return cfg


# -----------------------------------------------------------------------------------------------
# allocator
# -----------------------------------------------------------------------------------------------
class BlockedAllocator:
    """Free-list allocator over ``num_blocks`` KV blocks (LIFO reuse keeps hot blocks in cache)."""

    def __init__(self, num_blocks):
        if num_blocks < 1:
            raise ValueError("num_blocks must be >= 1")
        self._num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))
        self._allocated = set()

    @property
    def free_blocks(self):
        return len(self._free)

    @property
    def num_blocks(self):
        return self._num_blocks

    def allocate(self, num_blocks):
        if num_blocks > len(self._free):
            raise ValueError(f"Not enough free blocks in the KV-cache to allocate {num_blocks} blocks "
                             f"({len(self._free)} free)")
        out = [self._free.pop() for _ in range(num_blocks)]
        self._allocated.update(out)
        return torch.tensor(out, dtype=torch.int32)

    def free(self, blocks):
        blocks = blocks.tolist() if isinstance(blocks, torch.Tensor) else list(blocks)
        for b in blocks:
            if b not in self._allocated:
                raise ValueError(f"block {b} is not allocated")
            self._allocated.remove(b)
            self._free.append(b)


# -----------------------------------------------------------------------------------------------
# sequence descriptor
# -----------------------------------------------------------------------------------------------
class DSSequenceDescriptor:

    def __init__(self, uid, tracking_id, max_blocks):
        self.uid = uid
        self.tracking_id = tracking_id
        self.seen_tokens = 0
        self.in_flight_tokens = 0
        self._blocks: List[int] = []
        self.max_blocks = max_blocks

    @property
    def cur_allocated_blocks(self):
        return len(self._blocks)

    @property
    def kv_blocks(self):
        return list(self._blocks)

    def extend_kv_cache(self, new_blocks):
        self._blocks.extend(int(b) for b in (new_blocks.tolist() if isinstance(new_blocks, torch.Tensor) else
                                              new_blocks))

    def free_kv_cache(self):
        b, self._blocks = self._blocks, []
        return b

    def pre_forward(self, num_tokens):
        self.in_flight_tokens = num_tokens

    def post_forward(self):
        self.seen_tokens += self.in_flight_tokens
        self.in_flight_tokens = 0

    def __repr__(self):
        return f"DSSequenceDescriptor(uid={self.uid}, seen={self.seen_tokens}, blocks={len(self._blocks)})"


# -----------------------------------------------------------------------------------------------
# KV cache
# -----------------------------------------------------------------------------------------------
class BlockedKVCache:
    """Per-layer paged K/V storage: ``cache[layer]`` is [num_blocks, block_size, 2, n_kv_heads, head_dim]."""

    def __init__(self, num_layers, n_kv_heads, head_dim, block_size, dtype, device, memory_config, tp_group=None,
                 num_blocks=None):
        self.num_layers, self.n_kv_heads, self.head_dim, self.block_size = num_layers, n_kv_heads, head_dim, block_size
        per_block = num_layers * block_size * 2 * n_kv_heads * head_dim * torch.tensor([], dtype=dtype).element_size()
        if num_blocks is None:
            if device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(device)
                if memory_config.mode == "reserve":
                    budget = max(0, free - memory_config.size)
                else:
                    budget = min(free, memory_config.size)
            else:
                budget = memory_config.size if memory_config.mode == "allocate" else 256 * 2**20
            num_blocks = max(1, budget // per_block)
            if tp_group is not None and dist.get_world_size(tp_group) > 1:
                t = torch.tensor([num_blocks], device=device if device.type == "cuda" else "cpu")
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=tp_group)
                num_blocks = int(t.item())
        self.num_blocks = int(num_blocks)
        self.cache = torch.zeros(num_layers, self.num_blocks, block_size, 2, n_kv_heads, head_dim, dtype=dtype,
                                 device=device)

    def get_cache(self, layer):
        return self.cache[layer]

    def offload(self, blocks):
        raise NotImplementedError("use the HCache latent path (put() -> latents, restore_kv()) to move KV off-GPU")


# -----------------------------------------------------------------------------------------------
# state manager
# -----------------------------------------------------------------------------------------------
class DSStateManager:

    def __init__(self, config: DSStateManagerConfig, kv_cache: BlockedKVCache):
        self._config = config
        self.kv_cache = kv_cache
        self._allocator = BlockedAllocator(kv_cache.num_blocks)
        self._seqs: Dict[int, DSSequenceDescriptor] = {}
        self._free_tracking = list(range(config.max_tracked_sequences - 1, -1, -1))
        self.max_blocks_per_seq = (config.max_context + kv_cache.block_size - 1) // kv_cache.block_size

    @property
    def free_blocks(self):
        return self._allocator.free_blocks

    @property
    def n_tracked_sequences(self):
        return len(self._seqs)

    @property
    def tracked_sequences(self):
        return self._seqs

    def get_sequence(self, uid) -> Optional[DSSequenceDescriptor]:
        return self._seqs.get(uid)

    def get_or_create_sequence(self, uid):
        s = self._seqs.get(uid)
        if s is None:
            if not self._free_tracking:
                raise RuntimeError("max_tracked_sequences exceeded")
            s = DSSequenceDescriptor(uid, self._free_tracking.pop(), self.max_blocks_per_seq)
            self._seqs[uid] = s
        return s

    def blocks_needed(self, seq: DSSequenceDescriptor, n_new_tokens):
        total = seq.seen_tokens + n_new_tokens
        need = (total + self.kv_cache.block_size - 1) // self.kv_cache.block_size
        return max(0, need - seq.cur_allocated_blocks)

    def allocate_blocks(self, n):
        return self._allocator.allocate(n)

    def maybe_allocate_kv(self, seq, n_new_tokens):
        n = self.blocks_needed(seq, n_new_tokens)
        if n:
            seq.extend_kv_cache(self._allocator.allocate(n))

    def free_kv(self, seq):
        blocks = seq.free_kv_cache()
        if blocks:
            self._allocator.free(blocks)

    def flush_sequence(self, uid):
        s = self._seqs.pop(uid, None)
        if s is None:
            return
        self.free_kv(s)
        self._free_tracking.append(s.tracking_id)


# -----------------------------------------------------------------------------------------------
# ragged batch
# -----------------------------------------------------------------------------------------------
class RaggedBatchWrapper:
    """Host-built batch metadata; ``finalize`` ships it to the device in one async copy each."""

    def __init__(self, config: DSStateManagerConfig, device, max_blocks_per_seq):
        self._config = config
        self.device = device
        self.max_blocks = max_blocks_per_seq
        self.clear()

    def clear(self):
        self._seqs: List[DSSequenceDescriptor] = []
        self._tokens: List[torch.Tensor] = []
        self.seq_meta_host = []  # (q_start, n_new, seen)
        self.current_tokens = 0

    @property
    def current_sequences(self):
        return len(self._seqs)

    def insert_sequence(self, seq: DSSequenceDescriptor, tokens: torch.Tensor, do_checks=True):
        n = int(tokens.numel())
        if do_checks:
            if self.current_tokens + n > self._config.max_ragged_batch_size:
                raise RuntimeError("ragged batch token budget exceeded")
            if len(self._seqs) + 1 > self._config.max_ragged_sequence_count:
                raise RuntimeError("ragged batch sequence budget exceeded")
        self.seq_meta_host.append((self.current_tokens, n, seq.seen_tokens))
        self._seqs.append(seq)
        self._tokens.append(tokens.reshape(-1).to(torch.int64))
        self.current_tokens += n

    def set_attention_geometry(self, n_q, n_kv, rows_per_atom):
        """Lets ``finalize`` also build the paged-attention work atoms (the model's query/KV head counts)."""
        self._geom = (int(n_q), int(n_kv), int(rows_per_atom))

    def _pinned_slot(self, need):
        """One of two rotating pinned int32 staging buffers; a slot is reused only after its H2D drained."""
        slots = self.__dict__.setdefault("_slots", [None, None])
        evs = self.__dict__.setdefault("_slot_events", [None, None])
        i = self.__dict__.get("_slot_next", 0)
        self._slot_next = i ^ 1
        if evs[i] is not None:
            evs[i].synchronize()
        if slots[i] is None or slots[i].numel() < need:
            slots[i] = torch.empty(max(need, 4096), dtype=torch.int32, pin_memory=self.device.type == "cuda")
        return i, slots[i]

    def finalize(self):
        """Ship the batch description to the device: the native builder (csrc/host/ragged_meta.cpp) writes seq_meta,
        token -> sequence / position maps, last-token rows, the KV block table and the attention atoms into ONE
        pinned int32 buffer, sent with one async H2D copy into a persistent device buffer (plus one for the token
        ids); the device tensors below are views of it."""
        import ctypes
        import numpy as np
        from ...ops import native
        S, T = len(self._seqs), self.current_tokens
        mb = self.max_blocks
        n_new = np.fromiter((nn for (_, nn, _) in self.seq_meta_host), dtype=np.int32, count=S)
        seen = np.fromiter((sn for (_, _, sn) in self.seq_meta_host), dtype=np.int32, count=S)
        blk_lists = [seq.kv_blocks for seq in self._seqs]
        off = np.zeros(S + 1, dtype=np.int64)
        if S:
            off[1:] = np.cumsum([len(b) for b in blk_lists])
        flat = np.fromiter((b for bl in blk_lists for b in bl), dtype=np.int32, count=int(off[-1]))
        n_q, n_kv, rpa = getattr(self, "_geom", (1, 1, 1 << 30))
        lib = native.host_lib()
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        need = ctypes.c_int64(0)
        lib.hds_ragged_meta_build(P(n_new), P(seen), S, P(flat), P(off), mb, n_q, n_kv, rpa, None, 0,
                                  ctypes.byref(need))
        si, host = self._pinned_slot(int(need.value))
        A = lib.hds_ragged_meta_build(P(n_new), P(seen), S, P(flat), P(off), mb, n_q, n_kv, rpa,
                                      ctypes.c_void_p(host.data_ptr()), host.numel(), ctypes.byref(need))
        if A < 0:
            raise RuntimeError(f"ragged metadata builder failed ({A})")
        n = int(need.value)
        dev_buf = self.__dict__.get("_dev_meta")
        if dev_buf is None or dev_buf.numel() < n:
            dev_buf = self._dev_meta = torch.empty(max(n, 4096), dtype=torch.int32, device=self.device)
        dev_buf[:n].copy_(host[:n], non_blocking=True)
        ids = torch.cat(self._tokens) if self._tokens else torch.zeros(0, dtype=torch.int64)
        if self.device.type == "cuda":
            ids = ids.pin_memory()
            ev = torch.cuda.Event()
            ev.record()
            self._slot_events[si] = ev
        self.input_ids = ids.to(self.device, non_blocking=True)
        o = 0

        def take(k, shape):
            nonlocal o
            v = dev_buf[o:o + k].view(*shape)
            o += k
            return v

        self.seq_meta = take(3 * S, (S, 3))
        self.tok_seq = take(T, (T, ))
        self.tok_pos = take(T, (T, ))
        self.last_token_idx = take(S, (S, ))
        self.block_tables = take(S * mb, (S, mb))
        self.atoms = take(3 * A, (A, 3)) if hasattr(self, "_geom") else None
        self.n_atoms = int(A) if hasattr(self, "_geom") else None
        self.tables_host = host[4 * S + 2 * T:4 * S + 2 * T + S * mb].view(S, mb).clone() if S else \
            torch.zeros(1, mb, dtype=torch.int32)
        if S == 0:  # keep 1-row shapes for empty batches (kernels never run on them)
            self.seq_meta = torch.zeros(1, 3, dtype=torch.int32, device=self.device)
            self.block_tables = torch.zeros(1, mb, dtype=torch.int32, device=self.device)
            self.last_token_idx = torch.zeros(1, dtype=torch.int32, device=self.device)

    @property
    def sequences(self):
        return self._seqs

    # reference-compatible host shadow of the in-flight descriptors: [start_idx, n_tokens, seen_tokens, pad]
    @property
    def _inflight_seq_descriptors_shadow(self):
        return [(q0, nn, seen, 0) for (q0, nn, seen) in self.seq_meta_host]
