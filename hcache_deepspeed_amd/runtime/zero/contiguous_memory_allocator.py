"""Defragmenting contiguous allocator for ZeRO-3 parameter storage (reference runtime/zero/
contiguous_memory_allocator.py :16).

One pre-allocated flat buffer; ``allocate_tensor(size)`` returns a view into it, moving (compacting) live tensors
when free space is fragmented; parameters assigned with ``assign_to_param`` follow their tensor across moves.
The flat-shard ZeRO of this framework mostly avoids fragmentation by construction (rank-major unit buffers);
this allocator keeps the reference API for user code and for the offload staging pools.
"""
import torch


class ContiguousMemoryAllocator:

    def __init__(self, size, dtype, device):
        self.buffer = torch.zeros(size, dtype=dtype, device=device)
        self.contiguous_sizes = {0: size}  # address -> free block size
        self.tensor_addresses = {}  # tensor id -> address
        self.tensor_sizes = {}  # tensor id -> size
        self.tensor_ids = {}  # address -> tensor id
        self.tensor_map = {}  # tensor id -> tensor view
        self.id_to_params = {}  # tensor id -> [(param, numel, shape)]
        self.total_size = size
        self.total_free = size
        self.largest_contiguous = size
        self._max_allocated = 0
        self.count = 0

    def allocate_tensor(self, size):
        assert size <= self.total_free, "not enough memory in the contiguous buffer"
        if self.largest_contiguous < size:
            self._defragment_memory()
        self._reset_param_data()
        self.total_free -= size
        address = self._get_new_tensor_address(size)
        self._mark_as_occupied(address, size)
        tid = self.count
        self.count += 1
        t = self.buffer.narrow(0, address, size)
        self.tensor_addresses[tid] = address
        self.tensor_sizes[tid] = size
        self.tensor_ids[address] = tid
        self.tensor_map[tid] = t
        t._hds_alloc_id = tid
        self._max_allocated = max(self._max_allocated, self.total_size - self.total_free)
        return t

    def assign_to_param(self, tensor, param, numel, shape):
        tid = tensor._hds_alloc_id
        assert tid in self.tensor_map, "tensor was not allocated by this allocator"
        assert tensor.numel() >= numel
        self.id_to_params.setdefault(tid, []).append((param, numel, shape))
        param.data = tensor.narrow(0, 0, numel).view(shape)

    def release_tensor(self, tensor):
        self.release_tensor_with_id(tensor._hds_alloc_id)

    def release_tensor_with_id(self, tensor_id):
        assert tensor_id in self.tensor_map, f"tensor id {tensor_id} not allocated"
        size = self.tensor_sizes[tensor_id]
        self._release_tensor(tensor_id)
        self.total_free += size
        self._unassign_params(tensor_id)

    def max_allocated(self):
        return self._max_allocated

    def print_allocation(self, resolution=200):
        total = self.buffer.numel()
        empty = ["."] * resolution
        for tid, addr in self.tensor_addresses.items():
            lo = addr * resolution // total
            hi = (addr + self.tensor_sizes[tid]) * resolution // total
            for i in range(lo, max(lo + 1, hi)):
                empty[min(i, resolution - 1)] = "|"
        print("".join(empty))

    # -- internals ----------------------------------------------------------------------------
    def _reset_param_data(self):
        for tid, params in self.id_to_params.items():
            t = self.tensor_map[tid]
            for p, numel, shape in params:
                p.data = t.narrow(0, 0, numel).view(shape)

    def _unassign_params(self, tensor_id):
        self.id_to_params.pop(tensor_id, None)

    def _release_tensor(self, tensor_id):
        address = self.tensor_addresses.pop(tensor_id)
        size = self.tensor_sizes.pop(tensor_id)
        self.tensor_ids.pop(address)
        self.tensor_map.pop(tensor_id)
        self._consolidate_address(address, size)

    def _consolidate_address(self, address, size):
        end = address + size
        if end in self.contiguous_sizes:
            size += self.contiguous_sizes.pop(end)
        for a, s in list(self.contiguous_sizes.items()):
            if a + s == address:
                self.contiguous_sizes.pop(a)
                address, size = a, s + size
                break
        self.contiguous_sizes[address] = size
        self.largest_contiguous = max(self.contiguous_sizes.values(), default=0)

    def _defragment_memory(self):
        """Slide every live tensor to the front of the buffer (in address order) and rebind views/params."""
        cursor = 0
        for address in sorted(self.tensor_ids):
            tid = self.tensor_ids[address]
            size = self.tensor_sizes[tid]
            if address != cursor:
                self.buffer.narrow(0, cursor, size).copy_(self.buffer.narrow(0, address, size).clone())
                self._replace_old_address_with_new(tid, cursor)
            cursor += size
        self.tensor_ids = {self.tensor_addresses[t]: t for t in self.tensor_addresses}
        self.contiguous_sizes = {cursor: self.total_size - cursor} if cursor < self.total_size else {}
        self.largest_contiguous = self.total_size - cursor

    def _replace_old_address_with_new(self, tensor_id, new_address):
        size = self.tensor_sizes[tensor_id]
        t = self.buffer.narrow(0, new_address, size)
        t._hds_alloc_id = tensor_id
        self.tensor_addresses[tensor_id] = new_address
        self.tensor_map[tensor_id] = t
        for p, numel, shape in self.id_to_params.get(tensor_id, []):
            p.data = t.narrow(0, 0, numel).view(shape)

    def _get_new_tensor_address(self, size):
        best = None
        for a, s in self.contiguous_sizes.items():
            if s >= size and (best is None or s < self.contiguous_sizes[best]):
                best = a  # best fit
        assert best is not None, "no contiguous block large enough after defragmentation"
        return best

    def _mark_as_occupied(self, address, size):
        free = self.contiguous_sizes.pop(address)
        if free > size:
            self.contiguous_sizes[address + size] = free - size
        self.largest_contiguous = max(self.contiguous_sizes.values(), default=0)
