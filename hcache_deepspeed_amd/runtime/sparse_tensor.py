"""Sparse (row-indexed) gradient tensor for embedding gradients (reference runtime/sparse_tensor.py :13).

Data-parallel reduction of sparse embedding gradients all-gathers (indices, values) instead of all-reducing the
dense [V, H] tensor (the engine's ``sparse_gradients`` option, reference engine.py:2683-2750)."""
import torch


class SparseTensor:

    def __init__(self, dense_tensor=None):
        self.orig_dense_tensor = dense_tensor
        self.is_sparse = dense_tensor is not None and dense_tensor.is_sparse
        if dense_tensor is not None:
            if dense_tensor.is_sparse:
                if dense_tensor.sparse_dim() != 1:  # row-sparse (hybrid) form: [nnz_rows] indices, [nnz_rows, H]
                    dense_tensor = dense_tensor.to_dense().to_sparse(1)
                dense_tensor = dense_tensor.coalesce()
                self.indices = dense_tensor.indices().flatten()
                self.values = dense_tensor.values()
            else:
                rows = dense_tensor.abs().sum(dim=1)
                self.indices = rows.nonzero().flatten()
                self.values = dense_tensor[self.indices]
            self.dense_size = list(dense_tensor.size())
        else:
            self.indices = None
            self.values = None
            self.dense_size = None

    def to_coo_tensor(self):
        return torch.sparse_coo_tensor(self.indices.unsqueeze(0), self.values, self.dense_size)

    @staticmethod
    def type():
        return "deepspeed.SparseTensor"

    def to_dense(self):
        full = self.indices.unsqueeze(1).expand(-1, self.dense_size[1])
        return self.values.new_zeros(self.dense_size).scatter_add_(0, full, self.values)

    def sparse_size(self):
        return self.indices.numel() + self.values.numel(), self.dense_size[0] * self.dense_size[1]

    def add(self, b):
        assert self.dense_size == b.dense_size
        self.indices = torch.cat([self.indices, b.indices])
        self.values = torch.cat([self.values, b.values])

    def __str__(self):
        s, d = self.sparse_size()
        return (f"DeepSpeed.SparseTensor(indices_size={tuple(self.indices.size())}, "
                f"values_size={tuple(self.values.size())}, dense_size={self.dense_size}, "
                f"device={self.indices.device}, reduction_factor={d / max(1, s)})")

    __repr__ = __str__


def all_reduce_sparse(sparse, group=None, average=True):
    """DP reduction of a :class:`SparseTensor`: all-gather variable-length (indices, values) and concatenate
    (duplicates are summed by ``to_dense``)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([sparse.indices.numel()], device=sparse.indices.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(int(s.item()) for s in sizes))
    idx = sparse.indices.new_zeros(mx)
    idx[:int(n.item())] = sparse.indices
    val = sparse.values.new_zeros(mx, sparse.values.shape[1])
    val[:int(n.item())] = sparse.values
    gi = [torch.zeros_like(idx) for _ in range(world)]
    gv = [torch.zeros_like(val) for _ in range(world)]
    dist.all_gather(gi, idx, group=group)
    dist.all_gather(gv, val, group=group)
    out = SparseTensor()
    out.dense_size = sparse.dense_size
    out.indices = torch.cat([g[:int(s.item())] for g, s in zip(gi, sizes)])
    out.values = torch.cat([g[:int(s.item())] for g, s in zip(gv, sizes)])
    if average:
        out.values = out.values / world
    return out
