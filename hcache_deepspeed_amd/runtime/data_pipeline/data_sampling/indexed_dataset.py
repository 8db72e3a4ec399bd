"""Memory-mapped indexed datasets (the ``.bin`` / ``.idx`` pair of Megatron-style corpora).

Reference parity: deepspeed/runtime/data_pipeline/data_sampling/indexed_dataset.py (``MMapIndexedDataset`` :369,
``MMapIndexedDatasetBuilder``, ``make_builder`` / ``make_dataset``). The on-disk format is the same, so corpora and
data-analyzer outputs written by either framework read in the other:

``<prefix>.idx``: magic ``MMIDIDX\\0\\0``, u64 version (1), u8 dtype code, u64 item count N, u64 document count D,
then int32 sizes[N], int64 byte pointers[N] (exclusive scan of sizes * itemsize), int64 doc_idx[D].
``<prefix>.bin``: the items' elements back to back.

Reads are zero-copy ``np.frombuffer`` views over one ``np.memmap`` per file; the builder streams items straight to
the ``.bin`` file and keeps only the sizes in memory.
"""
import os
import shutil
import struct

import numpy as np
import torch

_MAGIC = b"MMIDIDX\x00\x00"

# dtype code table of the reference's data-sampling indexed dataset
DTYPES = {
    1: np.uint8,
    2: np.int8,
    3: np.int16,
    4: np.int32,
    5: np.int64,
    6: np.uint16,
    7: np.uint32,
    8: np.uint64,
}
_TORCH = {torch.uint8: np.uint8, torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32,
          torch.int64: np.int64}


def _np_dtype(dtype):
    if isinstance(dtype, torch.dtype):
        if dtype not in _TORCH:
            raise ValueError(f"{dtype} not supported by indexed datasets")
        return np.dtype(_TORCH[dtype])
    return np.dtype(dtype)


def code(dtype):
    dt = _np_dtype(dtype)
    for c, npdt in DTYPES.items():
        if np.dtype(npdt) == dt:
            return c
    raise ValueError(f"{dtype} not supported; use one of {sorted(np.dtype(d).name for d in DTYPES.values())}")


def index_file_path(prefix):
    return prefix + ".idx"


def data_file_path(prefix):
    return prefix + ".bin"


def best_fitting_dtype(vocab_size=None):
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def _pointers(sizes, itemsize):
    sizes = np.asarray(sizes, dtype=np.int64)
    ptr = np.zeros(len(sizes), dtype=np.int64)
    if len(sizes) > 1:
        np.cumsum(sizes[:-1] * itemsize, out=ptr[1:])
    return ptr


def write_index(path, dtype, sizes, doc_idx):
    with open(path, "wb") as f:
        f.write(_MAGIC)
        f.write(struct.pack("<Q", 1))
        f.write(struct.pack("<B", code(dtype)))
        f.write(struct.pack("<Q", len(sizes)))
        f.write(struct.pack("<Q", len(doc_idx)))
        f.write(np.asarray(sizes, dtype=np.int32).tobytes(order="C"))
        f.write(_pointers(sizes, _np_dtype(dtype).itemsize).tobytes(order="C"))
        f.write(np.asarray(doc_idx, dtype=np.int64).tobytes(order="C"))


class MMapIndexedDataset(torch.utils.data.Dataset):
    """Read-only view of ``<prefix>.bin`` / ``<prefix>.idx``; ``ds[i]`` is a numpy array (a slice is a list)."""

    def __init__(self, path, skip_warmup=True):
        super().__init__()
        self._path = path
        self._open()

    def _open(self):
        idx = index_file_path(self._path)
        with open(idx, "rb") as f:
            if f.read(9) != _MAGIC:
                raise ValueError(f"{idx}: not an MMIDIDX index file")
            (version, ) = struct.unpack("<Q", f.read(8))
            if version != 1:
                raise ValueError(f"{idx}: unsupported index version {version}")
            (dcode, ) = struct.unpack("<B", f.read(1))
            self._dtype = np.dtype(DTYPES[dcode])
            (n, ) = struct.unpack("<Q", f.read(8))
            (d, ) = struct.unpack("<Q", f.read(8))
            off = f.tell()
        self._idx_map = np.memmap(idx, mode="r", order="C")
        buf = memoryview(self._idx_map)
        self._sizes = np.frombuffer(buf, dtype=np.int32, count=n, offset=off)
        self._ptrs = np.frombuffer(buf, dtype=np.int64, count=n, offset=off + 4 * n)
        self._doc_idx = np.frombuffer(buf, dtype=np.int64, count=d, offset=off + 12 * n)
        binp = data_file_path(self._path)
        self._bin_map = np.memmap(binp, mode="r", order="C") if os.path.getsize(binp) > 0 else np.zeros(0, np.uint8)
        self._bin = memoryview(self._bin_map)

    def __getstate__(self):
        return self._path

    def __setstate__(self, path):
        self._path = path
        self._open()

    def __len__(self):
        return len(self._sizes)

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return np.frombuffer(self._bin, dtype=self._dtype, count=int(self._sizes[idx]), offset=int(self._ptrs[idx]))
        if isinstance(idx, slice):
            start, stop, step = idx.indices(len(self))
            if step != 1:
                return [self[i] for i in range(start, stop, step)]
            if stop <= start:
                return []
            sizes = self._sizes[start:stop]
            flat = np.frombuffer(self._bin, dtype=self._dtype, count=int(sizes.sum()), offset=int(self._ptrs[start]))
            return np.split(flat, np.cumsum(sizes)[:-1])
        raise TypeError(f"unsupported index {type(idx)}")

    def get(self, idx, offset=0, length=None):
        size = int(self._sizes[idx])
        length = size - offset if length is None else length
        return np.frombuffer(self._bin, dtype=self._dtype, count=length,
                             offset=int(self._ptrs[idx]) + offset * self._dtype.itemsize)

    @property
    def sizes(self):
        return self._sizes

    def size(self, index):
        return int(self._sizes[index])

    @property
    def doc_idx(self):
        return self._doc_idx

    def get_doc_idx(self):
        return self._doc_idx

    @property
    def dtype(self):
        return self._dtype

    @property
    def supports_prefetch(self):
        return False

    @staticmethod
    def exists(path):
        return os.path.exists(index_file_path(path)) and os.path.exists(data_file_path(path))


class MMapIndexedDatasetBuilder:
    """Streams items to ``<out_file>`` (the ``.bin``); :meth:`finalize` writes the index."""

    def __init__(self, out_file, dtype=np.int64):
        self._dtype = _np_dtype(dtype)
        self._file = open(out_file, "wb")
        self._sizes = []
        self._doc_idx = [0]

    def add_item(self, tensor):
        arr = tensor.detach().cpu().numpy() if torch.is_tensor(tensor) else np.asarray(tensor)
        self.add_item_numpy(arr)

    def add_item_numpy(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self._dtype).reshape(-1)
        self._file.write(arr.tobytes(order="C"))
        self._sizes.append(arr.size)

    def add_items(self, arr_list):
        for a in arr_list:
            self.add_item(a)

    def end_document(self):
        self._doc_idx.append(len(self._sizes))

    def merge_file_(self, another_prefix):
        other = MMapIndexedDataset(another_prefix)
        if other.dtype != self._dtype:
            raise ValueError(f"merge: dtype {other.dtype} != {self._dtype}")
        base = len(self._sizes)
        self._sizes.extend(int(s) for s in other.sizes)
        self._doc_idx.extend(base + int(d) for d in other.doc_idx[1:])
        with open(data_file_path(another_prefix), "rb") as f:
            shutil.copyfileobj(f, self._file)

    def finalize(self, index_file):
        self._file.close()
        write_index(index_file, self._dtype, self._sizes, self._doc_idx)


def make_builder(out_file, impl="mmap", vocab_size=None, dtype=None):
    if impl not in ("mmap", "infer"):
        raise ValueError(f"indexed dataset impl {impl!r}: only 'mmap' is written by this framework")
    return MMapIndexedDatasetBuilder(out_file, dtype=dtype or best_fitting_dtype(vocab_size))


def make_dataset(path, impl="mmap", skip_warmup=True):
    if not MMapIndexedDataset.exists(path):
        return None
    return MMapIndexedDataset(path, skip_warmup)


def dataset_exists(path, impl="mmap"):
    return MMapIndexedDataset.exists(path)


def create_mmap_dataset_builder(fname, dtype):
    os.makedirs(os.path.dirname(fname) or ".", exist_ok=True)
    return MMapIndexedDatasetBuilder(data_file_path(fname), dtype=dtype)


def close_mmap_dataset_builder(builder, fname):
    builder.end_document()
    builder.finalize(index_file_path(fname))
