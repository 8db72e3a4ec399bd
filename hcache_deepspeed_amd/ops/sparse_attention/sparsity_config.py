"""Block-sparse attention layouts.

Reference parity: ops/sparse_attention/sparsity_config.py -- ``SparsityConfig`` (:10), ``DenseSparsityConfig``
(:63), ``FixedSparsityConfig`` (:95, Sparse Transformers "fixed" pattern), ``VariableSparsityConfig`` (:239),
``BigBirdSparsityConfig`` (:411), ``BSLongformerSparsityConfig`` and ``LocalSlidingWindowSparsityConfig``.
A layout is an int64 tensor [num_heads, num_blocks, num_blocks]; 1 = the (query block, key block) pair is
computed. ``attention='unidirectional'`` keeps only blocks on or below the diagonal.

The HIP kernel (csrc/kernels/sparse_attn.hip) works on 64 x 64 blocks (one LDS tile = two MFMA row groups);
layouts with ``block`` a multiple of 64 run natively, smaller blocks run on the torch gather path.
"""
import random

import torch


class SparsityConfig:

    def __init__(self, num_heads, block=16, different_layout_per_head=False):
        self.num_heads = num_heads
        self.block = block
        self.different_layout_per_head = different_layout_per_head
        self.num_layout_heads = num_heads if different_layout_per_head else 1

    def setup_layout(self, seq_len):
        if seq_len % self.block != 0:
            raise ValueError(f"Sequence Length, {seq_len}, needs to be dividable by Block size {self.block}!")
        nb = seq_len // self.block
        return torch.zeros((self.num_heads, nb, nb), dtype=torch.int64)

    def check_and_propagate_first_head_layout(self, layout):
        if not self.different_layout_per_head:
            layout[1:self.num_heads, :, :] = layout[0, :, :]
        return layout

    def make_layout(self, seq_len):
        raise NotImplementedError


def _check_attention(attention):
    if attention not in ("unidirectional", "bidirectional"):
        raise NotImplementedError("only 'uni/bi-directional' attentions are supported for now!")
    return attention


class DenseSparsityConfig(SparsityConfig):
    """All blocks set (a dense layout, for comparison)."""

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        layout[:, :, :] = 1
        return layout


class FixedSparsityConfig(SparsityConfig):
    """Local windows of ``num_local_blocks`` plus ``num_global_blocks`` summary blocks at the END of each window
    (different heads may pick different summary positions, ``num_different_global_patterns``)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_local_blocks=4, num_global_blocks=1,
                 attention="bidirectional", horizontal_global_attention=False, num_different_global_patterns=1):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_local_blocks = num_local_blocks
        if num_local_blocks % num_global_blocks != 0:
            raise ValueError(f"Number of blocks in a local window, {num_local_blocks}, "
                             f"must be dividable by number of global blocks, {num_global_blocks}!")
        self.num_global_blocks = num_global_blocks
        self.attention = _check_attention(attention)
        if attention != "bidirectional" and horizontal_global_attention:
            raise ValueError("only \"bi-directional\" attentions can support horizontal global attention!")
        self.horizontal_global_attention = horizontal_global_attention
        if num_different_global_patterns > 1 and not different_layout_per_head:
            raise ValueError("Number of different layouts cannot be more than one when you have set a single layout "
                             "for all heads! Set different_layout_per_head to True.")
        if num_different_global_patterns > (num_local_blocks // num_global_blocks):
            raise ValueError(f"Number of layout versions (num_different_global_patterns), "
                             f"{num_different_global_patterns}, cannot be larger than number of local window blocks "
                             f"divided by number of global blocks, {num_local_blocks} / {num_global_blocks} = "
                             f"{num_local_blocks // num_global_blocks}!")
        self.num_different_global_patterns = num_different_global_patterns

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        w = self.num_local_blocks
        for s in range(0, nb, w):
            e = min(s + w, nb)
            for r in range(s, e):
                hi = r + 1 if self.attention == "unidirectional" else e
                layout[h, r, s:hi] = 1
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        w, g = self.num_local_blocks, self.num_global_blocks
        shift = (h % self.num_different_global_patterns) * g
        # summary blocks: the last g blocks of every window, moved left by the head's pattern shift
        for s in range(0, nb, w):
            first = s + w - g - shift
            if first >= nb:  # a partial last window keeps its summary inside the sequence
                first = max(s, nb - g)
            for c in range(first, min(first + g, nb)):
                lo = c if self.attention == "unidirectional" else 0
                layout[h, lo:, c] = 1
                if self.horizontal_global_attention:
                    layout[h, c, :] = 1
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            layout = self.set_local_layout(h, layout)
            layout = self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class VariableSparsityConfig(SparsityConfig):
    """Random blocks + variable-size local windows (the last size repeats) + explicit global blocks."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=0,
                 local_window_blocks=(4, ), global_block_indices=(0, ), global_block_end_indices=None,
                 attention="bidirectional", horizontal_global_attention=False):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_random_blocks = num_random_blocks
        self.local_window_blocks = list(local_window_blocks)
        self.global_block_indices = list(global_block_indices)
        if global_block_end_indices is not None:
            if len(global_block_indices) != len(global_block_end_indices):
                raise ValueError("Global block start indices length must equal global block end indices length")
            for s, e in zip(global_block_indices, global_block_end_indices):
                if s >= e:
                    raise ValueError("Global block start index must be smaller than global block end index")
        self.global_block_end_indices = None if global_block_end_indices is None else list(global_block_end_indices)
        self.attention = _check_attention(attention)
        if attention != "bidirectional" and horizontal_global_attention:
            raise ValueError("only \"bi-directional\" attentions can support horizontal global attention!")
        self.horizontal_global_attention = horizontal_global_attention

    def set_random_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError(f"Number of random blocks, {self.num_random_blocks}, must be smaller than overall "
                             f"number of blocks in a row, {nb}!")
        for r in range(nb):
            cols = range(r + 1) if self.attention == "unidirectional" else range(nb)
            for c in random.sample(list(cols), min(self.num_random_blocks, len(cols))):
                layout[h, r, c] = 1
        return layout

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        s = 0
        i = 0
        while s < nb:
            w = self.local_window_blocks[min(i, len(self.local_window_blocks) - 1)]
            e = min(s + w, nb)
            for r in range(s, e):
                hi = r + 1 if self.attention == "unidirectional" else e
                layout[h, r, s:hi] = 1
            s, i = e, i + 1
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s >= nb:
                continue
            e = min(e, nb)
            for c in range(s, e):
                lo = c if self.attention == "unidirectional" else 0
                layout[h, lo:, c] = 1
                if self.horizontal_global_attention:
                    layout[h, c, :] = 1
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            layout = self.set_random_layout(h, layout)
            layout = self.set_local_layout(h, layout)
            layout = self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


def _sliding(layout, h, w, attention):
    nb = layout.shape[1]
    if nb < w:
        raise ValueError(f"Number of sliding window blocks, {w}, must be smaller than overall number of blocks "
                         f"in a row, {nb}!")
    half = w // 2
    for r in range(nb):
        lo = max(0, r - half)
        hi = r + 1 if attention == "unidirectional" else min(nb, r + half + 1)
        layout[h, r, lo:hi] = 1
    return layout


class BigBirdSparsityConfig(SparsityConfig):
    """Random + sliding window + global (ITC: the first ``num_global_blocks`` rows and columns)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=1,
                 num_sliding_window_blocks=3, num_global_blocks=1, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_random_blocks = num_random_blocks
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.num_global_blocks = num_global_blocks
        self.attention = _check_attention(attention)

    def set_random_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError(f"Number of random blocks, {self.num_random_blocks}, must be smaller than overall "
                             f"number of blocks in a row, {nb}!")
        for r in range(nb):
            cols = list(range(r + 1)) if self.attention == "unidirectional" else list(range(nb))
            for c in random.sample(cols, min(self.num_random_blocks, len(cols))):
                layout[h, r, c] = 1
        return layout

    def set_sliding_window_layout(self, h, layout):
        return _sliding(layout, h, self.num_sliding_window_blocks, self.attention)

    def set_global_layout_itc(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_global_blocks:
            raise ValueError(f"Number of global blocks, {self.num_global_blocks}, must be smaller than overall number "
                             f"of blocks in a row, {nb}!")
        g = self.num_global_blocks
        layout[h, :g, :] = 1
        layout[h, :, :g] = 1
        if self.attention == "unidirectional":
            layout[h] = torch.tril(layout[h])
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            layout = self.set_random_layout(h, layout)
            layout = self.set_sliding_window_layout(h, layout)
            layout = self.set_global_layout_itc(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class BSLongformerSparsityConfig(SparsityConfig):
    """Block-sparse Longformer: sliding window + global blocks (indices or [start, end) ranges)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_sliding_window_blocks=3,
                 global_block_indices=(0, ), global_block_end_indices=None, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.global_block_indices = list(global_block_indices)
        self.attention = _check_attention(attention)
        if global_block_end_indices is not None:
            if len(global_block_indices) != len(global_block_end_indices):
                raise ValueError("Global block start indices length must equal global block end indices length")
            for s, e in zip(global_block_indices, global_block_end_indices):
                if s >= e:
                    raise ValueError("Global block start index must be smaller than global block end index")
        self.global_block_end_indices = None if global_block_end_indices is None else list(global_block_end_indices)

    def set_sliding_window_layout(self, h, layout):
        return _sliding(layout, h, self.num_sliding_window_blocks, self.attention)

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s >= nb:
                continue
            e = min(e, nb)
            layout[h, s:e, :] = 1
            layout[h, :, s:e] = 1
        if self.attention == "unidirectional":
            layout[h] = torch.tril(layout[h])
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            layout = self.set_sliding_window_layout(h, layout)
            layout = self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class LocalSlidingWindowSparsityConfig(SparsityConfig):
    """Sliding window only."""

    def __init__(self, num_heads, block=16, num_sliding_window_blocks=3, attention="unidirectional"):
        super().__init__(num_heads, block)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.attention = _check_attention(attention)

    def set_sliding_window_layout(self, h, layout):
        return _sliding(layout, h, self.num_sliding_window_blocks, self.attention)

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            layout = self.set_sliding_window_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)
