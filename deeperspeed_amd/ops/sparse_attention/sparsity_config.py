"""Block-sparse attention layouts.

Reference parity: deepspeed/ops/sparse_attention/sparsity_config.py:9-740.  Every config
produces an int64 layout [num_heads, S/block, S/block] (1 = block computed); the patterns
(Dense, Fixed, Variable, BigBird, BSLongformer, LocalSlidingWindow) and their argument
validation match the reference so layouts are interchangeable.  Random blocks use Python's
`random` module (seed it for reproducibility, as with the reference).
"""

import random

import torch

_ATTN = ("unidirectional", "bidirectional")


class SparsityConfig:
    """Shared properties: number of heads, block size, one layout for all heads or not."""

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
            layout[1:self.num_heads] = layout[0]
        return layout

    def make_layout(self, seq_len):  # pragma: no cover - abstract
        raise NotImplementedError


def _check_attention(attention, horizontal_global_attention=False):
    if attention not in _ATTN:
        raise NotImplementedError('only "uni/bi-directional" attentions are supported for now!')
    if attention != "bidirectional" and horizontal_global_attention:
        raise ValueError('only "bi-directional" attentions can support horizontal global attention!')


def _check_global_ranges(starts, ends):
    if ends is None:
        return
    if len(starts) != len(ends):
        raise ValueError(f"Global block start indices length, {len(starts)}, must be same as global block end "
                         f"indices length, {len(ends)}!")
    for s, e in zip(starts, ends):
        if s >= e:
            raise ValueError(f"Global block start index, {s}, must be smaller than global block end index, {e}!")


def _window(layout, h, lo, hi, causal):
    """Dense (lower-triangular if causal) block window on rows/cols [lo, hi)."""
    for row in range(lo, hi):
        layout[h, row, lo:(row + 1 if causal else hi)] = 1


class DenseSparsityConfig(SparsityConfig):
    """All blocks present (for comparison with the sparse patterns)."""

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        layout[:] = 1
        return layout


class FixedSparsityConfig(SparsityConfig):
    """`Fixed` pattern of Sparse Transformers (arXiv:1904.10509): local windows of
    `num_local_blocks` plus `num_global_blocks` representative blocks per window that every
    (later, if unidirectional) row attends to."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_local_blocks=4, num_global_blocks=1,
                 attention="bidirectional", horizontal_global_attention=False, num_different_global_patterns=1):
        super().__init__(num_heads, block, different_layout_per_head)
        if num_global_blocks > 0 and num_local_blocks % num_global_blocks != 0:
            raise ValueError(f"Number of blocks in a local window, {num_local_blocks}, must be dividable by number "
                             f"of global blocks, {num_global_blocks}!")
        _check_attention(attention, horizontal_global_attention)
        if num_different_global_patterns > 1 and not different_layout_per_head:
            raise ValueError("Number of different layouts cannot be more than one when you have set a single layout "
                             "for all heads! Set different_layout_per_head to True.")
        if num_global_blocks > 0 and num_different_global_patterns > num_local_blocks // num_global_blocks:
            raise ValueError(f"Number of layout versions (num_different_global_patterns), "
                             f"{num_different_global_patterns}, cannot be larger than number of local window blocks "
                             f"divided by number of global blocks, {num_local_blocks} / {num_global_blocks} = "
                             f"{num_local_blocks // num_global_blocks}!")
        self.num_local_blocks = num_local_blocks
        self.num_global_blocks = num_global_blocks
        self.attention = attention
        self.horizontal_global_attention = horizontal_global_attention
        self.num_different_global_patterns = num_different_global_patterns

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        for lo in range(0, nb, self.num_local_blocks):
            _window(layout, h, lo, min(lo + self.num_local_blocks, nb), self.attention == "unidirectional")
        return layout

    def _global_cols(self, layout, h, lo, hi):
        first_row = 0 if self.attention == "bidirectional" else lo
        layout[h, first_row:, lo:hi] = 1
        if self.horizontal_global_attention:
            layout[h, lo:hi, :] = 1

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        # the representative blocks sit at the END of each window; head h uses pattern h % P
        first = self.num_local_blocks - (1 + h % self.num_different_global_patterns) * self.num_global_blocks
        full_end = nb - nb % self.num_local_blocks
        for i in range(first, full_end, self.num_local_blocks):
            self._global_cols(layout, h, i, i + self.num_global_blocks)
        if full_end < nb:  # trailing partial window
            start = min(full_end + first, nb - self.num_global_blocks)
            self._global_cols(layout, h, start, start + self.num_global_blocks)
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_local_layout(h, layout)
            if self.num_global_blocks > 0:
                self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class VariableSparsityConfig(SparsityConfig):
    """Fixed extended with random blocks, a list of local window sizes (the last size
    repeats) and explicit global block indices / ranges."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=0,
                 local_window_blocks=[4], global_block_indices=[0], global_block_end_indices=None,
                 attention="bidirectional", horizontal_global_attention=False):
        super().__init__(num_heads, block, different_layout_per_head)
        _check_global_ranges(global_block_indices, global_block_end_indices)
        _check_attention(attention, horizontal_global_attention)
        self.num_random_blocks = num_random_blocks
        self.local_window_blocks = local_window_blocks
        self.global_block_indices = global_block_indices
        self.global_block_end_indices = global_block_end_indices
        self.attention = attention
        self.horizontal_global_attention = horizontal_global_attention

    def set_random_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError(f"Number of random blocks, {self.num_random_blocks}, must be smaller than overal number "
                             f"of blocks in a row, {nb}!")
        for row in range(nb):
            layout[h, row, random.sample(range(nb), self.num_random_blocks)] = 1
        return layout

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        causal = self.attention == "unidirectional"
        lo = 0
        size = self.local_window_blocks[-1]
        for size in self.local_window_blocks:
            _window(layout, h, lo, min(lo + size, nb), causal)
            lo += size
        for start in range(lo, nb, size):
            _window(layout, h, start, min(start + size, nb), causal)
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [s + 1 for s in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s >= nb:
                continue
            e = min(e, nb)
            if self.horizontal_global_attention:
                layout[h, s:e, :] = 1
            layout[h, (0 if self.attention == "bidirectional" else s):, s:e] = 1
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_random_layout(h, layout)
            self.set_local_layout(h, layout)
            self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class BigBirdSparsityConfig(SparsityConfig):
    """BigBird (arXiv:2007.14062): random + sliding window + ITC global blocks."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=1,
                 num_sliding_window_blocks=3, num_global_blocks=1, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_random_blocks = num_random_blocks
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.num_global_blocks = num_global_blocks
        self.attention = attention

    def set_random_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError(f"Number of random blocks, {self.num_random_blocks}, must be smaller than overal number "
                             f"of blocks in a row, {nb}!")
        for row in range(nb):
            pool = range(nb) if self.attention == "bidirectional" else range(row + 1)
            layout[h, row, random.sample(pool, self.num_random_blocks)] = 1
        return layout

    def set_sliding_window_layout(self, h, layout):
        _sliding(layout, h, self.num_sliding_window_blocks, self.attention == "bidirectional")
        return layout

    def set_global_layout_itc(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_global_blocks:
            raise ValueError(f"Number of global blocks, {self.num_global_blocks}, must be smaller than overal number "
                             f"of blocks in a row, {nb}!")
        layout[h, :self.num_global_blocks, :] = 1
        layout[h, :, :self.num_global_blocks] = 1
        if self.attention == "unidirectional":
            layout = torch.tril(layout)
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_random_layout(h, layout)
            self.set_sliding_window_layout(h, layout)
            layout = self.set_global_layout_itc(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


def _sliding(layout, h, window, bidirectional):
    nb = layout.shape[1]
    if nb < window:
        raise ValueError(f"Number of sliding window blocks, {window}, must be smaller than overal number of blocks "
                         f"in a row, {nb}!")
    w = window // 2
    for row in range(nb):
        layout[h, row, max(0, row - w):(min(row + w + 1, nb) if bidirectional else row + 1)] = 1


class BSLongformerSparsityConfig(SparsityConfig):
    """Block-sparse Longformer (arXiv:2004.05150): sliding window + global rows/columns."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_sliding_window_blocks=3,
                 global_block_indices=[0], global_block_end_indices=None, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        _check_global_ranges(global_block_indices, global_block_end_indices)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.global_block_indices = global_block_indices
        self.global_block_end_indices = global_block_end_indices
        self.attention = attention

    def set_sliding_window_layout(self, h, layout):
        _sliding(layout, h, self.num_sliding_window_blocks, True)  # window is symmetric here; tril below
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [s + 1 for s in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s < nb:
                e = min(e, nb)
                layout[h, s:e, :] = 1
                layout[h, :, s:e] = 1
        if self.attention == "unidirectional":
            layout = torch.tril(layout)
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_sliding_window_layout(h, layout)
            layout = self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class LocalSlidingWindowSparsityConfig(SparsityConfig):
    """Sliding-window-only pattern (causal by default)."""

    def __init__(self, num_heads, block=16, num_sliding_window_blocks=3, attention="unidirectional"):
        super().__init__(num_heads, block)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.attention = attention

    def set_sliding_window_layout(self, h, layout):
        _sliding(layout, h, self.num_sliding_window_blocks, self.attention == "bidirectional")
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_sliding_window_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)
