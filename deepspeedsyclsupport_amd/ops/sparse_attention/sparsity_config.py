"""Block-sparse attention layouts (reference `ops/sparse_attention/sparsity_config.py`: Dense, Fixed, Variable,
BigBird, BSLongformer, LocalSlidingWindow). A layout is an int tensor [num_heads, num_blocks, num_blocks]; entry
(h, i, j) = 1 when query block i of head h attends to key block j."""
import random

import torch


class SparsityConfig:

    def __init__(self, num_heads, block=16, different_layout_per_head=False):
        self.num_heads = num_heads
        self.block = block
        self.different_layout_per_head = different_layout_per_head
        self.num_layout_heads = num_heads if different_layout_per_head else 1

    def setup_layout(self, seq_len):
        if seq_len % self.block:
            raise ValueError(f"Sequence Length, {seq_len}, needs to be dividable by Block size {self.block}!")
        nb = seq_len // self.block
        return torch.zeros((self.num_heads, nb, nb), dtype=torch.int64)

    def check_and_propagate_first_head_layout(self, layout):
        if not self.different_layout_per_head:
            layout[1:] = layout[0]
        return layout

    def make_layout(self, seq_len):
        raise NotImplementedError


class DenseSparsityConfig(SparsityConfig):

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        layout[:] = 1
        return layout


def _causal(layout, h):
    nb = layout.shape[1]
    layout[h] &= torch.tril(torch.ones(nb, nb, dtype=layout.dtype))


class FixedSparsityConfig(SparsityConfig):
    """Local windows of `num_local_blocks` + per-window global representative blocks (Child et al. 2019)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_local_blocks=4, num_global_blocks=1,
                 attention="bidirectional", horizontal_global_attention=False, num_different_global_patterns=1):
        super().__init__(num_heads, block, different_layout_per_head)
        if num_local_blocks % num_global_blocks:
            raise ValueError("num_local_blocks must be divisible by num_global_blocks")
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError('only "uni/bi-directional" attentions are supported')
        if attention != "bidirectional" and horizontal_global_attention:
            raise ValueError("horizontal global attention needs bidirectional attention")
        if num_different_global_patterns > 1 and not different_layout_per_head:
            raise ValueError("num_different_global_patterns > 1 needs different_layout_per_head")
        if num_different_global_patterns > num_local_blocks // num_global_blocks:
            raise ValueError("too many global patterns for the window")
        self.num_local_blocks, self.num_global_blocks = num_local_blocks, num_global_blocks
        self.attention = attention
        self.horizontal_global_attention = horizontal_global_attention
        self.num_different_global_patterns = num_different_global_patterns

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        for s in range(0, nb, self.num_local_blocks):
            e = min(s + self.num_local_blocks, nb)
            layout[h, s:e, s:e] = 1
        if self.attention == "unidirectional":
            _causal(layout, h)
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        W, G = self.num_local_blocks, self.num_global_blocks
        first = W - (1 + h % self.num_different_global_patterns) * G
        full_end = nb - nb % W
        starts = list(range(first, full_end, W))
        if full_end < nb:  # short last window
            starts.append(min(full_end + first, nb - G))
        for c in starts:
            r0 = 0 if self.attention == "bidirectional" else c
            layout[h, r0:, c:c + G] = 1
            if self.horizontal_global_attention:
                layout[h, c:c + G, :] = 1
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_local_layout(h, layout)
            self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class VariableSparsityConfig(SparsityConfig):
    """Random blocks + variable-size local windows + explicit global block indices."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=0,
                 local_window_blocks=[4], global_block_indices=[0], global_block_end_indices=None,
                 attention="bidirectional", horizontal_global_attention=False):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_random_blocks = num_random_blocks
        self.local_window_blocks = local_window_blocks
        self.global_block_indices = global_block_indices
        if global_block_end_indices is not None:
            if len(global_block_indices) != len(global_block_end_indices):
                raise ValueError("global block start/end index lists differ in length")
            for s, e in zip(global_block_indices, global_block_end_indices):
                if s >= e:
                    raise ValueError("global block start index must be < end index")
        self.global_block_end_indices = global_block_end_indices
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError('only "uni/bi-directional" attentions are supported')
        if attention != "bidirectional" and horizontal_global_attention:
            raise ValueError("horizontal global attention needs bidirectional attention")
        self.attention = attention
        self.horizontal_global_attention = horizontal_global_attention

    def set_random_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_random_blocks:
            raise ValueError("more random blocks than blocks per row")
        for row in range(nb):
            hi = nb if self.attention == "bidirectional" else row + 1
            cols = random.sample(range(hi), min(self.num_random_blocks, hi))
            layout[h, row, cols] = 1
        return layout

    def set_local_layout(self, h, layout):
        nb = layout.shape[1]
        s = 0
        wins = list(self.local_window_blocks)
        i = 0
        while s < nb:
            w = wins[min(i, len(wins) - 1)]
            e = min(s + w, nb)
            layout[h, s:e, s:e] = 1
            s, i = e, i + 1
        if self.attention == "unidirectional":
            _causal(layout, h)
        return layout

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s >= nb:
                continue
            e = min(e, nb)
            r0 = 0 if self.attention == "bidirectional" else s
            layout[h, r0:, s:e] = 1
            if self.horizontal_global_attention:
                layout[h, s:e, :] = 1
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_random_layout(h, layout)
            self.set_local_layout(h, layout)
            self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class BigBirdSparsityConfig(SparsityConfig):
    """Random + sliding window + global (ITC) blocks (Zaheer et al. 2020)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_random_blocks=1,
                 num_sliding_window_blocks=3, num_global_blocks=1, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_random_blocks = num_random_blocks
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.num_global_blocks = num_global_blocks
        if attention not in ("unidirectional", "bidirectional"):
            raise NotImplementedError('only "uni/bi-directional" attentions are supported')
        self.attention = attention

    def set_random_layout(self, h, layout):
        return VariableSparsityConfig.set_random_layout(self, h, layout)

    def set_sliding_window_layout(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_sliding_window_blocks:
            raise ValueError("sliding window wider than the sequence")
        w = self.num_sliding_window_blocks // 2
        idx = torch.arange(nb)
        band = (idx[None, :] - idx[:, None]).abs() <= w
        layout[h] |= band.to(layout.dtype)
        if self.attention == "unidirectional":
            _causal(layout, h)
        return layout

    def set_global_layout_itc(self, h, layout):
        nb = layout.shape[1]
        if nb < self.num_global_blocks:
            raise ValueError("more global blocks than blocks")
        g = self.num_global_blocks
        layout[h, :g, :] = 1
        layout[h, :, :g] = 1
        if self.attention == "unidirectional":
            _causal(layout, h)
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_random_layout(h, layout)
            self.set_sliding_window_layout(h, layout)
            self.set_global_layout_itc(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class BSLongformerSparsityConfig(SparsityConfig):
    """Sliding window + global blocks given by index (block-sparse Longformer, Beltagy et al. 2020)."""

    def __init__(self, num_heads, block=16, different_layout_per_head=False, num_sliding_window_blocks=3,
                 global_block_indices=[0], global_block_end_indices=None, attention="bidirectional"):
        super().__init__(num_heads, block, different_layout_per_head)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.global_block_indices = global_block_indices
        self.global_block_end_indices = global_block_end_indices
        self.attention = attention

    def set_sliding_window_layout(self, h, layout):
        return BigBirdSparsityConfig.set_sliding_window_layout(self, h, layout)

    def set_global_layout(self, h, layout):
        nb = layout.shape[1]
        ends = self.global_block_end_indices or [i + 1 for i in self.global_block_indices]
        for s, e in zip(self.global_block_indices, ends):
            if s < nb:
                layout[h, s:min(e, nb), :] = 1
                layout[h, :, s:min(e, nb)] = 1
        if self.attention == "unidirectional":
            _causal(layout, h)
        return layout

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_sliding_window_layout(h, layout)
            self.set_global_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)


class LocalSlidingWindowSparsityConfig(SparsityConfig):
    """Purely local sliding window (each block attends to `num_sliding_window_blocks` around it)."""

    def __init__(self, num_heads, block=16, num_sliding_window_blocks=3, attention="unidirectional"):
        super().__init__(num_heads, block)
        self.num_sliding_window_blocks = num_sliding_window_blocks
        self.attention = attention

    def set_sliding_window_layout(self, h, layout):
        return BigBirdSparsityConfig.set_sliding_window_layout(self, h, layout)

    def make_layout(self, seq_len):
        layout = self.setup_layout(seq_len)
        for h in range(self.num_layout_heads):
            self.set_sliding_window_layout(h, layout)
        return self.check_and_propagate_first_head_layout(layout)
