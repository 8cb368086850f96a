"""Host-side assembly of one ragged batch (reference `inference/v2/ragged/ragged_wrapper.py:31-193`).

Sequences are inserted one by one with their new tokens; `finalize()` orders them (single-token decodes of known
sequences first: the paged decode kernel takes a leading slice; prompts and prompt chunks after), builds every index
table the kernels need and ships them to the device in ONE packed pinned copy (`RaggedMeta.build`). The kernels of
`inference/v2/kernels/ragged_ops.py` and `DSInferenceModel.forward_ragged` read the tables from `.meta`.
"""
from typing import List

import torch

from ...model_implementations.transformer import RaggedMeta
from .sequence_descriptor import DSSequenceDescriptor


def to_padded(original_size: int) -> int:
    """Round a count up to the next power of two below 64, to the next multiple of 64 above (the granularity the
    reference pads its metadata buffers to)."""
    if original_size <= 0:
        return 1
    if original_size < 64:
        return 1 << (original_size - 1).bit_length()
    return -(-original_size // 64) * 64


class RaggedBatchWrapper:

    def __init__(self, config=None, block_size=None, device=None):
        """`config`: the state-manager config (`max_ragged_batch_size`, `max_ragged_sequence_count` bound what may be
        inserted); `block_size`: KV block size in tokens (default: the sequences' own)."""
        self._config = config
        self._block_size = block_size
        self._device = device
        self.clear()

    # ------------------------------------------------------------------------------------------ assembly
    def clear(self) -> None:
        self._seqs: List[DSSequenceDescriptor] = []
        self._toks: List[torch.Tensor] = []
        self._n_tokens = 0
        self._is_finalized = False
        self.meta = None
        self.order = []
        self._ids = None

    def insert_sequence(self, seq_descriptor: DSSequenceDescriptor, tokens: torch.Tensor, do_checks=True) -> None:
        if self._is_finalized:
            raise RuntimeError("the batch is finalized: clear() it before inserting")
        tokens = tokens.reshape(-1)
        if do_checks and self._config is not None:
            if len(self._seqs) + 1 > self._config.max_ragged_sequence_count:
                raise RuntimeError(f"Ragged batch is full due to sequence limit: "
                                   f"{self._config.max_ragged_sequence_count}")
            if self._n_tokens + tokens.numel() > self._config.max_ragged_batch_size:
                raise RuntimeError(f"Ragged batch is full due to capacity limit: "
                                   f"{self._config.max_ragged_batch_size}")
        self._seqs.append(seq_descriptor)
        self._toks.append(tokens)
        self._n_tokens += tokens.numel()

    def finalize(self, padding=False) -> None:
        """Build and upload the index tables. `padding` is accepted for signature parity: the in-tree kernels take
        exact counts, nothing is padded."""
        if not self._seqs:
            raise RuntimeError("cannot finalize an empty ragged batch")
        n = [t.numel() for t in self._toks]
        is_decode = [n[i] == 1 and self._seqs[i].seen_tokens > 0 for i in range(len(n))]
        self.order = sorted(range(len(n)), key=lambda i: 0 if is_decode[i] else 1)
        seqs = [self._seqs[i] for i in self.order]
        bs = self._block_size or seqs[0].block_size
        self.meta = RaggedMeta.build([s.seen_tokens for s in seqs], [n[i] for i in self.order],
                                     [s.blocks for s in seqs], sum(is_decode), bs, self._device)
        ids = torch.cat([self._toks[i] for i in self.order])
        if self._device is not None:
            ids = ids.to(self._device, non_blocking=True)
        self._ids = ids
        self._is_finalized = True

    def restore_order(self, rows: torch.Tensor) -> torch.Tensor:
        """Per-sequence rows in kernel order -> rows in insertion order."""
        inv = [0] * len(self.order)
        for j, i in enumerate(self.order):
            inv[i] = j
        return rows.index_select(0, torch.tensor(inv, device=rows.device))

    # ------------------------------------------------------------------------------------------ views
    def _need(self):
        if not self._is_finalized:
            raise RuntimeError("finalize() the batch first")
        return self.meta

    def input_ids(self, on_device=True) -> torch.Tensor:
        self._need()
        return self._ids if on_device else self._ids.cpu()

    def batch_metadata_buffer(self, on_device=True) -> torch.Tensor:
        """[total tokens, total sequences] int32."""
        t = torch.tensor([self.current_tokens, self.current_sequences], dtype=torch.int32)
        return t.to(self._ids.device) if on_device and self._ids is not None else t

    def inflight_seq_descriptors(self, on_device=True) -> torch.Tensor:
        """[S, 4] int32 per sequence (kernel order): first token row, new tokens, tokens already cached, 0."""
        m = self._need()
        cu = m.cu_q[:-1]
        out = torch.stack([cu, m.cu_q[1:] - cu, m.start_pos, torch.zeros_like(cu)], dim=1)
        return out if on_device else out.cpu()

    def tokens_to_seq(self, on_device=True) -> torch.Tensor:
        m = self._need()
        return m.seq_ids if on_device else m.seq_ids.cpu()

    def kv_ptrs(self, on_device=True) -> torch.Tensor:
        """[S, max blocks] int32 block table (the in-tree kernels index blocks, they do not take raw pointers)."""
        m = self._need()
        return m.block_tables if on_device else m.block_tables.cpu()

    def masks(self, on_device=True):
        return None

    @property
    def current_tokens(self) -> int:
        return self._n_tokens

    @property
    def current_sequences(self) -> int:
        return len(self._seqs)

    @property
    def tensor_toks(self) -> torch.Tensor:
        dev = self._ids.device if self._ids is not None else "cpu"
        return torch.tensor([self._n_tokens], dtype=torch.int32, device=dev)
