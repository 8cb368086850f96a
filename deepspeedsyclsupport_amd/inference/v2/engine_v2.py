"""Ragged-batching inference engine (reference `inference/v2/engine_v2.py:30-240`, FastGen's put / query /
can_schedule / flush contract).

`put(uids, tokens)` runs ONE scheduling step over a ragged batch as ONE forward (reference `ragged_wrapper.py:31-193`
+ `engine_v2.py:107-153`): the new tokens of every sequence — single-token decodes first, then prompts and
SplitFuse prompt chunks of any length continuing from their cached prefix — are concatenated; the GEMMs run over all
T tokens at once, the fused QKV epilogue appends every token's K/V to the paged cache, the paged decode kernel
serves the decode rows and the ragged paged flash-prefill kernel (`csrc/attn/paged_prefill.hip`) the chunk rows.
All per-step metadata goes to the device in one packed copy; nothing syncs back to the host. It returns one row of
logits per sequence, in the order given. KV blocks are allocated on demand from a per-engine block pool sized from
free HBM (RESERVE mode) or an explicit block count (ALLOCATE mode).
"""
from typing import Iterable, Tuple

import torch

from ..model_implementations.transformer import DSInferenceModel
from .config_v2 import AllocationMode, RaggedInferenceEngineConfig
from .ragged import DSStateManager, PlaceholderSequenceDescriptor, RaggedBatchWrapper
from .scheduling_utils import SchedulingError, SchedulingResult


class InferenceEngineV2:

    def __init__(self, model: DSInferenceModel, engine_config: RaggedInferenceEngineConfig = None):
        self._config = engine_config or RaggedInferenceEngineConfig()
        self._model = model
        sm = self._config.state_manager
        bs = self._config.kv_cache.block_size
        spec = model.spec
        hk = max(spec.num_kv_heads // model.tp_size, 1)
        if sm.memory_config.mode == AllocationMode.ALLOCATE:
            num_blocks = int(sm.memory_config.size)
        else:
            from ..kv_cache import BlockedKVCache
            if model.device is not None and torch.device(model.device).type == "cuda":
                free, _ = torch.cuda.mem_get_info(model.device)
                avail = max(free - int(sm.memory_config.size), 0)
            else:
                avail = 256 * 2**20  # host rehearsal: a small fixed pool
            num_blocks = BlockedKVCache.blocks_for_memory(avail, spec.num_layers, hk, bs, spec.head_dim, model.dtype)
        model.allocate_cache(num_blocks, bs)
        self._state_manager = DSStateManager(sm, num_blocks, bs)
        self._state_manager.attach_cache(getattr(model, "cache", None))
        self._device = model.device if model.device is not None else torch.device("cpu")
        self._batch = RaggedBatchWrapper(sm, bs, self._device)

    # ------------------------------------------------------------------------------------------ properties
    @property
    def free_blocks(self):
        return torch.tensor([self._state_manager.free_blocks])

    @property
    def n_kv_cache_groups(self):
        return 1

    @property
    def model(self):
        return self._model

    # ------------------------------------------------------------------------------------------ forward
    @torch.no_grad()
    def put(self, batch_uids: Iterable[int], batch_tokens: Iterable[torch.Tensor], do_checks=True) -> torch.Tensor:
        uids = list(batch_uids)
        toks = [t.reshape(-1) for t in batch_tokens]
        if do_checks:
            res = self.can_schedule(uids, [t.numel() for t in toks])
            if res != SchedulingResult.Success:
                raise SchedulingError(res)
        batch = self._batch
        batch.clear()
        seqs = []
        for uid, t in zip(uids, toks):
            seq = self._state_manager.get_or_create_sequence(uid)
            self._state_manager.allocate_blocks(seq, t.numel())
            seq.pre_forward(t.numel())
            batch.insert_sequence(seq, t, do_checks=False)
            seqs.append(seq)
        batch.finalize()
        logits = self._model.forward_ragged(batch.input_ids(), batch.meta)
        out = batch.restore_order(logits)
        for s in seqs:
            s.post_forward()
        return out

    # ------------------------------------------------------------------------------------------ scheduling
    def _kv_requirements(self, seq, max_tokens, max_blocks):
        room = self._config.state_manager.max_context - seq.seen_tokens
        n = min(max_tokens, max(room, 0))
        while n > 0 and seq.blocks_needed(n) > max_blocks:
            # shrink to what the free blocks can hold (whole blocks beyond the current tail)
            tail = len(seq.blocks) * seq.block_size - seq.seen_tokens
            n = min(n - 1, tail + max_blocks * seq.block_size)
        return n, seq.blocks_needed(n)

    def query(self, uid: int, max_request_tokens: int, max_request_blocks) -> Tuple[int, int]:
        seq = self._state_manager.get_sequence(uid)
        if seq is None:
            if self._state_manager.n_tracked_sequences >= self._config.state_manager.max_tracked_sequences:
                return (0, 0)
            seq = PlaceholderSequenceDescriptor(self._state_manager.block_size)
        return self._kv_requirements(seq, max_request_tokens, int(max_request_blocks))

    def can_schedule(self, uids: Iterable[int], lengths: Iterable[int]) -> SchedulingResult:
        sm = self._config.state_manager
        uids, lengths = list(uids), list(lengths)
        if len(uids) > sm.max_ragged_sequence_count:
            return SchedulingResult.BatchSequenceLimitExceeded
        cur, free = self._state_manager.n_tracked_sequences, self._state_manager.free_blocks
        total = 0
        for uid, n in zip(uids, lengths):
            seq = self._state_manager.get_sequence(uid)
            if seq is None:
                cur += 1
                seq = PlaceholderSequenceDescriptor(self._state_manager.block_size)
            if seq.seen_tokens + n > sm.max_context:
                return SchedulingResult.SequenceTokenLimitExceeded
            got, blocks = self._kv_requirements(seq, n, free)
            if got != n:
                return SchedulingResult.KVCacheLimitExceeded
            free -= blocks
            total += n
        if cur > sm.max_tracked_sequences:
            return SchedulingResult.EngineSequenceLimitExceeded
        if total > sm.max_ragged_batch_size:
            return SchedulingResult.BatchTokenLimitExceeded
        return SchedulingResult.Success

    def flush(self, uid: int) -> None:
        self._state_manager.flush_sequence(uid)

    def serialize(self, save_path: str) -> None:
        """Save the (sharded) injected weights + spec so the engine can be rebuilt without the HF checkpoint."""
        import dataclasses
        import json
        import os
        os.makedirs(save_path, exist_ok=True)
        from safetensors.torch import save_file
        sd = {k: v.detach().contiguous().cpu() for k, v in self._model.state_dict().items()}
        save_file(sd, os.path.join(save_path, f"params_rank_{self._model.tp_rank}.safetensors"))
        if self._model.tp_rank == 0:
            with open(os.path.join(save_path, "ds_model_config.json"), "w") as f:
                json.dump(dataclasses.asdict(self._model.spec), f)
            with open(os.path.join(save_path, "ds_model_meta.json"), "w") as f:
                json.dump({"dtype": str(self._model.dtype).replace("torch.", ""), "tp_size": self._model.tp_size}, f)
