"""Inference engine (reference `inference/engine.py:42-620`: TP group creation, kernel injection / AutoTP, dtype
conversion, CUDA-graph capture, generate wrapper, checkpoint loading).

MI355X design:
* Kernel injection replaces the whole HF decoder with `DSInferenceModel` (paged KV cache, HIP decode attention,
  fused norm/act kernels, hipBLASLt GEMMs) instead of patching modules one by one; AutoTP (no injection) shards the
  HF model's own Linear layers (`module_inject.auto_tp`).
* Decode steps are captured once per batch size into a HIP graph (`enable_cuda_graph`) over static input/metadata
  buffers; each step is then one graph launch (the per-layer launch overhead dominates small-batch decode).
* Tensor parallel groups are consecutive ranks (one node's GPUs over xGMI); two all-reduces per layer.
"""
import time

import torch

from .. import comm as dist
from ..accelerator import get_accelerator
from ..utils.logging import log_dist
from .config import DeepSpeedInferenceConfig
from .model_implementations import convert
from .model_implementations.transformer import BatchMeta, DSInferenceModel


class GenerationOutput:

    def __init__(self, logits):
        self.logits = logits

    def __getitem__(self, i):
        return (self.logits, )[i]


class InferenceEngine(torch.nn.Module):
    inference_mp_group = None
    inference_ep_group = None

    def __init__(self, model, config: DeepSpeedInferenceConfig):
        super().__init__()
        self._config = config
        self.dtype = config.dtype
        self.injection_dict = config.injection_policy
        self.mp_group = config.tensor_parallel.tp_group
        self.mpu = config.tensor_parallel.mpu
        self.quantize_merge_count = 1
        self.quantization_scales = None
        self.model_profile_enabled = False
        self._model_times = []
        self.cuda_graph_created = False
        self._graphs = {}
        acc = get_accelerator()
        self.device = torch.device(acc.device_name(acc.current_device())) if acc.device_name() != "cpu" \
            else torch.device("cpu")

        tp = config.tensor_parallel.tp_size
        if tp > 1 or (dist.is_initialized() and dist.get_world_size() > 1):
            if not dist.is_initialized():
                dist.init_distributed(dist_backend=acc.communication_backend_name())
        self.tp_size = tp if tp > 1 else 1
        if self.tp_size > 1:
            self._create_model_parallel_group(config)
            self.tp_rank = dist.get_rank(self.mp_group)
        else:
            self.tp_rank = 0

        if config.checkpoint is not None and not isinstance(model, torch.nn.Module):
            raise ValueError("init_inference expects an nn.Module (meta-tensor checkpoint loading: pass the model)")
        if config.checkpoint is not None:
            self._load_client_checkpoint(model, config)

        self.injected = False
        self.encoder_injected = 0
        from ..module_inject import encoder as enc
        if self.injection_dict:
            # user-specified tensor parallelism (reference engine.py:135-154): only the listed blocks are sharded
            if config.replace_with_kernel_inject:
                raise ValueError("Cannot use both user specified injection policy and kernel injection")
            from ..module_inject.auto_tp import AutoTP
            from ..module_inject.policy import DSPolicy
            by_policy = {k: v for k, v in self.injection_dict.items()
                         if isinstance(v, type) and issubclass(v, DSPolicy)}
            by_names = {k: v for k, v in self.injection_dict.items() if k not in by_policy}
            if by_policy:
                # {client layer class: policy class}: every such layer becomes one fused inference layer
                from ..module_inject.containers import replace_layers_with_policy
                model = model.to(self.device)
                self.policy_injected = sum(
                    replace_layers_with_policy(model, layer_cls, policy_cls, config, getattr(model, "config", None))
                    for layer_cls, policy_cls in by_policy.items())
            if by_names:
                AutoTP(model, self.mp_group, self.tp_size, self.tp_rank, injection_policy=by_names).apply()
                self._patch_head_indexed_bias(model)
            self.module = model.to(self.device)
            if self.dtype in (torch.float16, torch.bfloat16, torch.float32):
                self.module = self.module.to(self.dtype)
            self.module.eval()
            log_dist(f"InferenceEngine: user injection policy over {len(self.injection_dict)} block classes, "
                     f"tp={self.tp_size}", ranks=[0])
            return
        if not isinstance(model, torch.nn.Module):
            # diffusers-style pipeline (reference engine.py: generic_injection for non-Module models)
            from ..module_inject.replace_module import generic_injection
            dt = self.dtype if self.dtype in (torch.float16, torch.bfloat16) else None
            self.module = generic_injection(model, dtype=dt, enable_cuda_graph=config.enable_cuda_graph)
            self.pipeline_injected = True  # forward() calls the pipeline itself
            log_dist("InferenceEngine: diffusers pipeline injected (UNet / VAE / text encoder)", ranks=[0])
            return
        if config.replace_with_kernel_inject and not convert.supported(model) and enc.supported(model):
            # bidirectional encoders (BERT family): fused layers swapped in place, HF embeddings / heads kept
            dt = self.dtype if self.dtype in (torch.float16, torch.bfloat16, torch.float32) else torch.bfloat16
            self.encoder_injected = enc.inject(model, self.mp_group, self.tp_size, self.tp_rank, dt, self.device)
            self.module = model
        elif (config.replace_with_kernel_inject or _is_native(model)) and convert.supported(model):
            self.module = convert.from_model(model, self.mp_group, self.tp_size, self.tp_rank, self.dtype, self.device,
                                             max_positions=config.max_out_tokens)
            self.injected = True
            if config.quant.enabled and config.quant.weight.enabled:
                self.module.quantize_weights(config.quant.weight.num_bits, config.quant.weight.group_size)
            else:
                self._apply_decode_layout(config)
            del model
        else:
            if self.tp_size > 1:
                from ..module_inject.auto_tp import AutoTP
                AutoTP(model, self.mp_group, self.tp_size, self.tp_rank).apply()
                self._patch_head_indexed_bias(model)
            self.module = model.to(self.device)
            if self.dtype in (torch.float16, torch.bfloat16, torch.float32):
                self.module = self.module.to(self.dtype)
        self.module.eval()
        log_dist(f"InferenceEngine: injected={self.injected} tp={self.tp_size} dtype={self.dtype}", ranks=[0])

    # ---- models whose attention bias is indexed by head: after the heads are divided over the TP ranks the
    # model's own builder must return this rank's heads only (reference `inference/engine.py:105-110, 214-236`)
    def _patch_head_indexed_bias(self, model):
        if self.tp_size <= 1:
            return
        from ..module_inject.auto_tp_model_utils import set_tp_group
        set_tp_group(self.mp_group, self.tp_size, self.tp_rank)
        self.module = model
        self.build_alibi_tensor()
        self.build_attn_bias()

    def remove_mask_prepare_for_bloom(self):
        """Old HF BLOOM expands the padding mask itself; the fused layers take the [batch, seq] mask as it is."""
        tr = getattr(self.module, "transformer", None)
        if tr is not None and hasattr(tr, "_prepare_attn_mask"):
            tr._prepare_attn_mask = lambda attention_mask, *args, **kwargs: attention_mask

    def build_alibi_tensor(self):
        from ..module_inject import auto_tp_model_utils as U
        tr = getattr(self.module, "transformer", None)
        if tr is not None and hasattr(tr, "build_alibi_tensor"):            # BLOOM
            tr.build_alibi_tensor = U.build_bloom_alibi_tensor
        if tr is not None and hasattr(tr, "build_mpt_alibi_tensor"):        # MPT
            tr.build_mpt_alibi_tensor_orig = tr.build_mpt_alibi_tensor
            type(tr).build_mpt_alibi_tensor = U.build_mpt_alibi_tensor
        inner = getattr(self.module, "model", None)
        if inner is not None and hasattr(inner, "get_alibi_mask"):          # Baichuan
            inner.get_alibi_mask_orig = inner.get_alibi_mask
            type(inner).get_alibi_mask = U.get_alibi_mask

    def build_attn_bias(self):
        from ..module_inject import auto_tp_model_utils as U
        tr = getattr(self.module, "transformer", None)
        if tr is not None and hasattr(tr, "_attn_bias"):                    # MPT (remote-code versions)
            tr._attn_bias_orig = tr._attn_bias
            type(tr)._attn_bias = U.build_mpt_atten_bias_tensor

    def _apply_decode_layout(self, config):
        """`decode_layout` of the inference config: a shuffled copy of the bf16 projection weights for batched
        decode when it is asked for, or ("auto") when it costs less than a quarter of the device memory."""
        mode = getattr(config, "decode_layout", "auto")
        m = self.module
        if mode == "row_major" or self.dtype != torch.bfloat16 or self.device.type != "cuda" or self.tp_size != 1 \
                or not hasattr(m, "add_decode_layout"):
            return
        if mode == "shuffled":
            m.quantize_weights(16)
            return
        if mode == "auto":
            total = torch.cuda.get_device_properties(self.device).total_memory
            if m.projection_bytes() > total // 4:
                return
        n = m.add_decode_layout()
        log_dist(f"InferenceEngine: {n} layers keep a shuffled decode copy of their projection weights "
                 f"({m.projection_bytes() / 2**30:.1f} GiB extra)", ranks=[0])

    @classmethod
    def from_ds_model(cls, ds_model: DSInferenceModel, config: DeepSpeedInferenceConfig, tp_group=None, tp_size=1,
                      tp_rank=0):
        """Wrap an already-built injected model (hybrid engine, benchmarks) without re-converting weights."""
        eng = cls.__new__(cls)
        torch.nn.Module.__init__(eng)
        eng._config, eng.dtype, eng.injected, eng.module = config, ds_model.dtype, True, ds_model
        eng.device = ds_model.device if ds_model.device is not None else torch.device("cpu")
        eng._graphs, eng.cuda_graph_created, eng.model_profile_enabled, eng._model_times = {}, False, False, []
        eng.tp_size, eng.tp_rank, eng.mp_group, eng.mpu = tp_size, tp_rank, tp_group, None
        eng.injection_dict = None
        return eng

    def _load_client_checkpoint(self, model, config):
        """`checkpoint=` JSON / dict (reference `inference/engine.py:400-418,441-503`): HF-layout shard lists
        (`bloom`, `ds_model`) stream into the (possibly meta-device) client model file by file before injection;
        Megatron `mp_rank_*` lists are merged / split to this job's tensor-parallel degree and loaded into the
        client model's module."""
        from ..runtime.state_dict_factory import AUTO_MODULE_KEY, SDLoaderFactory, load_hf_shards
        desc = SDLoaderFactory.get_sd_loader_json(config.checkpoint)
        if isinstance(desc, dict):
            keys = load_hf_shards(model, desc, base_dir=config.base_dir or "")
            log_dist(f"InferenceEngine: loaded {len(keys)} tensors from {desc['type']} checkpoint", ranks=[0])
            return
        # int8 serving quantises after injection (DSInferenceModel.quantize_weights, pre-shuffled for the int8
        # kernels), so the checkpoint loads in its stored precision here
        _, sd, _ = desc.load(self.tp_size, self.tp_rank, module_key=AUTO_MODULE_KEY)
        module_sd = sd[desc._choose_module_key(sd)]
        model.load_state_dict(module_sd, strict=False, assign=any(p.is_meta for p in model.parameters()))
        log_dist(f"InferenceEngine: Megatron checkpoint ({len(desc.ckpt_list)} files) loaded at tp={self.tp_size}",
                 ranks=[0])

    # ------------------------------------------------------------------------------------------ groups
    def _create_model_parallel_group(self, config):
        if self.mpu is not None:
            self.mp_group = self.mpu.get_model_parallel_group()
        elif self.mp_group is None:
            world, rank, tp = dist.get_world_size(), dist.get_rank(), self.tp_size
            assert world % tp == 0, f"world {world} not divisible by tp {tp}"
            for start in range(0, world, tp):
                ranks = list(range(start, start + tp))
                g = dist.new_group(ranks)
                if rank in ranks:
                    self.mp_group = g
        InferenceEngine.inference_mp_group = self.mp_group

    # ------------------------------------------------------------------------------------------ profiling
    def profile_model_time(self, use_cuda_events=True):
        self.model_profile_enabled = True

    def model_times(self):
        out, self._model_times = self._model_times, []
        return out

    # ------------------------------------------------------------------------------------------ helpers
    def _cache_for(self, total_tokens_per_seq, batch):
        bs = self._config.kv_block_size
        per_seq = (total_tokens_per_seq + bs - 1) // bs
        need = per_seq * batch
        c = self.module.cache
        if c is None or c.num_blocks < need or c.block_size != bs:
            self.module.allocate_cache(max(need, per_seq * min(self._config.max_batch_size, batch * 2)), bs)
            self._graphs.clear()
        return per_seq

    def _meta(self, block_tables, starts, n_new, max_len):
        dev = self.device
        st = torch.tensor(starts, dtype=torch.int32, device=dev)
        pos = (st[:, None] + torch.arange(n_new, dtype=torch.int32, device=dev)[None, :]).reshape(-1)
        return BatchMeta(block_tables=block_tables, start_pos=st, seq_lens=st + n_new, pos_ids=pos.contiguous(),
                         n_new=n_new, max_len=max_len, prefill_from_zero=all(s == 0 for s in starts))

    @staticmethod
    def _unpad(input_ids, attention_mask):
        rows = []
        for b in range(input_ids.shape[0]):
            ids = input_ids[b]
            if attention_mask is not None:
                ids = ids[attention_mask[b].bool()]
            rows.append(ids)
        return rows

    # ------------------------------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        start = time.time() if self.model_profile_enabled else None
        if not self.injected:
            out = self.module(*inputs, **kwargs)
        else:
            input_ids = inputs[0] if inputs else kwargs["input_ids"]
            out = GenerationOutput(self._full_logits(input_ids.to(self.device), kwargs.get("attention_mask")))
        if start is not None:
            get_accelerator().synchronize()
            self._model_times.append(time.time() - start)
        return out

    @torch.no_grad()
    def _full_logits(self, input_ids, attention_mask=None):
        B, S = input_ids.shape
        per_seq = self._cache_for(S, B)
        alloc = self.module.cache.allocator
        blocks = alloc.allocate(per_seq * B)
        try:
            bt = torch.tensor(blocks, dtype=torch.int32, device=self.device).view(B, per_seq)
            if attention_mask is None or bool(attention_mask.all()):
                meta = self._meta(bt, [0] * B, S, S)
                return self.module(input_ids, meta, all_logits=True)
            V = self.module.spec.vocab_size
            out = torch.zeros(B, S, V, dtype=self.dtype, device=self.device)
            for b, ids in enumerate(self._unpad(input_ids, attention_mask)):
                meta = self._meta(bt[b:b + 1], [0], ids.numel(), ids.numel())
                lg = self.module(ids[None], meta, all_logits=True)[0]
                out[b, attention_mask[b].bool()] = lg
            return out
        finally:
            alloc.free(blocks)

    # ------------------------------------------------------------------------------------------ generate
    def _sample(self, logits, do_sample, temperature, top_k, top_p, generator):
        if not do_sample:
            return logits.argmax(-1)
        logits = logits.float() / max(temperature, 1e-5)
        if top_k and top_k > 0:
            kth = torch.topk(logits, min(top_k, logits.shape[-1]), dim=-1).values[..., -1:]
            logits = logits.masked_fill(logits < kth, float("-inf"))
        if top_p is not None and top_p < 1.0:
            srt, idx = torch.sort(logits, descending=True, dim=-1)
            cum = srt.softmax(-1).cumsum(-1)
            drop = cum - srt.softmax(-1) > top_p
            srt = srt.masked_fill(drop, float("-inf"))
            logits = torch.full_like(logits, float("-inf")).scatter(-1, idx, srt)
        probs = logits.softmax(-1)
        return torch.multinomial(probs, 1, generator=generator).squeeze(-1)

    def _moe_capturable(self, ids):
        """MoE layers capture only on the device routing path (the reference fallback reads counts on the host)."""
        if not self.module.spec.num_experts:
            return True
        from ..ops import moe_ops
        probe = torch.empty(ids.shape[0], self.module.spec.hidden_size, dtype=self.dtype, device=self.device)
        return all(moe_ops.native_moe_ok(probe, l.router_w, l.fc1_w, l.fc2_w, l.spec.moe_top_k)
                   for l in self.module.layers)

    def _decode_step(self, ids, bt, lens, max_len):
        """One decode step for every sequence (ids [B, 1]); uses a captured HIP graph when enabled."""
        B = ids.shape[0]
        graphable = (self._config.enable_cuda_graph and self.device.type == "cuda" and self.dtype == torch.bfloat16
                     and self.module.spec.head_dim in (64, 128, 256) and self._moe_capturable(ids))
        if not graphable:  # the gather-based fallback attention syncs with the host and cannot be captured
            meta = self._meta(bt, lens, 1, max_len)
            return self.module(ids, meta)
        key = (B, bt.shape[1])
        g = self._graphs.get(key)
        st = torch.tensor(lens, dtype=torch.int32, device=self.device)
        if g is None:
            static = dict(ids=ids.clone(), bt=bt.clone(), st=st.clone())
            cap = bt.shape[1] * self.module.cache.block_size

            def run():
                meta = BatchMeta(block_tables=static["bt"], start_pos=static["st"], seq_lens=static["st"] + 1,
                                 pos_ids=static["st"], n_new=1, max_len=cap, prefill_from_zero=False)
                return self.module(static["ids"], meta)

            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                run()  # warm up allocations / library handles outside capture
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                static["out"] = run()
            g = self._graphs[key] = (graph, static)
            self.cuda_graph_created = True
        graph, static = g
        static["ids"].copy_(ids)
        static["bt"].copy_(bt)
        static["st"].copy_(st)
        graph.replay()
        return static["out"]

    @torch.no_grad()
    def generate(self, input_ids=None, attention_mask=None, max_new_tokens=None, max_length=None, do_sample=False,
                 temperature=1.0, top_k=0, top_p=1.0, eos_token_id=None, pad_token_id=None, seed=None, **kwargs):
        if not self.injected:
            return self.module.generate(input_ids=input_ids, attention_mask=attention_mask,
                                        max_new_tokens=max_new_tokens, max_length=max_length, do_sample=do_sample,
                                        **kwargs)
        input_ids = input_ids.to(self.device)
        B, S = input_ids.shape
        if max_new_tokens is None:
            max_new_tokens = (max_length - S) if max_length else self._config.max_out_tokens - S
        max_new_tokens = max(int(max_new_tokens), 0)
        if attention_mask is not None:
            attention_mask = attention_mask.to(self.device)
        rows = self._unpad(input_ids, attention_mask)
        lens = [int(r.numel()) for r in rows]
        total = max(lens) + max_new_tokens
        per_seq = self._cache_for(total, B)
        alloc = self.module.cache.allocator
        blocks = alloc.allocate(per_seq * B)
        gen = None
        if do_sample:
            gen = torch.Generator(device=self.device)
            gen.manual_seed(seed if seed is not None else int(torch.initial_seed()) % (2**31))
        eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
        pad = pad_token_id if pad_token_id is not None else (next(iter(eos)) if eos else 0)
        try:
            bt = torch.tensor(blocks, dtype=torch.int32, device=self.device).view(B, per_seq)
            # prefill (one batched launch when all prompts have the same length)
            if len(set(lens)) == 1:
                meta = self._meta(bt, [0] * B, lens[0], lens[0])
                logits = self.module(torch.stack(rows), meta)
            else:
                logits = torch.cat([
                    self.module(rows[b][None], self._meta(bt[b:b + 1], [0], lens[b], lens[b]))
                    for b in range(B)
                ])
            out_tokens = []
            done = torch.zeros(B, dtype=torch.bool, device=self.device)
            eos_t = torch.tensor(sorted(eos), device=self.device) if eos else None
            cur = list(lens)
            max_len = per_seq * self.module.cache.block_size
            for step in range(max_new_tokens):
                nxt = self._sample(logits, do_sample, temperature, top_k, top_p, gen)
                nxt = torch.where(done, torch.full_like(nxt, pad), nxt)
                out_tokens.append(nxt)
                if eos_t is not None:
                    done = done | torch.isin(nxt, eos_t)
                    if (step & 15) == 15 and bool(done.all()):
                        break
                if step == max_new_tokens - 1:
                    break
                logits = self._decode_step(nxt[:, None].contiguous(), bt, cur, max_len)
                cur = [c + 1 for c in cur]
        finally:
            alloc.free(blocks)
        if not out_tokens:
            return input_ids
        gen_ids = torch.stack(out_tokens, 1).to(input_ids.dtype)
        return torch.cat([input_ids, gen_ids], 1)

    def _generate(self, *args, **kwargs):
        return self.generate(*args, **kwargs)

    def destroy(self):
        self._graphs.clear()
        if self.injected:
            self.module.cache = None


def _is_native(model):
    from ..models.llama import LlamaForCausalLM
    return isinstance(model, LlamaForCausalLM)
