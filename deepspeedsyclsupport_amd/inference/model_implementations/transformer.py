"""Kernel-injected inference transformer (reference v1 `model_implementations/transformers/ds_transformer.py`,
`ops/transformer/inference/{ds_attention.py, ds_mlp.py}` and the v2 model implementations).

One decoder-layer implementation parametrised by `DSModelSpec` covers the architectures the reference injects
(Llama/Llama-2/Mistral/Qwen2, GPT-2, BLOOM, OPT, GPT-NeoX): norm type, positional scheme (rotary-half, rotary
GPT-J, ALiBi, learned), gated or plain MLP, biases, parallel residual. Hot path per layer:
  fused (residual +) norm -> QKV GEMM (hipBLASLt) -> RoPE (HIP) -> KV append into the blocked cache (HIP) ->
  attention: prefill = SDPA, decode = paged flash-decoding kernel (HIP) -> O GEMM -> TP all-reduce ->
  fused residual + norm -> MLP GEMM -> fused gated activation (HIP) -> GEMM -> TP all-reduce.
Tensor parallelism is column-parallel QKV/FC1 (sharded by heads / intermediate), row-parallel O/FC2 with one RCCL
all-reduce each (bias added once after it), vocab-parallel LM head with an all-gather of logits.
Weight-only int8/int4 quantisation keeps group-quantised weights and dequantises into a per-layer workspace.
"""
import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import comm as dist
from ...ops import reference
from ...ops import moe_ops
from ...ops.transformer import functional as DF


@dataclass
class DSModelSpec:
    arch: str
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    intermediate_size: int
    head_dim: int = 0
    norm: str = "rms"                # "rms" | "ln"
    norm_eps: float = 1e-5
    pos: str = "rope"                # "rope" | "rope_gptj" | "alibi" | "learned" | "none"
    rope_theta: float = 10000.0
    rotary_dim: int = 0
    act: str = "silu"                # activation name (ACT_CODES)
    gated_mlp: bool = True
    qkv_bias: bool = False
    o_bias: bool = False
    mlp_bias: bool = False
    parallel_residual: bool = False
    shared_parallel_norm: bool = False  # GPT-J style single norm for attn+mlp
    embed_norm: bool = False         # BLOOM word_embeddings_layernorm
    final_norm: bool = True
    tie_embeddings: bool = False
    max_positions: int = 4096
    learned_pos_offset: int = 0      # OPT uses 2
    sliding_window: int = 0
    layer_windows: tuple = ()        # per-layer sliding windows (GPT-Neo local/global layers); () -> sliding_window
    attn_scale: float = 0.0          # softmax scale; 0 -> 1/sqrt(head_dim) (GPT-Neo uses 1.0)
    lm_head_bias: bool = False
    num_experts: int = 0             # > 0: MoE MLP (Mixtral-style top-k router over gated experts)
    moe_top_k: int = 2
    moe_renormalize: bool = True     # renormalise the top-k routing weights to sum to 1
    moe_residual: bool = False       # PR-MoE: softmax(coefficient(x)) mixes the routed experts with a dense MLP

    def __post_init__(self):
        if not self.head_dim:
            self.head_dim = self.hidden_size // self.num_heads
        if not self.rotary_dim:
            self.rotary_dim = self.head_dim


SKINNY_MAX_ROWS = 16  # decode batches up to this many token rows use the weight-streaming skinny GEMM kernels


def _skinny_rows_ok(m, *ks):
    """Rows <= 8 run on the VALU GEMV for any K % 8 == 0; 9..16 need the MFMA kernel (every K % 256 == 0)."""
    if m <= 8:
        return all(k % 8 == 0 for k in ks)
    return m <= SKINNY_MAX_ROWS and all(k % 256 == 0 for k in ks)


def alibi_slopes(n_heads):
    closest = 2**math.floor(math.log2(n_heads))
    base = 2**(-(2**-(math.log2(closest) - 3)))
    slopes = [base**i for i in range(1, closest + 1)]
    if closest != n_heads:
        extra_base = 2**(-(2**-(math.log2(2 * closest) - 3)))
        n_rem = min(closest, n_heads - closest)
        slopes += [extra_base**i for i in range(1, 2 * n_rem + 1, 2)]
    return torch.tensor(slopes, dtype=torch.float32)


class QuantLinearWeight:
    """Decode-layout weight. Group-quantised (int8 / int4): symmetric int8 with K a multiple of 64 and int4 with K a
    multiple of 128 are kept in MFMA operand order for the decode streams (`ops/int8_gemv.py`, `ops/int4_gemv.py`);
    everything else is dequantised into a temporary right before its GEMM. bits=16: the bf16 weight itself re-laid in
    operand order (`ops/bf16_gemv.py`), with or without a row-major copy for prefill (`group_size` < 0: keep one).
    `i8` holds whichever stream object applies."""

    def __init__(self, w, bits=8, group_size=64):
        from ...ops.bf16_gemv import Bf16Weight
        from ...ops.int4_gemv import Int4Weight
        from ...ops.int8_gemv import Int8Weight
        from ...ops.quantizer import quantize
        self.shape = w.shape
        self.dtype = w.dtype
        self.i8 = None
        if bits == 16:
            if not Bf16Weight.supported(w):
                raise ValueError(f"bf16 decode layout needs a bf16 [N, K] weight with K % 64 == 0, got {tuple(w.shape)}")
            self.i8 = Bf16Weight(w, keep_row_major=group_size < 0)
            self.qt = None
            return
        if Int8Weight.supported(w, bits, group_size):
            self.i8 = Int8Weight(w, group_size)
        elif Int4Weight.supported(w, bits, group_size):
            self.i8 = Int4Weight(w, group_size)
        self.qt = None if self.i8 is not None else \
            quantize(w, group_size=min(group_size, w.numel()), bits=bits, symmetric=True)

    def materialize(self):
        if self.i8 is not None:
            return self.i8.materialize()
        from ...ops.quantizer import dequantize
        return dequantize(self.qt, self.dtype)


def _weight(w):
    return w.materialize() if isinstance(w, QuantLinearWeight) else w


def materialize(h):
    """A layer of the weight-only decode path returns its output still in the GEMV workspace (`PendingAcc`); anything
    other than the next such layer's input norm takes the plain tensor."""
    return h.finalize() if hasattr(h, "finalize_rms") else h


@dataclass
class BatchMeta:
    block_tables: torch.Tensor       # [B, max_blocks] int32 (device)
    start_pos: torch.Tensor          # [B] int32 tokens already cached
    seq_lens: torch.Tensor           # [B] int32 = start_pos + n_new
    pos_ids: torch.Tensor            # [B*n_new] int32 absolute positions
    n_new: int
    max_len: int                     # host upper bound of seq_lens (kernel split sizing)
    prefill_from_zero: bool          # every sequence starts at position 0 (pure prefill)


@dataclass
class RaggedMeta:
    """One ragged batch (inference v2 `put()`): the new tokens of every sequence concatenated, decode sequences (one
    token each) first, then prompt / chunk sequences. Device tensors come from ONE packed host->device copy
    (`RaggedMeta.build`); the host lists are kept so no step needs a device->host sync."""
    block_tables: torch.Tensor       # [S, max_blocks] int32
    start_pos: torch.Tensor          # [S] tokens cached before this step
    seq_lens: torch.Tensor           # [S] start + new
    pos_ids: torch.Tensor            # [T] absolute position (= cache slot) of every token
    seq_ids: torch.Tensor            # [T] sequence of every token
    cu_q: torch.Tensor               # [S + 1] token offsets
    work: torch.Tensor               # [W, 2] (sequence, 128-row query block) for the prefill sequences
    last_idx: torch.Tensor           # [S] row of each sequence's last token
    n_decode: int                    # sequences [0, n_decode) are single-token decodes
    cu_host: List[int]
    start_host: List[int]
    max_len: int                     # host upper bound of seq_lens (decode split sizing)
    block_size: int

    @staticmethod
    def build(starts, n_new, block_lists, n_decode, block_size, device):
        S = len(starts)
        cu = [0]
        for n in n_new:
            cu.append(cu[-1] + n)
        T = cu[-1]
        width = max(1, max(len(b) for b in block_lists))
        pos, sid = [], []
        for i, (st, n) in enumerate(zip(starts, n_new)):
            pos.extend(range(st, st + n))
            sid.extend([i] * n)
        work = [(i, qb) for i in range(n_decode, S) for qb in range(-(-n_new[i] // 128))]
        bt = []
        for b in block_lists:
            bt.extend(list(b) + [0] * (width - len(b)))
        lens = [st + n for st, n in zip(starts, n_new)]
        last = [c - 1 for c in cu[1:]]
        flat = pos + sid + list(starts) + lens + cu + [x for w in work for x in w] + last + bt
        buf = torch.tensor(flat, dtype=torch.int32)
        if device is not None and torch.device(device).type == "cuda":
            buf = buf.pin_memory().to(device, non_blocking=True)
        views, o = [], 0
        for n in (T, T, S, S, S + 1, 2 * len(work), S, S * width):
            views.append(buf[o:o + n])
            o += n
        pos_t, sid_t, st_t, len_t, cu_t, work_t, last_t, bt_t = views
        return RaggedMeta(block_tables=bt_t.view(S, width), start_pos=st_t, seq_lens=len_t, pos_ids=pos_t,
                          seq_ids=sid_t, cu_q=cu_t, work=work_t.view(-1, 2), last_idx=last_t.long(),
                          n_decode=n_decode, cu_host=cu, start_host=list(starts), max_len=width * block_size,
                          block_size=block_size)


class DSInferenceLayer(nn.Module):

    def __init__(self, spec: DSModelSpec, layer_idx: int, tp_group=None, tp_size=1, dtype=torch.bfloat16,
                 device=None):
        super().__init__()
        self.spec = spec
        self.layer_idx = layer_idx
        self.tp_group = tp_group
        self.tp = tp_size
        assert spec.num_heads % tp_size == 0, "heads must divide tp size"
        self.hq = spec.num_heads // tp_size
        self.hk = max(spec.num_kv_heads // tp_size, 1)
        D = spec.head_dim
        H = spec.hidden_size
        I = spec.intermediate_size // tp_size
        kw = dict(dtype=dtype, device=device)
        self.ln1_w = nn.Parameter(torch.ones(H, **kw), requires_grad=False)
        self.ln1_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False) if spec.norm == "ln" else None
        self.ln2_w = nn.Parameter(torch.ones(H, **kw), requires_grad=False)
        self.ln2_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False) if spec.norm == "ln" else None
        self.qkv_w = nn.Parameter(torch.empty((self.hq + 2 * self.hk) * D, H, **kw), requires_grad=False)
        self.qkv_b = nn.Parameter(torch.zeros((self.hq + 2 * self.hk) * D, **kw), requires_grad=False) \
            if spec.qkv_bias else None
        self.o_w = nn.Parameter(torch.empty(H, self.hq * D, **kw), requires_grad=False)
        self.o_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False) if spec.o_bias else None
        G = 2 if spec.gated_mlp else 1
        E = spec.num_experts
        if E:  # experts stacked [E, ...] and sharded by intermediate (TP) like a dense MLP; router replicated
            self.router_w = nn.Parameter(torch.empty(E, H, **kw), requires_grad=False)
            self.fc1_w = nn.Parameter(torch.empty(E, G * I, H, **kw), requires_grad=False)
            self.fc2_w = nn.Parameter(torch.empty(E, H, I, **kw), requires_grad=False)
        else:
            self.router_w = None
            self.fc1_w = nn.Parameter(torch.empty(G * I, H, **kw), requires_grad=False)
            self.fc2_w = nn.Parameter(torch.empty(H, I, **kw), requires_grad=False)
        if E:  # per-expert biases (Megatron-style experts); fc2's is pre-divided by the TP degree (summed back)
            self.fc1_b = nn.Parameter(torch.zeros(E, G * I, **kw), requires_grad=False) if spec.mlp_bias else None
            self.fc2_b = nn.Parameter(torch.zeros(E, H, **kw), requires_grad=False) if spec.mlp_bias else None
        else:
            self.fc1_b = nn.Parameter(torch.zeros(G * I, **kw), requires_grad=False) if spec.mlp_bias else None
            self.fc2_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False) if spec.mlp_bias else None
        if E and spec.moe_residual:  # dense MLP beside the experts + the 2-way mixing coefficient
            self.res_fc1_w = nn.Parameter(torch.empty(G * I, H, **kw), requires_grad=False)
            self.res_fc1_b = nn.Parameter(torch.zeros(G * I, **kw), requires_grad=False)
            self.res_fc2_w = nn.Parameter(torch.empty(H, I, **kw), requires_grad=False)
            self.res_fc2_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False)
            self.coef_w = nn.Parameter(torch.empty(2, H, **kw), requires_grad=False)
            self.coef_b = nn.Parameter(torch.zeros(2, **kw), requires_grad=False)
        self.quant = {}
        # bf16 weights ALSO held in the shuffled decode layout (name -> Bf16Weight), next to the row-major parameters:
        # decode steps of SH_MIN_ROWS..16 token rows stream these, everything else uses the parameters
        self.sh = {}
        # split (aliased) projections: name -> list of weights / biases applied side by side (hybrid engine shares
        # the training module's separate q/k/v and gate/up tensors instead of fusing copies)
        self.split_w, self.split_b = {}, {}

    # ------------------------------------------------------------------------------------------ helpers
    def quantize_weights(self, bits=8, group_size=64):
        self.sh = {}
        for name in ("qkv_w", "o_w") + (() if self.spec.num_experts else ("fc1_w", "fc2_w")):
            self.quant[name] = QuantLinearWeight(getattr(self, name).data, bits, group_size)
            getattr(self, name).data = torch.empty(0, dtype=getattr(self, name).dtype,
                                                   device=getattr(self, name).device)

    SH_MIN_ROWS = 2  # measured on Llama-2-7B: the row-major stream wins at 1 token row, the shuffled one from 2 up

    def add_decode_layout(self):
        """Keep a second copy of the four projection weights in MFMA operand order (`ops/bf16_gemv.py`): twice the
        weight memory — 288 GB of HBM is sized for it — for up to 1.2x on batched decode steps (2 - 16 token rows). No-op
        for quantised, split or non-bf16 weights."""
        from ...ops.bf16_gemv import Bf16Weight
        if self.quant or self.split_w or self.spec.num_experts:
            return False
        ws = {n: getattr(self, n) for n in ("qkv_w", "o_w", "fc1_w", "fc2_w")}
        if not all(w.is_cuda and Bf16Weight.supported(w.data) for w in ws.values()):
            return False
        self.sh = {n: Bf16Weight(w.data) for n, w in ws.items()}
        return True

    def _linear(self, x, name, bias=None):
        """x . W^T (+ bias). Int8 weight-only layers run `Int8Weight.linear`: at decode sizes (<= 16 token rows) the
        fused-dequant MFMA stream over the pre-shuffled weight (`csrc/gemv/skinny_int8.hip`, never materialises a
        bf16 weight); larger batches dequantise into a bf16 temporary for a library GEMM (reference
        `ds_vector_matmul_int8`)."""
        if name in self.split_w:
            bs = self.split_b.get(name) or [None] * len(self.split_w[name])
            return torch.cat([F.linear(x, w, b) for w, b in zip(self.split_w[name], bs)], -1)
        qw = self.quant.get(name)
        if qw is not None and qw.i8 is not None:
            return qw.i8.linear(x, bias)
        return F.linear(x, self._w(name), bias)

    def _w(self, name):
        return self.quant[name].materialize() if name in self.quant else getattr(self, name)

    def _norm(self, x, w, b, residual=None):
        if self.spec.norm == "rms":
            return DF.rms_norm(x, w, self.spec.norm_eps, residual)
        return DF.layer_norm(x, w, b, self.spec.norm_eps, residual)

    def _allreduce(self, x):
        if self.tp > 1:
            dist.inference_all_reduce(x, group=self.tp_group)
        return x

    # ------------------------------------------------------------------------------------------ attention
    def _attend(self, qkv, meta: BatchMeta, cache, rope, alibi):
        """qkv [B, n, (Hq+2Hk)*D] -> attention output [B, n, Hq*D] (RoPE + cache append + prefill/decode attention)."""
        if isinstance(meta, RaggedMeta):
            return self._attend_ragged(qkv, meta, cache, rope, alibi)
        spec = self.spec
        pending = qkv if hasattr(qkv, "finalize_rms") else None  # un-finalized weight-only GEMV (PendingAcc)
        if pending is not None and not (pending.acc.is_cuda and cache.k[self.layer_idx].dtype == torch.bfloat16):
            qkv, pending = pending.finalize(), None
        B, n, D = (pending.lead[0] if pending is not None else qkv.shape[0]), meta.n_new, spec.head_dim
        kc, vc = cache.k[self.layer_idx], cache.v[self.layer_idx]
        k = v = None
        scale = spec.attn_scale or 1.0 / math.sqrt(D)
        window = spec.layer_windows[self.layer_idx] if spec.layer_windows else spec.sliding_window
        # ALiBi / windowed prompts and chunk continuations: ragged paged flash prefill over the cache
        # (head dims other than 128 always take it: the dense flash forward is a 128-wide kernel)
        paged = n > 1 and D in PAGED_HEAD_DIMS and (pending is not None or (qkv.is_cuda and
                                                                             qkv.dtype == torch.bfloat16)) \
            and kc.dtype == torch.bfloat16 and (not meta.prefill_from_zero or alibi is not None or bool(window)
                                                or D != 128)
        if pending is not None or (qkv.is_cuda and qkv.dtype == torch.bfloat16 and kc.dtype == torch.bfloat16):
            # one fused HIP epilogue: split + RoPE(q, k) + scatter k/v into the paged cache (and, for a pending
            # weight-only GEMV, its finalize pass: the sums are read straight from the split-K workspace)
            from ...ops.native import hip_ops
            rot = spec.rotary_dim if spec.pos in ("rope", "rope_gptj") else 0
            want_kv = meta.prefill_from_zero and n > 1 and not paged
            src = pending._take() if pending is not None else qkv.contiguous()
            outs = hip_ops().qkv_rope_append(src, rope[0] if rot else None, rope[1] if rot else None,
                                             meta.pos_ids, kc, vc, meta.block_tables, meta.start_pos, n, self.hq,
                                             self.hk, rot, spec.pos == "rope_gptj", want_kv, None,
                                             pending.M if pending is not None else 0,
                                             pending.bias if pending is not None else None)
            q = outs[0].view(B, n, self.hq, D)
            if want_kv:
                k, v = outs[1].view(B, n, self.hk, D), outs[2].view(B, n, self.hk, D)
        else:
            q, k, v = qkv.view(B, n, self.hq + 2 * self.hk, D).split([self.hq, self.hk, self.hk], dim=2)
            q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
            if spec.pos in ("rope", "rope_gptj"):
                inter = spec.pos == "rope_gptj"
                pos = meta.pos_ids.view(B, n)
                DF.apply_rotary_pos_emb(q, rope[0], rope[1], position_ids=pos, rotary_dim=spec.rotary_dim,
                                        interleaved=inter)
                DF.apply_rotary_pos_emb(k, rope[0], rope[1], position_ids=pos, rotary_dim=spec.rotary_dim,
                                        interleaved=inter)
            _kv_append(k, v, kc, vc, meta)
        if n == 1:
            o = _decode_attention(q.view(B, self.hq, D), kc, vc, meta, scale, alibi, window)
        elif paged:
            o = _paged_attention_uniform(q, kc, vc, meta, scale, alibi, window)
        elif meta.prefill_from_zero:
            o = _prefill_attention(q, k, v, scale, alibi, window)
        else:
            o = _cached_attention(q, kc, vc, meta, scale, alibi, window)
        return o.reshape(B, n, self.hq * D)

    def _attend_ragged(self, qkv, meta: "RaggedMeta", cache, rope, alibi):
        """Ragged batch: qkv [1, T, (Hq+2Hk)*D] -> [1, T, Hq*D]. One fused epilogue (RoPE + paged-cache append) for
        all tokens, then the paged decode kernel for the leading single-token sequences and the ragged paged
        flash-prefill kernel for the prompt / chunk sequences (`csrc/attn/paged_prefill.hip`)."""
        spec = self.spec
        T, D = meta.cu_host[-1], spec.head_dim
        kc, vc = cache.k[self.layer_idx], cache.v[self.layer_idx]
        rot = spec.rotary_dim if spec.pos in ("rope", "rope_gptj") else 0
        inter = spec.pos == "rope_gptj"
        pending = qkv if hasattr(qkv, "finalize_rms") else None
        if pending is not None and not (pending.acc.is_cuda and kc.dtype == torch.bfloat16):
            qkv, pending = pending.finalize(), None
        if pending is not None or (qkv.is_cuda and qkv.dtype == torch.bfloat16 and kc.dtype == torch.bfloat16):
            from ...ops.native import hip_ops
            src = pending._take() if pending is not None else qkv.reshape(T, -1).contiguous()
            q = hip_ops().qkv_rope_append(src, rope[0] if rot else None,
                                          rope[1] if rot else None, meta.pos_ids, kc, vc, meta.block_tables,
                                          meta.start_pos, 1, self.hq, self.hk, rot, inter, False, meta.seq_ids,
                                          pending.M if pending is not None else 0,
                                          pending.bias if pending is not None else None)[0]
        else:
            q, k, v = qkv.reshape(1, T, self.hq + 2 * self.hk, D).split([self.hq, self.hk, self.hk], dim=2)
            q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
            if rot:
                pos = meta.pos_ids.view(1, T)
                DF.apply_rotary_pos_emb(q, rope[0], rope[1], position_ids=pos, rotary_dim=rot, interleaved=inter)
                DF.apply_rotary_pos_emb(k, rope[0], rope[1], position_ids=pos, rotary_dim=rot, interleaved=inter)
            _kv_append_ragged(k[0], v[0], kc, vc, meta)
            q = q[0]
        scale = spec.attn_scale or 1.0 / math.sqrt(D)
        window = spec.layer_windows[self.layer_idx] if spec.layer_windows else spec.sliding_window
        return _ragged_attention(q, kc, vc, meta, scale, alibi, window).reshape(1, T, self.hq * D)

    def _attention(self, x, meta: BatchMeta, cache, rope, alibi):
        qkv = self._linear(x, "qkv_w", self.qkv_b)
        out = self._linear(self._attend(qkv, meta, cache, rope, alibi), "o_w")
        out = self._allreduce(out)
        if self.o_b is not None:
            out = out + self.o_b
        return out

    def _act(self, h):
        if self.spec.gated_mlp:
            return DF.gated_activation(h, self.spec.act)
        return DF.bias_activation(h, None, self.spec.act)

    def _moe(self, x):
        """Top-k routed experts (reference v2 `modules/implementations/moe/cutlass_multi_gemm.py` +
        `kernels/ragged_ops/top_k_gating`): fp32 softmax router -> top-k -> expert-contiguous scatter -> grouped
        MFMA GEMM pair -> weighted gather, all on device without a host sync (`ops/moe_ops.py`). Experts are
        TP-sharded along the intermediate dim, so one all-reduce finishes the block exactly like a dense MLP."""
        out = moe_ops.moe_block(x, self.router_w, self.fc1_w, self.fc2_w, self.spec.moe_top_k, self._act,
                                self.spec.moe_renormalize, fc1_b=self.fc1_b, fc2_b=self.fc2_b)
        if self.spec.moe_residual:
            # PR-MoE (reference `ops/transformer/inference/moe_inference.py:300-330`, `moe_res_matmul`): the dense
            # branch is TP-sharded like the experts, so both are summed by the one all-reduce below
            dense = F.linear(self._act(F.linear(x, self.res_fc1_w, self.res_fc1_b)), self.res_fc2_w)
            coef = torch.softmax(F.linear(x, self.coef_w, self.coef_b).float(), -1).to(x.dtype)
            out = self._allreduce(out * coef[..., 0:1] + dense * coef[..., 1:2])
            return out + self.res_fc2_b * coef[..., 1:2]
        return self._allreduce(out)

    def _mlp(self, x):
        if self.spec.num_experts:
            return self._moe(x)
        h = self._linear(x, "fc1_w", self.fc1_b)
        if self.spec.gated_mlp:
            h = DF.gated_activation(h, self.spec.act)
        else:
            h = DF.bias_activation(h, None, self.spec.act)
        out = self._linear(h, "fc2_w")
        out = self._allreduce(out)
        if self.fc2_b is not None:
            out = out + self.fc2_b
        return out

    # ------------------------------------------------------------------------------------------ decode fast path
    def _skinny_ok(self, h):
        spec = self.spec
        return (h.is_cuda and h.dtype == torch.bfloat16 and not self.quant and not self.split_w and spec.norm == "rms"
                and not spec.parallel_residual and not spec.num_experts and _skinny_rows_ok(h.numel() // h.shape[-1], spec.hidden_size,
                                                                    spec.intermediate_size // self.tp,
                                                                    self.hq * spec.head_dim))

    def _forward_skinny(self, h, residual, meta, cache, rope, alibi):
        """Decode (<= 8 token rows): 4 weight-streaming GEMVs with RMSNorm / residual / gated activation fused into
        their input stage, plus the fused QKV epilogue and the paged decode attention."""
        from ...ops.native import hip_ops
        from ...ops.transformer.functional import ACT_CODES
        ops, eps, tp1 = hip_ops(), self.spec.norm_eps, self.tp == 1
        res1 = torch.empty_like(h)
        qkv = ops.skinny_gemm(h, self.qkv_w, self.qkv_b, None, 1, False, 0, residual, self.ln1_w, eps, res1)
        attn = self._attend(qkv, meta, cache, rope, alibi)
        o = ops.skinny_gemm(attn, self.o_w, self.o_b if tp1 else None, None, 0, False, 0, None, None, 0.0, None)
        if not tp1:
            o = self._allreduce(o)
            if self.o_b is not None:
                o = o + self.o_b
        res2 = torch.empty_like(h)
        if self.spec.gated_mlp:  # gate/up rows paired in-kernel: writes act(gate) * up directly
            mid = ops.skinny_gemm(o, self.fc1_w, self.fc1_b, None, 1, True, ACT_CODES[self.spec.act], res1,
                                  self.ln2_w, eps, res2)
        else:
            mid = DF.bias_activation(
                ops.skinny_gemm(o, self.fc1_w, self.fc1_b, None, 1, False, 0, res1, self.ln2_w, eps, res2), None,
                self.spec.act)
        down = ops.skinny_gemm(mid, self.fc2_w, self.fc2_b if tp1 else None, None, 0, False, 0, None, None, 0.0, None)
        if not tp1:
            down = self._allreduce(down)
            if self.fc2_b is not None:
                down = down + self.fc2_b
        return down, res2

    # ------------------------------------------------------------------------------ weight-only decode fast path
    def _streams(self, h):
        """{projection name: weight-stream object} serving this input through the un-finalized decode GEMVs, or None:
        the quantised / shuffled-only weights, or the extra shuffled copies for SH_MIN_ROWS..16 token rows."""
        spec = self.spec
        if (not self.quant and not self.sh) or self.split_w or spec.norm != "rms" or spec.parallel_residual \
                or spec.num_experts or self.tp != 1:
            return None
        from ...ops.int8_gemv import PendingAcc, raw_ok
        names = ("qkv_w", "o_w", "fc1_w", "fc2_w")
        if self.quant:
            if not all(self.quant.get(n) is not None and self.quant[n].i8 is not None for n in names):
                return None
            q = {n: self.quant[n].i8 for n in names}
            return q if isinstance(h, PendingAcc) or raw_ok(h) else None
        if isinstance(h, PendingAcc):
            return self.sh
        rows = h.numel() // h.shape[-1]
        return self.sh if raw_ok(h) and rows >= self.SH_MIN_ROWS else None

    def _quant_skinny_ok(self, h):
        return self._streams(h) is not None

    def _forward_quant_skinny(self, h, residual, meta, cache, rope, alibi):
        """Decode (<= 16 token rows) over int8 / int4 weights: the four weight streams leave their sums in the fp32
        split-K workspace and the op that consumes each projection anyway — residual add + RMSNorm after the
        attention-output and MLP-down projections, the gated activation after gate/up, the RoPE + cache-append
        epilogue after QKV — converts and re-zeroes it (`csrc/gemv/skinny_finalize.hip`, `csrc/attn/decode_attn.hip`).
        The block output is returned still pending: the next layer's input norm consumes it."""
        from ...ops.int8_gemv import PendingAcc
        from ...ops.transformer.functional import ACT_CODES
        eps, q = self.spec.norm_eps, self._streams(h)
        if isinstance(h, PendingAcc):
            normed, res1 = h.finalize_rms(residual, self.ln1_w, eps)
        elif residual is None:
            normed, res1 = self._norm(h, self.ln1_w, None), h
        else:
            normed, res1 = self._norm(h, self.ln1_w, None, residual)
        # the fused QKV epilogue (RoPE + cache append) consumes the projection's sums straight from the workspace
        attn = self._attend(q["qkv_w"].raw(normed, self.qkv_b), meta, cache, rope, alibi)
        normed2, res2 = q["o_w"].raw(attn, self.o_b).finalize_rms(res1, self.ln2_w, eps)
        up = q["fc1_w"].raw(normed2, self.fc1_b)
        if self.spec.gated_mlp:
            mid = up.finalize_gated(ACT_CODES[self.spec.act])
        else:
            mid = DF.bias_activation(up.finalize(), None, self.spec.act)
        return q["fc2_w"].raw(mid, self.fc2_b), res2

    def forward(self, h, residual, meta, cache, rope, alibi):
        """Pre-norm block. Returns (block_output, residual) where the caller adds them (fused in the next norm)."""
        if self._quant_skinny_ok(h):
            return self._forward_quant_skinny(h, residual, meta, cache, rope, alibi)
        h = materialize(h)
        if self._skinny_ok(h):
            return self._forward_skinny(h, residual, meta, cache, rope, alibi)
        if self.spec.parallel_residual:
            x = h if residual is None else h + residual
            a_in = self._norm(x, self.ln1_w, self.ln1_b)
            m_in = a_in if self.spec.shared_parallel_norm else self._norm(x, self.ln2_w, self.ln2_b)
            out = self._attention(a_in, meta, cache, rope, alibi) + self._mlp(m_in)
            return out, x
        if residual is None:
            normed, residual = self._norm(h, self.ln1_w, self.ln1_b), h
        else:
            normed, residual = self._norm(h, self.ln1_w, self.ln1_b, residual)
        attn = self._attention(normed, meta, cache, rope, alibi)
        normed, residual = self._norm(attn, self.ln2_w, self.ln2_b, residual)
        return self._mlp(normed), residual


# ------------------------------------------------------------------------------------------------ attention impls
def _kv_append(k, v, kc, vc, meta):
    if k.is_cuda and kc.dtype == torch.bfloat16:
        from ...ops.native import hip_ops
        hip_ops().kv_append(k, v, kc, vc, meta.block_tables, meta.start_pos)
        return
    B, n, Hk, D = k.shape
    BS = kc.shape[2]
    for b in range(B):
        s0 = int(meta.start_pos[b])
        for j in range(n):
            t = s0 + j
            blk = int(meta.block_tables[b, t // BS])
            kc[blk, :, t % BS] = k[b, j]
            vc[blk, :, t % BS] = v[b, j]


def _alibi_bias(alibi, q_pos, k_len, device):
    # bias[h, i, j] = slope_h * (j - q_pos_i)
    kpos = torch.arange(k_len, device=device, dtype=torch.float32)
    return alibi.to(device)[:, None, None] * (kpos[None, None, :] - q_pos.float()[None, :, None])


def _prefill_attention(q, k, v, scale, alibi, window):
    """q,k,v [B, n, H, D] -> [B, n, Hq, D]; causal."""
    B, n, Hq, D = q.shape
    qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if alibi is None and not window:
        from ...ops.attention import attention
        return attention(qh, kh, vh, causal=True, softmax_scale=scale).transpose(1, 2)
    pos = torch.arange(n, device=q.device)
    mask = torch.zeros(Hq if alibi is not None else 1, n, n, device=q.device, dtype=torch.float32)
    if alibi is not None:
        mask = mask + _alibi_bias(alibi, pos, n, q.device)
    causal = pos[None, :] > pos[:, None]
    if window:
        causal = causal | (pos[None, :] <= pos[:, None] - window)
    mask = mask.masked_fill(causal[None], float("-inf")).to(q.dtype)
    if kh.shape[1] != Hq:
        rep = Hq // kh.shape[1]
        kh, vh = kh.repeat_interleave(rep, 1), vh.repeat_interleave(rep, 1)
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask[None], scale=scale)
    return o.transpose(1, 2)


def _gather_kv(kc, vc, meta, b, L):
    BS = kc.shape[2]
    nblk = (L + BS - 1) // BS
    ids = meta.block_tables[b, :nblk].long()
    k = kc[ids].transpose(0, 1).reshape(kc.shape[1], nblk * BS, kc.shape[3])[:, :L]
    v = vc[ids].transpose(0, 1).reshape(vc.shape[1], nblk * BS, vc.shape[3])[:, :L]
    return k, v


def _cached_attention(q, kc, vc, meta, scale, alibi, window):
    """General path (chunked prefill / non-bf16 decode): gather each sequence's cache and run SDPA."""
    B, n, Hq, D = q.shape
    outs = []
    seq_lens = meta.seq_lens.tolist()
    starts = meta.start_pos.tolist()
    for b in range(B):
        L = seq_lens[b]
        k, v = _gather_kv(kc, vc, meta, b, L)
        rep = Hq // k.shape[0]
        if rep > 1:
            k, v = k.repeat_interleave(rep, 0), v.repeat_interleave(rep, 0)
        qpos = torch.arange(starts[b], starts[b] + n, device=q.device)
        kpos = torch.arange(L, device=q.device)
        bad = kpos[None, :] > qpos[:, None]
        if window:
            bad = bad | (kpos[None, :] <= qpos[:, None] - window)
        mask = torch.zeros(Hq if alibi is not None else 1, n, L, device=q.device, dtype=torch.float32)
        if alibi is not None:
            mask = mask + _alibi_bias(alibi, qpos, L, q.device)
        mask = mask.masked_fill(bad[None], float("-inf")).to(q.dtype)
        o = F.scaled_dot_product_attention(q[b].transpose(0, 1).unsqueeze(0), k.unsqueeze(0), v.unsqueeze(0),
                                           attn_mask=mask.unsqueeze(0), scale=scale)
        outs.append(o[0].transpose(0, 1))
    return torch.stack(outs, 0)


PAGED_HEAD_DIMS = (64, 80, 96, 128, 256)  # instantiations of the paged prefill / decode kernels
_UNIFORM_TABLES = {}


def _uniform_tables(B, n, device):
    """(cu_q, work) of a uniform batch: every layer of every prefill with this (batch, length) shares one device
    copy, so the per-call host table build and H2D copy are paid once."""
    key = (B, n, str(device))
    hit = _UNIFORM_TABLES.get(key)
    if hit is None:
        nqb = -(-n // 128)
        seq = torch.arange(B, dtype=torch.int32).repeat_interleave(nqb)
        qb = torch.arange(nqb, dtype=torch.int32).repeat(B)
        if len(_UNIFORM_TABLES) > 256:
            _UNIFORM_TABLES.clear()
        hit = _UNIFORM_TABLES[key] = (torch.arange(0, (B + 1) * n, n, dtype=torch.int32).to(device),
                                      torch.stack([seq, qb], 1).contiguous().to(device))
    return hit


def _paged_attention_uniform(q, kc, vc, meta, scale, alibi, window):
    """Uniform batch (v1 engine): q [B, n, Hq, D] at positions start..start+n-1 per sequence -> [B, n, Hq, D]
    through the ragged paged flash-prefill kernel (K/V of the new tokens are already in the cache)."""
    from ...ops.native import hip_ops
    B, n, Hq, D = q.shape
    cu, work = _uniform_tables(B, n, q.device)
    o = hip_ops().paged_prefill(q.reshape(B * n, Hq, D).contiguous(), kc, vc, meta.block_tables, meta.start_pos, cu,
                                work, alibi, window, scale)
    return o.view(B, n, Hq, D)


def _kv_append_ragged(k, v, kc, vc, meta):
    """Host / non-bf16 path: k, v [T, Hk, D] into the paged cache at each token's (sequence, position)."""
    BS = kc.shape[2]
    slots = meta.pos_ids.long()
    blk = meta.block_tables.long()[meta.seq_ids.long(), slots // BS]
    kc[blk, :, slots % BS] = k.to(kc.dtype)
    vc[blk, :, slots % BS] = v.to(vc.dtype)


def _ragged_attention(q, kc, vc, meta, scale, alibi, window):
    """q [T, Hq, D] -> [T, Hq, D] over the paged cache (new tokens already appended)."""
    T, Hq, D = q.shape
    nd, S = meta.n_decode, len(meta.start_host)
    fast = q.is_cuda and q.dtype == torch.bfloat16 and kc.dtype == torch.bfloat16
    from ...ops.native import hip_ops
    if fast and D in PAGED_HEAD_DIMS and nd < S:
        out = hip_ops().paged_prefill(q.contiguous(), kc, vc, meta.block_tables, meta.start_pos, meta.cu_q, meta.work,
                                      alibi, window, scale)
    else:
        out = torch.empty_like(q)
        for i in range(nd, S):
            a, b = meta.cu_host[i], meta.cu_host[i + 1]
            out[a:b] = _seq_cached_attention(q[a:b], kc, vc, meta, i, scale, alibi, window)
    if nd:
        if fast and D in PAGED_HEAD_DIMS:
            out[:nd] = hip_ops().paged_decode(q[:nd].contiguous(), kc, vc, meta.block_tables[:nd], meta.seq_lens[:nd],
                                              meta.max_len, scale, alibi, window)
        else:
            for i in range(nd):
                out[i:i + 1] = _seq_cached_attention(q[i:i + 1], kc, vc, meta, i, scale, alibi, window)
    return out


def _seq_cached_attention(q, kc, vc, meta, i, scale, alibi, window):
    """Reference path for one ragged sequence: q [n, Hq, D] at positions start..start+n-1 over its cached keys."""
    n, Hq, D = q.shape
    st = meta.start_host[i]
    L = st + n
    BS = kc.shape[2]
    nblk = -(-L // BS)
    ids = meta.block_tables[i, :nblk].long()
    k = kc[ids].transpose(0, 1).reshape(kc.shape[1], nblk * BS, D)[:, :L]
    v = vc[ids].transpose(0, 1).reshape(vc.shape[1], nblk * BS, D)[:, :L]
    rep = Hq // k.shape[0]
    if rep > 1:
        k, v = k.repeat_interleave(rep, 0), v.repeat_interleave(rep, 0)
    qpos = torch.arange(st, L, device=q.device)
    kpos = torch.arange(L, device=q.device)
    bad = kpos[None, :] > qpos[:, None]
    if window:
        bad = bad | (kpos[None, :] <= qpos[:, None] - window)
    mask = torch.zeros(Hq if alibi is not None else 1, n, L, device=q.device, dtype=torch.float32)
    if alibi is not None:
        mask = mask + _alibi_bias(alibi, qpos, L, q.device)
    mask = mask.masked_fill(bad[None], float("-inf")).to(q.dtype)
    o = F.scaled_dot_product_attention(q.transpose(0, 1).unsqueeze(0), k.unsqueeze(0).to(q.dtype),
                                       v.unsqueeze(0).to(q.dtype), attn_mask=mask.unsqueeze(0), scale=scale)
    return o[0].transpose(0, 1)


def _decode_attention(q, kc, vc, meta, scale, alibi, window):
    if q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in PAGED_HEAD_DIMS:
        from ...ops.native import hip_ops
        return hip_ops().paged_decode(q, kc, vc, meta.block_tables, meta.seq_lens, meta.max_len, scale,
                                      alibi, window)
    B, Hq, D = q.shape
    return _cached_attention(q.view(B, 1, Hq, D), kc, vc, meta, scale, alibi, window).view(B, Hq, D)


# ------------------------------------------------------------------------------------------------ model
class DSInferenceModel(nn.Module):

    def __init__(self, spec: DSModelSpec, tp_group=None, tp_size=1, tp_rank=0, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.spec = spec
        self.tp_group, self.tp_size, self.tp_rank = tp_group, tp_size, tp_rank
        self.dtype = dtype
        self.device = device
        kw = dict(dtype=dtype, device=device)
        H = spec.hidden_size
        self.embed = nn.Parameter(torch.empty(spec.vocab_size, H, **kw), requires_grad=False)
        self.pos_embed = nn.Parameter(torch.empty(spec.max_positions + spec.learned_pos_offset, H, **kw),
                                      requires_grad=False) if spec.pos == "learned" else None
        if spec.embed_norm:
            self.embed_ln_w = nn.Parameter(torch.ones(H, **kw), requires_grad=False)
            self.embed_ln_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False)
        self.layers = nn.ModuleList([DSInferenceLayer(spec, i, tp_group, tp_size, dtype, device)
                                     for i in range(spec.num_layers)])
        self.norm_w = nn.Parameter(torch.ones(H, **kw), requires_grad=False)
        self.norm_b = nn.Parameter(torch.zeros(H, **kw), requires_grad=False) if spec.norm == "ln" else None
        vloc = (spec.vocab_size + tp_size - 1) // tp_size
        self.vocab_local = vloc
        self.lm_head = nn.Parameter(torch.empty(vloc, H, **kw), requires_grad=False)
        self.lm_head_b = nn.Parameter(torch.zeros(vloc, **kw), requires_grad=False) if spec.lm_head_bias else None
        if spec.pos in ("rope", "rope_gptj"):
            cos, sin = reference.rope_tables(max(spec.max_positions, 2048) * 2, spec.rotary_dim, spec.rope_theta,
                                             device=device)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
        else:
            self.rope_cos = self.rope_sin = None
        if spec.pos == "alibi":
            slopes = alibi_slopes(spec.num_heads)
            hq = spec.num_heads // tp_size
            self.register_buffer("alibi", slopes[tp_rank * hq:(tp_rank + 1) * hq].contiguous().to(device),
                                 persistent=False)
        else:
            self.alibi = None
        self.cache = None

    # ------------------------------------------------------------------------------------------ cache
    def allocate_cache(self, num_blocks, block_size=64):
        from ..kv_cache import BlockedKVCache
        hk = max(self.spec.num_kv_heads // self.tp_size, 1)
        self.cache = BlockedKVCache(self.spec.num_layers, num_blocks, hk, block_size, self.spec.head_dim, self.dtype,
                                    self.device)
        return self.cache

    # ------------------------------------------------------------------------------------------ forward
    def _embed(self, input_ids, meta):
        if self.pos_embed is not None:
            # token + learned position rows in one gather kernel (reference `ragged_ops/embed/embed.cu:19`)
            pos = meta.pos_ids.view(input_ids.shape).long() + self.spec.learned_pos_offset
            h = moe_ops.embed_gather(self.embed, input_ids, self.pos_embed, pos).view(*input_ids.shape, -1)
        else:
            h = F.embedding(input_ids, self.embed)
        if self.spec.embed_norm:
            h = DF.layer_norm(h, self.embed_ln_w, self.embed_ln_b, self.spec.norm_eps)
        return h

    def _logits(self, h):
        return self._gather_vocab(F.linear(h, self.lm_head, self.lm_head_b))

    def _gather_vocab(self, logits):
        if self.tp_size > 1:
            parts = [torch.empty_like(logits) for _ in range(self.tp_size)]
            dist.all_gather(parts, logits.contiguous(), group=self.tp_group)
            logits = torch.cat(parts, dim=-1)
        return logits[..., :self.spec.vocab_size]

    @torch.no_grad()
    def forward(self, input_ids, meta: BatchMeta, all_logits=False):
        """input_ids [B, n] -> logits [B, V] of the last new token (or [B, n, V] with all_logits)."""
        h = self._embed(input_ids, meta)
        residual = None
        rope = (self.rope_cos, self.rope_sin)
        for layer in self.layers:
            h, residual = layer(h, residual, meta, self.cache, rope, self.alibi)
        sh = getattr(self, "lm_head_sh", None)
        if sh is not None and not all_logits and hasattr(h, "finalize_rms") and len(h.lead) == 2 and h.lead[1] == 1 \
                and self.spec.final_norm and self.spec.norm == "rms":
            # decode step over the shuffled copies: the last block's sums go through the fused residual + final
            # RMSNorm finalize, then the LM head streams in operand order like every other projection
            normed, _ = h.finalize_rms(residual, self.norm_w, self.spec.norm_eps)
            return self._gather_vocab(sh.linear(normed[:, -1], self.lm_head_b))
        h = materialize(h)
        if not all_logits:
            h = h[:, -1].contiguous()
            residual = residual[:, -1].contiguous() if residual is not None else None
            if (h.is_cuda and h.dtype == torch.bfloat16 and self.spec.final_norm and self.spec.norm == "rms"
                    and _skinny_rows_ok(h.shape[0], self.spec.hidden_size)):
                # final RMSNorm (+ residual) fused into the LM-head GEMV
                from ...ops.native import hip_ops
                logits = hip_ops().skinny_gemm(h, self.lm_head, self.lm_head_b, None, 1, False, 0, residual,
                                               self.norm_w, self.spec.norm_eps, None)
                return self._gather_vocab(logits)
        x = h if residual is None else h + residual
        if self.spec.final_norm:
            if self.spec.norm == "rms":
                x = DF.rms_norm(x, self.norm_w, self.spec.norm_eps)
            else:
                x = DF.layer_norm(x, self.norm_w, self.norm_b, self.spec.norm_eps)
        return self._logits(x)

    @torch.no_grad()
    def forward_ragged(self, tokens, meta: RaggedMeta):
        """tokens [T] (every sequence's new tokens, concatenated as in `meta`) -> logits [S, V] of each sequence's
        last token. One forward for the whole ragged batch (inference v2 `put()`)."""
        ids = tokens.view(1, -1)
        h = self._embed(ids, meta)
        residual = None
        rope = (self.rope_cos, self.rope_sin)
        for layer in self.layers:
            h, residual = layer(h, residual, meta, self.cache, rope, self.alibi)
        h = materialize(h)
        h = h[0].index_select(0, meta.last_idx)
        residual = residual[0].index_select(0, meta.last_idx) if residual is not None else None
        if (h.is_cuda and h.dtype == torch.bfloat16 and self.spec.final_norm and self.spec.norm == "rms"
                and _skinny_rows_ok(h.shape[0], self.spec.hidden_size)):
            from ...ops.native import hip_ops
            logits = hip_ops().skinny_gemm(h, self.lm_head, self.lm_head_b, None, 1, False, 0, residual, self.norm_w,
                                           self.spec.norm_eps, None)
            return self._gather_vocab(logits)
        x = h if residual is None else h + residual
        if self.spec.final_norm:
            if self.spec.norm == "rms":
                x = DF.rms_norm(x, self.norm_w, self.spec.norm_eps)
            else:
                x = DF.layer_norm(x, self.norm_w, self.norm_b, self.spec.norm_eps)
        return self._logits(x)

    def quantize_weights(self, bits=8, group_size=64):
        """Weight-only int8 / int4 (`bits` 8 / 4), or bits=16: bf16 weights kept ONLY in the shuffled decode layout."""
        for layer in self.layers:
            layer.quantize_weights(bits, group_size)

    def add_decode_layout(self):
        """Second, shuffled copy of every layer's projection weights for batched decode (see the layer method);
        returns the number of layers that took one."""
        n = sum(bool(layer.add_decode_layout()) for layer in self.layers)
        from ...ops.bf16_gemv import Bf16Weight
        if n and self.tp_size == 1 and self.lm_head.is_cuda and Bf16Weight.supported(self.lm_head.data):
            self.lm_head_sh = Bf16Weight(self.lm_head.data)  # the LM head streams every decode step too
        return n

    def projection_bytes(self):
        return sum(getattr(layer, n).numel() * getattr(layer, n).element_size()
                   for layer in self.layers for n in ("qkv_w", "o_w", "fc1_w", "fc2_w") if hasattr(layer, n))
