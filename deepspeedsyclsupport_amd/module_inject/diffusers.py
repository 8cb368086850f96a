"""Diffusers injection: Stable-Diffusion-style pipelines (UNet, VAE, CLIP text encoder) on the MI355X kernels.

Reference behaviour: `module_inject/replace_module.py:generic_injection`, the UNet / VAE policies
(`module_inject/containers/{unet,vae}.py`), `model_implementations/diffusers/{unet,vae}.py` (DSUNet / DSVAE: the
whole UNet / VAE forward captured in a CUDA graph) and `ops/transformer/inference/diffusers_{attention,
transformer_block}.py` (fused attention and the fused LayerNorm / GEGLU / bias-add transformer block).

Here (diffusers itself is not required; modules are recognised by class name and attributes):
 * every `Attention` / `CrossAttention` module becomes `DSDiffusersAttention`: one fused QKV GEMM for self-attention
   (Q + fused KV GEMMs for cross-attention), the attention itself on the in-tree flash kernels — head dim 32/64 on
   `csrc/attn/flash_small.hip` (any context length), 128 on `flash_fwd.hip` — and the output projection with its bias
   in the GEMM epilogue; VAE-style 4-D inputs (group norm, residual connection, output rescale) are handled;
 * every `BasicTransformerBlock` with LayerNorms becomes `DSDiffusersTransformerBlock`: LayerNorm kernels with the
   residual adds fused in, GEGLU on the gated-activation kernel (the projection's halves swapped once so the gate
   comes first), the last bias + residual on the bias-add kernel;
 * the UNet / VAE / text encoder are wrapped in `DSUNet` / `DSVAE` / `DSClipEncoder`, which replay one HIP graph per
   input signature (shapes, dtypes and non-tensor arguments) after a warm-up on a side stream.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import flash_small as FS
from ..ops.spatial import nhwc_bias_add_add
from ..ops.transformer import functional as DF

_ATTN_NAMES = ("Attention", "CrossAttention")
_BLOCK_NAMES = ("BasicTransformerBlock", )
_UNET_NAMES = ("UNet2DConditionModel", )
_VAE_NAMES = ("AutoencoderKL", )


def is_attention(m):
    return (type(m).__name__ in _ATTN_NAMES and all(hasattr(m, a) for a in ("to_q", "to_k", "to_v", "to_out", "heads"))
            and getattr(m, "spatial_norm", None) is None and getattr(m, "norm_cross", None) is None
            and getattr(m, "norm_q", None) is None and getattr(m, "add_q_proj", None) is None)


def is_transformer_block(m):
    if type(m).__name__ not in _BLOCK_NAMES:
        return False
    norms = [getattr(m, n, None) for n in ("norm1", "norm2", "norm3")]
    ff = getattr(m, "ff", None)
    if any(not isinstance(n, nn.LayerNorm) for n in norms) or ff is None or not hasattr(ff, "net"):
        return False
    proj = getattr(ff.net[0], "proj", None)
    return (type(ff.net[0]).__name__ == "GEGLU" and isinstance(proj, nn.Linear) and isinstance(ff.net[-1], nn.Linear)
            and getattr(m, "attn2", None) is not None and not getattr(m, "only_cross_attention", False)
            and getattr(m, "pos_embed", None) is None)


def attention_core(q, k, v, heads, scale):
    """q [B, Nq, C], k/v [B, Nk, C] -> [B, Nq, C] on the in-tree kernels where the shape allows."""
    B, Nq, C = q.shape
    Nk, D = k.shape[1], C // heads
    q4, k4, v4 = q.view(B, Nq, heads, D), k.view(B, Nk, heads, D), v.view(B, Nk, heads, D)
    if FS.supported(q4) and k4.dtype == q4.dtype and v4.dtype == q4.dtype and not torch.is_grad_enabled():
        return FS.flash_small(q4, k4, v4, scale=scale).view(B, Nq, C)
    if D == 128 and q.is_cuda and q.dtype == torch.bfloat16:
        from ..ops.attention import attention
        o = attention(q4.transpose(1, 2), k4.transpose(1, 2), v4.transpose(1, 2), causal=False, softmax_scale=scale)
        return o.transpose(1, 2).reshape(B, Nq, C)
    o = F.scaled_dot_product_attention(q4.transpose(1, 2), k4.transpose(1, 2), v4.transpose(1, 2), scale=scale)
    return o.transpose(1, 2).reshape(B, Nq, C)


class DSDiffusersAttention(nn.Module):
    """Fused replacement of a diffusers `Attention` (reference `diffusers_attention.py:97-220`)."""

    def __init__(self, attn):
        super().__init__()
        self.heads = attn.heads
        self.scale = getattr(attn, "scale", None) or (attn.to_q.out_features // attn.heads)**-0.5
        self.cross = attn.to_k.in_features != attn.to_q.in_features or bool(getattr(attn, "is_cross_attention", False))
        qb = [attn.to_q.bias, attn.to_k.bias, attn.to_v.bias]
        self.inner = attn.to_q.out_features
        with torch.no_grad():
            if self.cross:
                self.q_w = nn.Parameter(attn.to_q.weight.detach().clone(), requires_grad=False)
                self.kv_w = nn.Parameter(torch.cat([attn.to_k.weight, attn.to_v.weight]).detach(), requires_grad=False)
                self.q_b = None if qb[0] is None else nn.Parameter(qb[0].detach().clone(), requires_grad=False)
                self.kv_b = None if qb[1] is None else nn.Parameter(torch.cat(qb[1:]).detach(), requires_grad=False)
            else:
                self.qkv_w = nn.Parameter(torch.cat([attn.to_q.weight, attn.to_k.weight, attn.to_v.weight]).detach(),
                                          requires_grad=False)
                self.qkv_b = None if qb[0] is None else nn.Parameter(torch.cat(qb).detach(), requires_grad=False)
            out = attn.to_out[0]
            self.out_w = nn.Parameter(out.weight.detach().clone(), requires_grad=False)
            self.out_b = None if out.bias is None else nn.Parameter(out.bias.detach().clone(), requires_grad=False)
        self.group_norm = getattr(attn, "group_norm", None)
        self.residual_connection = bool(getattr(attn, "residual_connection", False))
        self.rescale_output_factor = float(getattr(attn, "rescale_output_factor", 1.0))

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, context=None, **kwargs):
        ctx = encoder_hidden_states if encoder_hidden_states is not None else context
        residual = hidden_states
        four_d = hidden_states.dim() == 4
        if four_d:
            B, C, Hh, Ww = hidden_states.shape
            hidden_states = hidden_states.reshape(B, C, Hh * Ww).transpose(1, 2)
        if self.group_norm is not None:
            hidden_states = self.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2)
        if self.cross or ctx is not None:
            src = ctx if ctx is not None else hidden_states
            if self.cross:
                q = F.linear(hidden_states, self.q_w, self.q_b)
                k, v = F.linear(src, self.kv_w, self.kv_b).split(self.inner, dim=-1)
            else:  # a self-attention module called with a context: project each side with the fused weight's parts
                w_q, w_kv = self.qkv_w.split([self.inner, 2 * self.inner])
                b_q, b_kv = (None, None) if self.qkv_b is None else self.qkv_b.split([self.inner, 2 * self.inner])
                q = F.linear(hidden_states, w_q, b_q)
                k, v = F.linear(src, w_kv, b_kv).split(self.inner, dim=-1)
        else:
            q, k, v = F.linear(hidden_states, self.qkv_w, self.qkv_b).split(self.inner, dim=-1)
        if attention_mask is not None:
            B_, Nq = q.shape[0], q.shape[1]
            D = self.inner // self.heads
            mask = attention_mask[:, None] if attention_mask.dim() == 3 else attention_mask
            q4, k4, v4 = (t.reshape(B_, t.shape[1], self.heads, D) for t in (q, k, v))
            o = FS.attend(q4, k4, v4, mask=mask, scale=self.scale) if q.is_cuda else None
            if o is None:
                mask = mask if mask.dtype == torch.bool else mask.to(q.dtype)
                o = F.scaled_dot_product_attention(q4.transpose(1, 2), k4.transpose(1, 2), v4.transpose(1, 2),
                                                   attn_mask=mask, scale=self.scale).transpose(1, 2)
            o = o.reshape(B_, Nq, self.inner)
        else:
            o = attention_core(q.contiguous() if q.stride(-1) != 1 else q, k, v, self.heads, self.scale)
        o = F.linear(o, self.out_w, self.out_b)
        if four_d:
            o = o.transpose(-1, -2).reshape(B, C, Hh, Ww)
        if self.residual_connection:
            o = o + residual
        if self.rescale_output_factor != 1.0:
            o = o / self.rescale_output_factor
        return o


class Diffusers2DTransformerConfig:
    """Options of the fused diffusers transformer block (reference `diffusers_2d_transformer.py`)."""

    def __init__(self, int8_quantization=False):
        self.int8_quantization = int8_quantization


class DSDiffusersTransformerBlock(nn.Module):
    """Fused replacement of a LayerNorm `BasicTransformerBlock` (reference `diffusers_transformer_block.py:35-106`):
    LN1 -> self-attention -> (+res, LN2) -> cross-attention -> (+res, LN3) -> GEGLU FF -> (+bias, +res)."""

    def __init__(self, block):
        super().__init__()
        self.attn1 = block.attn1 if isinstance(block.attn1, DSDiffusersAttention) else DSDiffusersAttention(block.attn1)
        self.attn2 = block.attn2 if isinstance(block.attn2, DSDiffusersAttention) else DSDiffusersAttention(block.attn2)
        self.norms = nn.ModuleList([block.norm1, block.norm2, block.norm3])
        proj, out = block.ff.net[0].proj, block.ff.net[-1]
        inner = proj.out_features // 2
        with torch.no_grad():
            # diffusers GEGLU: hidden, gate = proj(x).chunk(2); hidden * gelu(gate). The kernel wants [gate | up].
            w = torch.cat([proj.weight[inner:], proj.weight[:inner]]).detach()
            b = torch.cat([proj.bias[inner:], proj.bias[:inner]]).detach() if proj.bias is not None else None
            self.ff1_w = nn.Parameter(w, requires_grad=False)
            self.ff1_b = None if b is None else nn.Parameter(b, requires_grad=False)
            self.ff2_w = nn.Parameter(out.weight.detach().clone(), requires_grad=False)
            self.ff2_b = nn.Parameter(out.bias.detach().clone() if out.bias is not None else
                                      torch.zeros(out.out_features, dtype=out.weight.dtype,
                                                  device=out.weight.device), requires_grad=False)

    def _ln(self, i, x, residual=None):
        n = self.norms[i]
        return DF.layer_norm(x, n.weight, n.bias, n.eps, residual)

    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None, encoder_attention_mask=None,
                timestep=None, cross_attention_kwargs=None, class_labels=None, context=None, **kwargs):
        ctx = encoder_hidden_states if encoder_hidden_states is not None else context
        a1 = self.attn1(self._ln(0, hidden_states), attention_mask=attention_mask)
        n2, r1 = self._ln(1, a1, residual=hidden_states)
        a2 = self.attn2(n2, encoder_hidden_states=ctx, attention_mask=encoder_attention_mask)
        n3, r2 = self._ln(2, a2, residual=r1)
        g = DF.gated_activation(F.linear(n3, self.ff1_w, self.ff1_b), "gelu")
        return nhwc_bias_add_add(F.linear(g, self.ff2_w), self.ff2_b, r2.contiguous())


def replace_modules(root):
    """Swap attention modules and LayerNorm transformer blocks under `root` in place. Returns the count."""
    n = 0
    for parent in list(root.modules()):
        for name, child in list(parent.named_children()):
            if is_transformer_block(child):
                setattr(parent, name, DSDiffusersTransformerBlock(child))
                n += 1
            elif is_attention(child):
                setattr(parent, name, DSDiffusersAttention(child))
                n += 1
    return n


# ------------------------------------------------------------------------------------------------ graph wrappers
def _signature(args, kwargs):
    def sig(x):
        if torch.is_tensor(x):
            return ("T", tuple(x.shape), x.dtype, x.device)
        if isinstance(x, (list, tuple)):
            return tuple(sig(y) for y in x)
        if isinstance(x, dict):
            return tuple((k, sig(v)) for k, v in sorted(x.items()))
        return ("V", repr(x))
    return (sig(args), sig(kwargs))


def _copy_into(dst, src):
    if torch.is_tensor(dst):
        dst.copy_(src)
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_into(d, s)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])


class GraphedCall:
    """One HIP graph per input signature around `fn` (reference `module_inject/features/cuda_graph.py` + DSUNet's
    `_create_cuda_graph` / `_graph_replay`): three warm-up calls on a side stream, capture with static input
    buffers, then every later call with the same signature copies its tensors in and replays. The outputs are the
    graph's static tensors (overwritten by the next replay), as in the reference."""

    def __init__(self, fn, enabled=True):
        self.fn = fn
        self.enabled = enabled
        self.graphs = {}

    def __call__(self, *args, **kwargs):
        if not self.enabled or not torch.cuda.is_available() or not any(
                torch.is_tensor(a) and a.is_cuda for a in list(args) + list(kwargs.values())):
            return self.fn(*args, **kwargs)
        key = _signature(args, kwargs)
        entry = self.graphs.get(key)
        if entry is None:
            static_args = [a.clone() if torch.is_tensor(a) else a for a in args]
            static_kwargs = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in kwargs.items()}
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side), torch.no_grad():
                for _ in range(3):
                    self.fn(*static_args, **static_kwargs)
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph), torch.no_grad():
                out = self.fn(*static_args, **static_kwargs)
            entry = (graph, static_args, static_kwargs, out)
            self.graphs[key] = entry
        graph, static_args, static_kwargs, out = entry
        _copy_into(static_args, list(args))
        _copy_into(static_kwargs, kwargs)
        graph.replay()
        return out


class DSUNet(nn.Module):
    """UNet wrapper replaying HIP graphs (reference `model_implementations/diffusers/unet.py`)."""

    def __init__(self, unet, enable_cuda_graph=True):
        super().__init__()
        self.unet = unet
        self.in_channels = getattr(unet, "in_channels", None)
        self.config = getattr(unet, "config", None)
        self.unet.requires_grad_(False)
        self._graphed = GraphedCall(self._forward, enable_cuda_graph)

    @property
    def device(self):
        return next(self.unet.parameters()).device

    @property
    def dtype(self):
        return next(self.unet.parameters()).dtype

    def _forward(self, sample, timestep, encoder_hidden_states, *args, **kwargs):
        return self.unet(sample, timestep, encoder_hidden_states, *args, **kwargs)

    def forward(self, sample, timestep, encoder_hidden_states, *args, **kwargs):
        if not torch.is_tensor(timestep):  # python scalars would otherwise be baked into one graph per value
            timestep = torch.tensor(timestep, device=sample.device)
        return self._graphed(sample, timestep, encoder_hidden_states, *args, **kwargs)


class DSVAE(nn.Module):
    """VAE wrapper replaying HIP graphs for decode / encode / forward (reference `diffusers/vae.py`)."""

    def __init__(self, vae, enable_cuda_graph=True):
        super().__init__()
        self.vae = vae
        self.config = getattr(vae, "config", None)
        self.vae.requires_grad_(False)
        self._decode = GraphedCall(lambda *a, **k: self.vae.decode(*a, **k), enable_cuda_graph)
        self._encode = GraphedCall(lambda *a, **k: self.vae.encode(*a, **k), enable_cuda_graph)
        self._forward = GraphedCall(lambda *a, **k: self.vae(*a, **k), enable_cuda_graph)

    @property
    def device(self):
        return next(self.vae.parameters()).device

    @property
    def dtype(self):
        return next(self.vae.parameters()).dtype

    def decode(self, *args, **kwargs):
        return self._decode(*args, **kwargs)

    def encode(self, *args, **kwargs):
        return self._encode(*args, **kwargs)

    def forward(self, *args, **kwargs):
        return self._forward(*args, **kwargs)


class DSClipEncoder(nn.Module):
    """Text-encoder wrapper (reference `model_implementations/transformers/clip_encoder.py`): CLIP layers swapped for
    the fused encoder layer (`module_inject/encoder.py`), the forward replayed from HIP graphs."""

    def __init__(self, enc, enable_cuda_graph=True):
        super().__init__()
        self.enc = enc
        self.config = getattr(enc, "config", None)
        self.enc.requires_grad_(False)
        self._graphed = GraphedCall(lambda *a, **k: self.enc(*a, **k), enable_cuda_graph)

    @property
    def device(self):
        return next(self.enc.parameters()).device

    @property
    def dtype(self):
        return next(self.enc.parameters()).dtype

    def forward(self, *args, **kwargs):
        return self._graphed(*args, **kwargs)


def inject_pipeline(pipe, dtype=None, enable_cuda_graph=True):
    """Diffusers pipeline injection (reference `generic_injection` for non-Module inputs). Returns the number of
    attention modules / transformer blocks replaced."""
    if dtype is not None and dtype not in (torch.float16, torch.bfloat16):
        raise ValueError("generic injection runs the half-precision kernels: dtype must be fp16 or bf16")
    n = 0
    te = getattr(pipe, "text_encoder", None)
    if isinstance(te, nn.Module) and not isinstance(te, DSClipEncoder):
        from . import encoder
        dev = next(te.parameters()).device
        if encoder.supported(te):
            n += encoder.inject(te, dtype=dtype or next(te.parameters()).dtype, device=dev)
        pipe.text_encoder = DSClipEncoder(te, enable_cuda_graph=enable_cuda_graph)
    for name in list(vars(pipe).keys()):
        sub = getattr(pipe, name)
        if not isinstance(sub, nn.Module):
            continue
        cls = type(sub).__name__
        if cls in _UNET_NAMES:
            n += replace_modules(sub)
            setattr(pipe, name, DSUNet(sub, enable_cuda_graph=enable_cuda_graph))
        elif cls in _VAE_NAMES:
            n += replace_modules(sub)
            setattr(pipe, name, DSVAE(sub, enable_cuda_graph=enable_cuda_graph))
    return n
