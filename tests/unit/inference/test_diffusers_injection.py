"""Diffusers pipeline injection (reference `module_inject/replace_module.py:generic_injection`, `containers/unet.py`,
`containers/vae.py`, `model_implementations/diffusers/{unet,vae}.py`). diffusers is not installed here: the modules
below re-implement the diffusers classes the policies match (Attention with AttnProcessor2_0 math, GEGLU
FeedForward, BasicTransformerBlock, a UNet2DConditionModel / AutoencoderKL skeleton) under the same class names,
so injection is checked against the unmodified modules' outputs (parity with real diffusers checkpoints unpinned)."""
import copy
import types

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


class Attention(nn.Module):

    def __init__(self, query_dim, cross_attention_dim=None, heads=4, dim_head=16, bias=False, norm_num_groups=None,
                 residual_connection=False, rescale_output_factor=1.0):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.scale = heads, dim_head**-0.5
        self.is_cross_attention = cross_attention_dim is not None
        cad = cross_attention_dim or query_dim
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(cad, inner, bias=bias)
        self.to_v = nn.Linear(cad, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(0.0)])
        self.group_norm = nn.GroupNorm(norm_num_groups, query_dim, eps=1e-6) if norm_num_groups else None
        self.spatial_norm = None
        self.norm_cross = None
        self.residual_connection, self.rescale_output_factor = residual_connection, rescale_output_factor

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None):
        residual = hidden_states
        nd = hidden_states.ndim
        if nd == 4:
            B, C, H, W = hidden_states.shape
            hidden_states = hidden_states.view(B, C, H * W).transpose(1, 2)
        if self.group_norm is not None:
            hidden_states = self.group_norm(hidden_states.transpose(1, 2)).transpose(1, 2)
        ctx = hidden_states if encoder_hidden_states is None else encoder_hidden_states
        q, k, v = self.to_q(hidden_states), self.to_k(ctx), self.to_v(ctx)
        b = q.shape[0]
        q, k, v = (t.view(b, -1, self.heads, t.shape[-1] // self.heads).transpose(1, 2) for t in (q, k, v))
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attention_mask, scale=self.scale)
        o = self.to_out[1](self.to_out[0](o.transpose(1, 2).reshape(b, -1, q.shape[1] * q.shape[-1])))
        if nd == 4:
            o = o.transpose(-1, -2).reshape(B, C, H, W)
        if self.residual_connection:
            o = o + residual
        return o / self.rescale_output_factor


class GEGLU(nn.Module):

    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        h, gate = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(gate)


class FeedForward(nn.Module):

    def __init__(self, dim, mult=4):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, dim * mult), nn.Dropout(0.0), nn.Linear(dim * mult, dim)])

    def forward(self, x):
        for m in self.net:
            x = m(x)
        return x


class BasicTransformerBlock(nn.Module):

    def __init__(self, dim, heads, dim_head, cross_dim):
        super().__init__()
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(dim), nn.LayerNorm(dim), nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads=heads, dim_head=dim_head)
        self.attn2 = Attention(dim, cross_attention_dim=cross_dim, heads=heads, dim_head=dim_head)
        self.ff = FeedForward(dim)
        self.only_cross_attention = False
        self.pos_embed = None

    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None, **kwargs):
        h = self.attn1(self.norm1(hidden_states)) + hidden_states
        h = self.attn2(self.norm2(h), encoder_hidden_states=encoder_hidden_states) + h
        return self.ff(self.norm3(h)) + h


class UNet2DConditionModel(nn.Module):

    def __init__(self, C=128, heads=2, dim_head=64, cross_dim=96):
        super().__init__()
        self.in_channels = 4
        self.config = types.SimpleNamespace(in_channels=4, sample_size=16)
        self.conv_in = nn.Conv2d(4, C, 3, padding=1)
        self.temb = nn.Linear(1, C)
        self.block = BasicTransformerBlock(C, heads, dim_head, cross_dim)
        self.norm_out = nn.GroupNorm(8, C)
        self.conv_out = nn.Conv2d(C, 4, 3, padding=1)

    def forward(self, sample, timestep, encoder_hidden_states, return_dict=True):
        B = sample.shape[0]
        t = timestep.reshape(-1, 1).to(sample.dtype).expand(B, 1)
        x = self.conv_in(sample) + self.temb(t)[:, :, None, None]
        _, C, H, W = x.shape
        tok = self.block(x.flatten(2).transpose(1, 2), encoder_hidden_states=encoder_hidden_states)
        x = tok.transpose(1, 2).reshape(B, C, H, W)
        out = self.conv_out(F.silu(self.norm_out(x)))
        return types.SimpleNamespace(sample=out) if return_dict else (out, )


class AutoencoderKL(nn.Module):

    def __init__(self, C=64):
        super().__init__()
        self.config = types.SimpleNamespace(scaling_factor=0.18215)
        self.post_quant = nn.Conv2d(4, C, 1)
        self.mid_attn = Attention(C, heads=1, dim_head=C, bias=True, norm_num_groups=8, residual_connection=True)
        self.out = nn.Conv2d(C, 3, 3, padding=1)
        self.enc = nn.Conv2d(3, 4, 3, padding=1)

    def decode(self, z, return_dict=True):
        x = self.out(self.mid_attn(self.post_quant(z)))
        return types.SimpleNamespace(sample=x) if return_dict else (x, )

    def encode(self, x, return_dict=True):
        return types.SimpleNamespace(latent=self.enc(x))


class TextEncoder(nn.Module):

    def __init__(self, dim=96):
        super().__init__()
        self.emb = nn.Embedding(100, dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, ids):
        return (self.proj(self.emb(ids)), )


class Pipeline:

    def __init__(self):
        torch.manual_seed(0)
        self.unet = UNet2DConditionModel()
        self.vae = AutoencoderKL()
        self.text_encoder = TextEncoder()
        self.scheduler = object()


def _inputs(dtype, device, seed=1):
    g = torch.Generator().manual_seed(seed)
    sample = torch.randn(2, 4, 16, 16, generator=g).to(device, dtype)
    ehs = torch.randn(2, 77, 96, generator=g).to(device, dtype)
    z = torch.randn(1, 4, 8, 8, generator=g).to(device, dtype)
    return sample, torch.tensor(10.0, device=device), ehs, z


def test_generic_injection_replaces_and_matches_cpu():
    from deepspeedsyclsupport_amd.module_inject import diffusers as DI
    from deepspeedsyclsupport_amd.module_inject.replace_module import generic_injection
    pipe = Pipeline()
    ref = copy.deepcopy(pipe)
    m = nn.Linear(2, 2)
    assert generic_injection(m) is m                       # plain modules pass through
    with pytest.raises(ValueError):
        generic_injection(Pipeline(), dtype=torch.float32)  # half-precision kernels only
    generic_injection(pipe, dtype=None, enable_cuda_graph=False)
    assert isinstance(pipe.unet, DI.DSUNet) and isinstance(pipe.vae, DI.DSVAE)
    assert isinstance(pipe.text_encoder, DI.DSClipEncoder)
    assert isinstance(pipe.unet.unet.block, DI.DSDiffusersTransformerBlock)
    assert isinstance(pipe.vae.vae.mid_attn, DI.DSDiffusersAttention)
    assert pipe.unet.in_channels == 4 and pipe.unet.dtype == torch.float32
    sample, t, ehs, z = _inputs(torch.float32, "cpu")
    with torch.no_grad():
        got = pipe.unet(sample, t, ehs).sample
        want = ref.unet(sample, t, ehs).sample
        torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(pipe.vae.decode(z).sample, ref.vae.decode(z).sample, rtol=1e-4, atol=1e-5)
        ids = torch.randint(0, 100, (2, 7))
        torch.testing.assert_close(pipe.text_encoder(ids)[0], ref.text_encoder(ids)[0])


@pytest.mark.gpu
def test_generic_injection_gpu_kernels_and_graphs():
    from deepspeedsyclsupport_amd.module_inject import diffusers as DI
    from deepspeedsyclsupport_amd.ops import flash_small as FS
    pipe = Pipeline()
    ref = copy.deepcopy(pipe)
    for mod in (pipe.unet, pipe.vae, pipe.text_encoder):
        mod.to("cuda", torch.bfloat16)
    for mod in (ref.unet, ref.vae, ref.text_encoder):
        mod.to("cuda")
    DI.inject_pipeline(pipe, dtype=torch.bfloat16, enable_cuda_graph=True)
    calls = []
    orig = FS.FlashSmallFunc.apply

    def spy(*a):
        calls.append(a[0].shape)
        return orig(*a)

    FS.FlashSmallFunc.apply = spy
    try:
        for seed in (1, 2, 3):  # first call captures, later ones replay the graph with new inputs
            sample, t, ehs, z = _inputs(torch.bfloat16, "cuda", seed)
            with torch.no_grad():
                got = pipe.unet(sample, t, ehs).sample.float().clone()
                want = ref.unet(sample.float(), t, ehs.float()).sample
                assert ((got - want).abs().max() / want.abs().max()).item() < 4e-2, seed
                dec = pipe.vae.decode(z).sample.float().clone()
                dref = ref.vae.decode(z.float()).sample
                assert ((dec - dref).abs().max() / dref.abs().max()).item() < 4e-2, seed
    finally:
        FS.FlashSmallFunc.apply = orig
    assert calls, "self / cross attention did not run on the flash_small kernel"
    assert any(s[1] == 256 for s in calls)  # 16x16 tokens (captured once; replays do not re-enter Python)
    assert len(pipe.unet._graphed.graphs) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["key_bool", "key_additive_3d", "per_query_shared", "per_query_batch"])
def test_masked_attention_runs_on_the_kernel(kind):
    """An attention mask no longer sends the injected Attention to the library path: padding masks travel as the
    kernel's per-key bias, per-(query, key) masks as its pair bias. Checked against the module's own fp32 math."""
    from deepspeedsyclsupport_amd.module_inject import diffusers as DI
    from deepspeedsyclsupport_amd.ops import flash_small as FS
    torch.manual_seed(0)
    B, Nq, Nk, heads, dh = 2, 96, 77, 4, 64
    attn = Attention(128, cross_attention_dim=96, heads=heads, dim_head=dh, bias=True).cuda()
    ds = DI.DSDiffusersAttention(copy.deepcopy(attn)).to(torch.bfloat16)
    x = torch.randn(B, Nq, 128, device="cuda")
    ctx = torch.randn(B, Nk, 96, device="cuda")
    g = torch.Generator().manual_seed(2)
    if kind == "key_bool":
        mask = torch.ones(B, 1, 1, Nk, dtype=torch.bool)
        mask[0, ..., 50:] = False
        mask[1, ..., 9:] = False
    elif kind == "key_additive_3d":
        mask = torch.zeros(B, 1, Nk)
        mask[0, :, 60:] = -1e4
        mask = mask.expand(B, Nq, Nk)  # expanded over queries with stride 0, as diffusers' prepare_attention_mask does
    elif kind == "per_query_shared":
        mask = torch.randn(1, 1, Nq, Nk, generator=g)
    else:
        mask = torch.randn(B, heads, Nq, Nk, generator=g)
    mask = mask.cuda()
    ref_mask = mask if mask.dim() == 4 else mask[:, None]
    calls = []
    orig = FS.FlashSmallFunc.apply

    def spy(*a):
        calls.append((a[3] is not None, a[4] is not None))
        return orig(*a)

    FS.FlashSmallFunc.apply = spy
    try:
        with torch.no_grad():
            got = ds(x.bfloat16(), encoder_hidden_states=ctx.bfloat16(), attention_mask=mask).float()
            want = attn(x, encoder_hidden_states=ctx, attention_mask=ref_mask)
    finally:
        FS.FlashSmallFunc.apply = orig
    assert calls == [(kind.startswith("key"), not kind.startswith("key"))]
    assert ((got - want).abs().max() / want.abs().max()).item() < 3e-2
