"""Host-side pieces of the small-head attention kernel: the numpy Philox keep mask the GPU test checks the kernel
against, the fp32 oracle, and the BERT layer's per-key mask detection (no GPU needed)."""
import torch

from deepspeedsyclsupport_amd.ops import flash_small as FS
from deepspeedsyclsupport_amd.ops.transformer.transformer import _per_key_mask


def test_keep_mask_rate_and_determinism():
    k = FS.keep_mask(7, 2, 3, 130, 0.1)
    assert k.shape == (2, 3, 130, 130)
    assert abs(k.float().mean().item() - 0.9) < 0.01
    assert torch.equal(k, FS.keep_mask(7, 2, 3, 130, 0.1))
    agree = FS.keep_mask(8, 2, 3, 130, 0.1).eq(k).float().mean().item()
    assert abs(agree - 0.82) < 0.02   # independent streams for different seeds
    assert FS.keep_mask(1, 1, 1, 64, 0.0).all()


def test_reference_matches_sdpa_with_biases():
    torch.manual_seed(0)
    Z, S, H, D = 4, 20, 2, 8
    q, k, v = (torch.randn(Z, S, H, D) for _ in range(3))
    b1, b2 = torch.randn(Z, S), torch.randn(2, H, S, S)
    out = FS.reference(q, k, v, b1, b2, b2_div=2)
    mask = b1[:, None, None, :] + b2.repeat_interleave(2, 0)
    ref = torch.nn.functional.scaled_dot_product_attention(*(t.transpose(1, 2) for t in (q, k, v)), attn_mask=mask)
    torch.testing.assert_close(out, ref.transpose(1, 2), rtol=1e-5, atol=1e-5)


def test_per_key_mask_forms():
    B, S = 2, 6
    m = torch.randn(B, 1, 1, S)
    assert torch.equal(_per_key_mask(m, B, S), m[:, 0, 0])
    assert torch.equal(_per_key_mask(m[:, 0], B, S), m[:, 0, 0])
    assert _per_key_mask(m[:, 0, 0], B, S) is not None
    assert _per_key_mask(torch.randn(B, 1, S, S), B, S) is None   # full [S, S] masks take the SDPA path
    assert _per_key_mask(None, B, S) is None
