"""Pre-shuffled int8 weight layout (ops/int8_gemv.py) on the host: lane mapping and exact round trip."""
import pytest
import torch

from deepspeedsyclsupport_amd.ops.int8_gemv import preshuffle, unshuffle


@pytest.mark.parametrize("N,K,gs", [(16, 64, 64), (37, 256, 64), (100, 1024, 128), (3, 192, 64)])
def test_preshuffle_lane_mapping_and_roundtrip(N, K, gs):
    g = torch.Generator().manual_seed(N * K)
    q = torch.randint(-127, 128, (N, K), generator=g).to(torch.int8)
    s = torch.rand(N * K // gs, generator=g)
    qsh, ssh = preshuffle(q, s, gs)
    nb = (N + 15) // 16
    assert qsh.shape == (nb, K // 64, 64, 16) and ssh.shape == (nb, K // gs, 16)
    # lane l of tile (nb, kq) holds row 16 nb + l % 16, columns 64 kq + 16 (l // 16) .. +16
    for _ in range(20):
        b = int(torch.randint(0, nb, (1, ), generator=g))
        kq = int(torch.randint(0, K // 64, (1, ), generator=g))
        lane = int(torch.randint(0, 64, (1, ), generator=g))
        row = 16 * b + lane % 16
        col = 64 * kq + 16 * (lane // 16)
        want = q[row, col:col + 16] if row < N else torch.zeros(16, dtype=torch.int8)
        assert torch.equal(qsh[b, kq, lane], want)
        grp = (64 * kq) // gs
        want_s = s.view(N, -1)[row, grp] if row < N else torch.tensor(0.0)
        assert ssh[b, grp, lane % 16] == want_s
    q2, s2 = unshuffle(qsh, ssh, N)
    assert torch.equal(q2, q) and torch.equal(s2, s)


def test_preshuffle_rejects_unaligned():
    with pytest.raises(ValueError):
        preshuffle(torch.zeros(16, 96, dtype=torch.int8), torch.zeros(16 * 96 // 32), 32)
