"""`link_hp_params` over hand-made flat partitions on 2 gloo ranks (reference `utils/mixed_precision_linkage.py`,
`tests/unit/runtime/zero/test_zero_tensor_fragment.py`: full hp params / optimizer states / grads assembled from the
ranks' fragments, and setters that write through to the owning partition)."""
import torch

from ..common import run_distributed


def _linked():
    import deepspeedsyclsupport_amd as ds
    from deepspeedsyclsupport_amd import comm as dist
    from deepspeedsyclsupport_amd.utils.mixed_precision_linkage import link_hp_params
    ds.init_distributed(dist_backend="gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    shapes = [(3, 5), (7, ), (4, 4), (9, )]  # 15 + 7 + 16 + 9 = 47 -> padded to 48, 24 per rank
    lps = [torch.randn(s).bfloat16() for s in shapes]
    flat = torch.cat([p.float().reshape(-1) for p in lps] + [torch.zeros(1)])
    psize = flat.numel() // w
    hp = flat[r * psize:(r + 1) * psize].clone()
    state = {"exp_avg": torch.arange(psize, dtype=torch.float32) + 100 * r, "exp_avg_sq": torch.ones(psize) * (r + 1),
             "step": 3}
    grads = {0: None}
    linked = link_hp_params(lps, hp, gradient_dict=grads, param_group_index=0, partition_start=r * psize,
                            partition_size=psize, partition_optimizer_state=state, dp_group=None)
    owned = [p for p in lps if p._hp_mapping is not None]
    assert len(linked) == len(owned) >= 2
    if r == 0:
        m = lps[2]._hp_mapping  # spans the partition boundary: elements 22..37 of the flat vector
        assert (m.lp_fragment_address.start, m.lp_fragment_address.numel) == (0, 2)
        assert (m.hp_fragment_address.start, m.hp_fragment_address.numel) == (22, 2)
        assert lps[3]._hp_mapping is None
    else:
        m = lps[2]._hp_mapping
        assert (m.lp_fragment_address.start, m.lp_fragment_address.numel) == (2, 14)
        assert (m.hp_fragment_address.start, m.hp_fragment_address.numel) == (0, 14)
        assert sorted(m.get_optim_state_keys()) == ["exp_avg", "exp_avg_sq"]
    # full tensors come back from the two ranks' fragments
    for p in lps:
        torch.testing.assert_close(p.get_full_hp_param(), p.float(), rtol=0, atol=0)
    full_m = lps[2].get_full_hp_param("exp_avg")
    want = torch.cat([torch.arange(22, 24, dtype=torch.float32), torch.arange(0, 14, dtype=torch.float32) + 100])
    torch.testing.assert_close(full_m.reshape(-1), want, rtol=0, atol=0)
    # setters write through to the owner's partition; lp <-> hp sync
    lps[2].set_full_hp_param(torch.full((4, 4), 7.0))
    torch.testing.assert_close(lps[2].get_full_hp_param(), torch.full((4, 4), 7.0))
    lps[2]._hp_mapping.update_lp()
    assert float(lps[2].reshape(-1)[lps[2]._hp_mapping.lp_fragment_address.start]) == 7.0
    # gradients of the parameters that meet the partition, in list order (the guard for a missing dict is tested below)
    grads[0] = [torch.full(p.shape, float(i + 1)).bfloat16() for i, p in enumerate(owned)]
    g = lps[0].get_full_hp_grad()  # collective: both ranks call it
    torch.testing.assert_close(g, torch.full((3, 5), 1.0))


def test_link_hp_params_two_ranks():
    run_distributed(_linked, 2)


def test_get_full_hp_grad_needs_live_gradients():
    from deepspeedsyclsupport_amd.utils.mixed_precision_linkage import link_hp_params
    p = torch.zeros(4, 2).bfloat16()
    hp = torch.zeros(8)
    link_hp_params([p], hp, gradient_dict={0: None}, partition_optimizer_state={})
    import pytest
    with pytest.raises(ValueError):
        p.get_full_hp_grad()
