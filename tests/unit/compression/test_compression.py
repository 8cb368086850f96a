"""Compression (reference `tests/unit/compression/test_compression.py`): QAT layers, pruning masks, redundancy
clean shrinking layers, layer reduction."""
import torch
import torch.nn as nn

from deepspeedsyclsupport_amd.compression import (LinearLayer_Compress, fake_quant, init_compression,
                                                  redundancy_clean)


class MLP(nn.Module):

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.layers = nn.ModuleList([nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 16)) for _ in range(4)])
        self.head = nn.Linear(16, 4)

    def forward(self, x):
        for l in self.layers:
            x = x + l(x)
        return self.head(x)


def _cfg(**tech):
    return {"compression_training": tech}


def test_fake_quant_levels():
    w = torch.randn(4, 64)
    q = fake_quant(w, 4, groups=4)
    for row in q:
        assert row.unique().numel() <= 15
    assert (q - w).abs().max() <= w.abs().max() / 7 / 2 + 1e-6


def test_weight_quantization_ste_trains():
    m = MLP()
    cfg = _cfg(weight_quantization={"shared_parameters": {"enabled": True, "quantize_weight_in_forward": True,
                                                          "quantize_groups": 2, "schedule_offset": 0},
                                    "different_groups": {"wq": {"params": {"start_bits": 8, "target_bits": 4,
                                                                           "quantization_period": 2},
                                                                "modules": ["layers.*"]}}})
    init_compression(m, cfg)
    lin = m.layers[0][0]
    assert isinstance(lin, LinearLayer_Compress) and lin.weight_quantization_enabled
    assert not isinstance(m.head, LinearLayer_Compress)
    opt = torch.optim.SGD(m.parameters(), lr=0.05)
    x, y = torch.randn(32, 16), torch.randint(0, 4, (32, ))
    losses = []
    for _ in range(20):
        loss = nn.functional.cross_entropy(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0] and lin.wq_bits == 4
    redundancy_clean(m, cfg)
    assert not lin.weight_quantization_enabled and lin.weight[0].unique().numel() <= 16 * 2


def test_sparse_and_row_pruning_clean():
    m = MLP()
    cfg = _cfg(sparse_pruning={"shared_parameters": {"enabled": True, "method": "l1", "schedule_offset": 0},
                               "different_groups": {"sp": {"params": {"dense_ratio": 0.5},
                                                           "modules": ["layers.0.0"]}}},
               row_pruning={"shared_parameters": {"enabled": True, "method": "topk", "schedule_offset": 0},
                            "different_groups": {"rp": {"params": {"dense_ratio": 0.25}, "modules": ["layers.1.0"],
                                                        "related_modules": [["layers.1.2"]]}}})
    init_compression(m, cfg)
    x = torch.randn(8, 16)
    m.eval()
    before = m(x)
    sp = m.layers[0][0]
    assert abs(float(sp.sparse_pruning_mask.mean()) - 0.5) < 0.02
    redundancy_clean(m, cfg)
    assert (m.layers[0][0].weight == 0).float().mean() >= 0.49
    assert m.layers[1][0].out_features == 8 and m.layers[1][2].in_features == 8
    torch.testing.assert_close(m(x), before, rtol=1e-5, atol=1e-5)  # masked forward == physically pruned forward


def test_layer_reduction():
    m = MLP()
    cfg = _cfg(layer_reduction={"enabled": True, "keep_number_layer": 2, "module_name_prefix": "layers",
                                "teacher_layer": [1, 3]})
    l1, l3 = m.layers[1], m.layers[3]
    init_compression(m, cfg)
    assert len(m.layers) == 2 and m.layers[0] is l1 and m.layers[1] is l3
