"""ZeRO++ communication (reference `partition_parameters.py:679-718, 1160-1255` qwZ, `groups.py:505-533` hpZ,
`runtime/comm/coalesced_collectives.py:31-68` + `stage3.py:1266-1291` qgZ), on flat groups.

* qwZ  — quantized weight all-gather: the rank's bf16 shard is group-quantised to int8 (gfx950 quantize kernel), the
         int8 payload and fp32 scales are all-gathered (2x fewer bytes on xGMI than bf16) and dequantised straight
         into the gathered flat buffer.
* hpZ  — hierarchical partition: after the forward all-gather every rank keeps the 1/hpz slice of the full group
         owned by its position in a small group of consecutive ranks (one node's GPUs on an xGMI mesh); the backward
         re-gather then runs only inside that group.
* qgZ  — quantized gradient reduce-scatter: the flat gradient is quantised per destination chunk, exchanged with ONE
         all-to-all (every peer pair has its own xGMI link, so all-to-all is the natural full-mesh collective), and
         each rank dequantises + sums the world's copies of its own chunk in one fused kernel (dequant_reduce).
"""
import torch

from ... import comm as dist
from ...ops.quantizer import quantize
from ...ops.quantizer.quantizer import QuantizedTensor, dequantize, dequant_reduce


def _qgroup(n, cap=2048):
    """Largest power-of-two quantisation group <= cap dividing n (n is a multiple of 64 for flat segments)."""
    gs = cap
    while gs > 1 and n % gs:
        gs //= 2
    return gs


@torch.no_grad()
def quantized_all_gather(full, shard, group, bits=8):
    """full[dp * seg] (bf16) <- dequant(all_gather(quant(shard)))."""
    dp = dist.get_world_size(group)
    seg = shard.numel()
    gs = _qgroup(seg)
    qt = quantize(shard, group_size=gs, bits=bits, symmetric=True)
    q_all = torch.empty(dp * qt.data.numel(), dtype=torch.int8, device=shard.device)
    s_all = torch.empty(dp * qt.scales.numel(), dtype=torch.float32, device=shard.device)
    dist.all_gather_into_tensor(q_all, qt.data, group=group)
    dist.all_gather_into_tensor(s_all, qt.scales, group=group)
    out = dequantize(QuantizedTensor(q_all, s_all, torch.empty(0, device=shard.device), torch.Size([dp * seg]), gs,
                                     bits, full.dtype))
    full.copy_(out.view(-1))
    return full


@torch.no_grad()
def quantized_reduce_scatter(out, inp, group, bits=8):
    """out[seg] <- sum over ranks of chunk `rank` of inp[dp * seg], exchanged as int8 through one all-to-all."""
    dp = dist.get_world_size(group)
    seg = out.numel()
    gs = _qgroup(seg)
    qt = quantize(inp.reshape(-1), group_size=gs, bits=bits, symmetric=True)  # groups never straddle chunks
    q_recv = torch.empty_like(qt.data)
    s_recv = torch.empty_like(qt.scales)
    dist.all_to_all_single(q_recv, qt.data, group=group)
    dist.all_to_all_single(s_recv, qt.scales, group=group)
    red = dequant_reduce(q_recv, s_recv, dp, gs, 1.0, dtype=torch.float32)
    out.copy_(red.view(-1))
    return out


class HpzState:
    """Secondary (intra-node) partitions for hpZ."""

    def __init__(self, group):
        self.group = group
        self.size = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def keep_secondary(self, g):
        sec = g.padded // self.size
        g.secondary = g.full[self.rank * sec:(self.rank + 1) * sec].clone()

    def gather_from_secondary(self, g):
        dist.all_gather_into_tensor(g.full, g.secondary, group=self.group)

    def can_use(self, g):
        return getattr(g, "secondary", None) is not None and g.padded % self.size == 0

    @staticmethod
    def drop(g):
        g.secondary = None
