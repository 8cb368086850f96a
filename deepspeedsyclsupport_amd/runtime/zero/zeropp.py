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


def swizzle_quant(inp, nodes, local, group_size, bits=8):
    """Quantise a flat gradient of `nodes * local` destination chunks with the chunks re-ordered
    [local index][node] instead of [node][local index] (reference `swizzled_quantize.cu:21`): what goes to local
    peer b — the chunks of every node's rank b — becomes one contiguous run, so the intra-node all-to-all needs no
    gather. Returns the QuantizedTensor of the re-ordered data."""
    seg = inp.numel() // (nodes * local)
    sw = inp.view(nodes, local, seg).transpose(0, 1).contiguous().view(-1)
    return quantize(sw, group_size=group_size, bits=bits, symmetric=True)


def quantized_reduction(q, scales, nsrc, group_size, bits=8):
    """Dequantise `nsrc` stacked copies, sum them, re-quantise the sum (reference `quant_reduce.cu:21`: the
    intra-node step of the two-level exchange). Returns a QuantizedTensor of numel / nsrc elements."""
    red = dequant_reduce(q, scales, nsrc, group_size, 1.0, dtype=torch.float32)
    return quantize(red.view(-1), group_size=group_size, bits=bits, symmetric=True)


@torch.no_grad()
def quantized_reduce_scatter_2level(out, inp, local_group, global_group, bits=8):
    """qgZ across nodes (reference `coalesced_collectives.py:31-68`): out[seg] <- sum over ALL ranks of this rank's
    chunk of inp[nodes * local * seg], moving only 1 / local of the single-level volume between nodes.

    rank = node * local + b (consecutive ranks share a node). Step 1, inside the node (xGMI all-to-all): peer b
    receives, from each of the node's ranks, the chunks destined for the ranks with local index b on every node, and
    sums them (fused dequant-reduce) — `nodes` partial chunks. Step 2, between nodes (ranks with the same local
    index): partial chunk a goes to node a; the `nodes` partials of this rank's own chunk are summed into `out`.
    """
    local = dist.get_world_size(local_group)
    nodes = dist.get_world_size(global_group)
    seg = out.numel()
    if inp.numel() != nodes * local * seg:
        raise ValueError(f"input of {inp.numel()} elements is not nodes * local * segment = {nodes * local * seg}")
    gs = _qgroup(seg)
    qt = swizzle_quant(inp.reshape(-1), nodes, local, gs, bits)
    q1, s1 = torch.empty_like(qt.data), torch.empty_like(qt.scales)
    dist.all_to_all_single(q1, qt.data, group=local_group)
    dist.all_to_all_single(s1, qt.scales, group=local_group)
    part = quantized_reduction(q1, s1, local, gs, bits)              # [nodes * seg]: this node's sums, by target node
    q2, s2 = torch.empty_like(part.data), torch.empty_like(part.scales)
    dist.all_to_all_single(q2, part.data, group=global_group)
    dist.all_to_all_single(s2, part.scales, group=global_group)
    out.copy_(dequant_reduce(q2, s2, nodes, gs, 1.0, dtype=torch.float32).view(-1))
    return out


def qgz_groups(dp_group):
    """(local group, cross-node group) for a two-level exchange over `dp_group`, or None when the group sits on one
    node (or is not the whole job, where the node split is unknown): then the single-level exchange is used."""
    from ...parallel import groups
    world = dist.get_world_size()
    if dist.get_world_size(dp_group) != world:
        return None
    return levels_from_table(groups._get_local_all_to_all_group())


def levels_from_table(table):
    """This rank's (local, cross-node) groups out of the `local_<node>` / `global_<local index>` table, or None when
    the table holds one node. (A group's size can only be asked by its members, so the rank's own groups are found
    by membership.)"""
    local = next((g for k, g in table.items() if k.startswith("local_") and dist.get_rank(g) >= 0), None)
    cross = next((g for k, g in table.items() if k.startswith("global_") and dist.get_rank(g) >= 0), None)
    if local is None or cross is None or dist.get_world_size(cross) < 2:
        return None
    return local, cross


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


@torch.no_grad()
def hierarchical_all_gather(full, shard, intra_group, inter_group):
    """full[nodes * local * seg] <- every rank's shard, in rank order (rank = node * local + local index), as two
    all-gathers (reference `runtime/zero/mics.py:234-300`): first between nodes among the ranks of one local index
    (each message is a whole shard, all local ranks use the network at once), then inside the node over xGMI with
    `nodes` shards per message; one strided copy puts the [local, node] result into rank order."""
    local = dist.get_world_size(intra_group)
    nodes = dist.get_world_size(inter_group)
    seg = shard.numel()
    if full.numel() != nodes * local * seg:
        raise ValueError(f"output of {full.numel()} elements is not nodes * local * shard = {nodes * local * seg}")
    across = torch.empty(nodes * seg, dtype=shard.dtype, device=shard.device)
    dist.all_gather_into_tensor(across, shard.contiguous(), group=inter_group)
    by_local = torch.empty(local * nodes * seg, dtype=shard.dtype, device=shard.device)
    dist.all_gather_into_tensor(by_local, across, group=intra_group)
    full.view(nodes, local, seg).copy_(by_local.view(local, nodes, seg).transpose(0, 1))
    return full

