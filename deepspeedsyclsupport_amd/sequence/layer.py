"""Ulysses sequence parallelism (reference `deepspeed/sequence/layer.py:15-109`).

Each rank holds S/P tokens of every sequence. Before attention one all-to-all re-shards Q/K/V from "all heads, S/P
tokens" to "H/P heads, all S tokens"; local attention runs over the full sequence; the inverse all-to-all restores the
token sharding. On an 8-GPU MI355X node the SP group is one xGMI full mesh, so each all-to-all moves (P-1)/P of the
tensor with every peer pair on its own link — the collective Ulysses wants.

MI355X additions over the reference:
* Q, K and V are exchanged in ONE fused all-to-all (the reference issues three, TODO at `layer.py:96`), GQA-aware:
  per destination rank the send buffer holds [q heads | k heads | v heads] for that rank, so K/V with fewer heads
  still travel in the same collective.
* Works on the [B, H, S, D] layout our attention kernels consume (and on the reference's [S, B, H, D] through
  `DistributedAttention(scatter_idx, gather_idx)`).
"""
import torch

from .. import comm as dist
from ..ops.attention import attention as _local_attention


def _a2a(x, group):
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=group)
    return out


def single_all_to_all(input, scatter_idx, gather_idx, group):
    """Scatter `scatter_idx` across the group and gather `gather_idx` (generic layout, one collective)."""
    P = dist.get_world_size(group)
    if P == 1:
        return input
    chunks = input.chunk(P, dim=scatter_idx)
    send = torch.stack(chunks, dim=0).contiguous()
    recv = _a2a(send, group)
    return torch.cat(list(recv.unbind(0)), dim=gather_idx).contiguous()


class _SeqAllToAll(torch.autograd.Function):

    @staticmethod
    def forward(ctx, group, input, scatter_idx, gather_idx):
        ctx.group, ctx.scatter_idx, ctx.gather_idx = group, scatter_idx, gather_idx
        return single_all_to_all(input, scatter_idx, gather_idx, group)

    @staticmethod
    def backward(ctx, grad):
        return None, _SeqAllToAll.apply(ctx.group, grad, ctx.gather_idx, ctx.scatter_idx), None, None


class DistributedAttention(torch.nn.Module):
    """Reference-compatible wrapper: `local_attention(q, k, v, *args)` on [S, B, H, D]-style tensors
    (scatter heads at `scatter_idx`, gather sequence at `gather_idx`)."""

    def __init__(self, local_attention, sequence_process_group, scatter_idx=2, gather_idx=0):
        super().__init__()
        self.local_attn = local_attention
        self.spg = sequence_process_group
        self.scatter_idx = scatter_idx
        self.gather_idx = gather_idx

    def forward(self, query, key, value, *args, **kwargs):
        q = _SeqAllToAll.apply(self.spg, query, self.scatter_idx, self.gather_idx)
        k = _SeqAllToAll.apply(self.spg, key, self.scatter_idx, self.gather_idx)
        v = _SeqAllToAll.apply(self.spg, value, self.scatter_idx, self.gather_idx)
        ctx = self.local_attn(q, k, v, *args, **kwargs)
        return _SeqAllToAll.apply(self.spg, ctx, self.gather_idx, self.scatter_idx)


# ---------------------------------------------------------------------------------------------- fused [B,H,S,D] path
def _heads_to_seq(q, k, v, group):
    """[B,Hq,s,D],[B,Hk,s,D],[B,Hk,s,D] (local tokens) -> [B,Hq/P,S,D], ... (local heads, all tokens). One a2a."""
    P = dist.get_world_size(group)
    B, Hq, s, D = q.shape
    Hk = k.shape[1]
    hq, hk = Hq // P, Hk // P
    # send[p] = [q heads of rank p | k heads of rank p | v heads of rank p], each [B, h, s, D]
    send = torch.cat([q.view(B, P, hq, s, D), k.view(B, P, hk, s, D), v.view(B, P, hk, s, D)], dim=2)
    send = send.transpose(0, 1).contiguous()  # [P, B, hq+2hk, s, D]
    recv = _a2a(send, group)  # recv[p] = rank p's tokens of my heads
    recv = recv.permute(1, 2, 0, 3, 4).reshape(B, hq + 2 * hk, P * s, D)  # token order = rank order
    return recv[:, :hq], recv[:, hq:hq + hk], recv[:, hq + hk:]


def _seq_to_heads(o, group):
    """[B, h, S, D] (local heads, all tokens) -> [B, h*P, S/P, D] (all heads, local tokens)."""
    P = dist.get_world_size(group)
    B, h, S, D = o.shape
    s = S // P
    send = o.view(B, h, P, s, D).permute(2, 0, 1, 3, 4).contiguous()  # [P, B, h, s, D]
    recv = _a2a(send, group)  # recv[p] = rank p's heads for my tokens
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * h, s, D)


class _FusedQKVToSeq(torch.autograd.Function):

    @staticmethod
    def forward(ctx, group, q, k, v):
        ctx.group = group
        ctx.hq, ctx.hk = q.shape[1], k.shape[1]
        qo, ko, vo = _heads_to_seq(q, k, v, group)
        return qo.contiguous(), ko.contiguous(), vo.contiguous()

    @staticmethod
    def backward(ctx, dq, dk, dv):
        P = dist.get_world_size(ctx.group)
        # inverse of the forward exchange: pack per source rank, a2a, unpack heads
        B, hq, S, D = dq.shape
        hk = dk.shape[1]
        s = S // P
        g = torch.cat([dq, dk, dv], dim=1).view(B, hq + 2 * hk, P, s, D).permute(2, 0, 1, 3, 4).contiguous()
        r = _a2a(g, ctx.group)  # r[p] = grads for rank p's heads, my tokens: [P, B, hq+2hk, s, D]
        r = r.transpose(0, 1)  # [B, P, hq+2hk, s, D]
        gq = r[:, :, :hq].reshape(B, P * hq, s, D)
        gk = r[:, :, hq:hq + hk].reshape(B, P * hk, s, D)
        gv = r[:, :, hq + hk:].reshape(B, P * hk, s, D)
        return None, gq.contiguous(), gk.contiguous(), gv.contiguous()


class _SeqToHeads(torch.autograd.Function):

    @staticmethod
    def forward(ctx, group, o):
        ctx.group = group
        return _seq_to_heads(o, group)

    @staticmethod
    def backward(ctx, g):
        P = dist.get_world_size(ctx.group)
        B, H, s, D = g.shape
        h = H // P
        send = g.reshape(B, P, h, s, D).transpose(0, 1).contiguous()  # [P, B, h, s, D] -> rank p gets its heads
        recv = _a2a(send, ctx.group)  # recv[p] = my heads, rank p's tokens
        return None, recv.permute(1, 2, 0, 3, 4).reshape(B, h, P * s, D).contiguous()


class UlyssesAttention(torch.nn.Module):
    """Drop-in for the local attention call of our models: q/k/v [B, H, S/P, D] -> o [B, H, S/P, D]."""

    def __init__(self, sequence_process_group, attn_fn=None, causal=True):
        super().__init__()
        self.spg = sequence_process_group
        self.attn_fn = attn_fn or _local_attention
        self.causal = causal

    def forward(self, q, k, v):
        P = dist.get_world_size(self.spg)
        if P == 1:
            return self.attn_fn(q, k, v, causal=self.causal)
        assert q.shape[1] % P == 0 and k.shape[1] % P == 0, \
            f"Ulysses needs heads divisible by sp={P} (q heads {q.shape[1]}, kv heads {k.shape[1]})"
        qs, ks, vs = _FusedQKVToSeq.apply(self.spg, q, k, v)
        o = self.attn_fn(qs, ks, vs, causal=self.causal)
        return _SeqToHeads.apply(self.spg, o.contiguous())


def shard_sequence(input_ids, labels=None, group=None, ignore_index=-100):
    """Split [B, S] token ids along S for this SP rank. Labels are pre-shifted on the FULL sequence (position t
    predicts t+1, last position ignored) so no cross-shard shift is needed; call the model with shift_labels=False.
    Returns (input_shard, label_shard, pos_offset)."""
    P = dist.get_world_size(group)
    r = dist.get_rank(group)
    B, S = input_ids.shape
    assert S % P == 0, f"sequence length {S} not divisible by sp={P}"
    s = S // P
    inp = input_ids[:, r * s:(r + 1) * s]
    lab = None
    if labels is not None:
        shifted = torch.full_like(labels, ignore_index)
        shifted[:, :-1] = labels[:, 1:]
        lab = shifted[:, r * s:(r + 1) * s]
    return inp, lab, r * s


def enable_sequence_parallel(model, group):
    """Install Ulysses attention into every attention module that supports it (`.seq_parallel` hook)."""
    n = 0
    for m in model.modules():
        if hasattr(m, "seq_parallel"):
            m.seq_parallel = UlyssesAttention(group)
            n += 1
    return n
