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
# Copy budget. all_to_all_single fixes both buffer layouts ([P, ...]: one contiguous chunk per peer), and the flash
# kernels need a uniform token stride, so each direction costs exactly one packing pass into the send buffer and one
# unpacking pass out of the receive buffer. Everything else is views: the packed buffer is filled by strided copies
# straight from whatever layout the producer left (no cat / contiguous staging), and the unpacked [B, heads, S, D]
# buffer is handed to attention as per-tensor views (the kernels take batch / head / token strides).
def _pack(dst, src):
    """One strided copy (a single HBM pass) of a view into (a view of) a communication buffer."""
    dst.copy_(src)


def _heads_to_seq(q, k, v, group):
    """[B,Hq,s,D],[B,Hk,s,D],[B,Hk,s,D] (local tokens) -> views [B,Hq/P,S,D], ... (local heads, all tokens) of one
    receive buffer. One a2a, one pass in, one pass out."""
    P = dist.get_world_size(group)
    B, Hq, s, D = q.shape
    Hk = k.shape[1]
    hq, hk = Hq // P, Hk // P
    h3 = hq + 2 * hk
    # send[p] = [q heads of rank p | k heads of rank p | v heads of rank p], each [B, h, s, D]
    send = torch.empty((P, B, h3, s, D), dtype=q.dtype, device=q.device)
    _pack(send[:, :, :hq], q.unflatten(1, (P, hq)).transpose(0, 1))
    _pack(send[:, :, hq:hq + hk], k.unflatten(1, (P, hk)).transpose(0, 1))
    _pack(send[:, :, hq + hk:], v.unflatten(1, (P, hk)).transpose(0, 1))
    recv = _a2a(send, group)  # recv[p] = rank p's tokens of my heads
    full = torch.empty((B, h3, P, s, D), dtype=q.dtype, device=q.device)  # token order = rank order
    _pack(full, recv.permute(1, 2, 0, 3, 4))
    full = full.view(B, h3, P * s, D)
    return full[:, :hq], full[:, hq:hq + hk], full[:, hq + hk:]


def _seq_to_heads(o, group):
    """[B, h, S, D] (local heads, all tokens; any strides) -> [B, h*P, S/P, D] (all heads, local tokens)."""
    P = dist.get_world_size(group)
    B, h, S, D = o.shape
    s = S // P
    send = torch.empty((P, B, h, s, D), dtype=o.dtype, device=o.device)
    _pack(send, o.unflatten(2, (P, s)).permute(2, 0, 1, 3, 4))
    recv = _a2a(send, group)  # recv[p] = rank p's heads for my tokens
    out = torch.empty((B, P, h, s, D), dtype=o.dtype, device=o.device)
    _pack(out, recv.transpose(0, 1))
    return out.view(B, P * h, s, D)


class _FusedQKVToSeq(torch.autograd.Function):

    @staticmethod
    def forward(ctx, group, q, k, v):
        ctx.group = group
        return _heads_to_seq(q, k, v, group)

    @staticmethod
    def backward(ctx, dq, dk, dv):
        P = dist.get_world_size(ctx.group)
        # inverse of the forward exchange: pack per source rank, a2a, unpack heads
        B, hq, S, D = dq.shape
        hk = dk.shape[1]
        s = S // P
        h3 = hq + 2 * hk
        g = torch.empty((P, B, h3, s, D), dtype=dq.dtype, device=dq.device)
        _pack(g[:, :, :hq], dq.unflatten(2, (P, s)).permute(2, 0, 1, 3, 4))
        _pack(g[:, :, hq:hq + hk], dk.unflatten(2, (P, s)).permute(2, 0, 1, 3, 4))
        _pack(g[:, :, hq + hk:], dv.unflatten(2, (P, s)).permute(2, 0, 1, 3, 4))
        r = _a2a(g, ctx.group)  # r[p] = grads for rank p's heads, my tokens: [P, B, hq+2hk, s, D]
        outs = []
        for lo, h in ((0, hq), (hq, hk), (hq + hk, hk)):  # unpack each tensor straight into its own [B, P*h, s, D]
            t = torch.empty((B, P, h, s, D), dtype=dq.dtype, device=dq.device)
            _pack(t, r[:, :, lo:lo + h].transpose(0, 1))
            outs.append(t.view(B, P * h, s, D))
        return (None, *outs)


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
        send = torch.empty((P, B, h, s, D), dtype=g.dtype, device=g.device)  # rank p gets its heads
        _pack(send, g.unflatten(1, (P, h)).transpose(0, 1))
        recv = _a2a(send, ctx.group)  # recv[p] = my heads, rank p's tokens
        out = torch.empty((B, h, P, s, D), dtype=g.dtype, device=g.device)
        _pack(out, recv.permute(1, 2, 0, 3, 4))
        return None, out.view(B, h, P * s, D)


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
        return _SeqToHeads.apply(self.spg, o)


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
