"""Ragged mixture-of-experts block on gfx950 kernels (inference v2 MoE path) plus ragged-batch row gathers.

Reference behaviour: `inference/v2/kernels/ragged_ops/top_k_gating/top_k_gating.cu:15` (fp32 softmax + top-k +
per-expert counts), `moe_scatter/moe_scatter.cu:23` and `moe_gather/moe_gather.cu:21` (permute tokens to an
expert-contiguous layout and back, weighted), the CUTLASS grouped `moe_gemm` (`cutlass_ops/moe_gemm`) driven by
`modules/implementations/moe/cutlass_multi_gemm.py`, `ragged_ops/embed/embed.cu:19`,
`logits_gather/logits_gather.cu:19`, and random-LTD's `csrc/random_ltd/gather_scatter.cu`.

MI355X design: the whole routed block is five kernel launches and NO host synchronisation — the expert slot of each
(token, choice) is claimed with an atomic on the expert's counter inside the gating kernel, the expert-sorted row
of a (token, choice) is derived on device from the counters' prefix sum, and the grouped MFMA GEMM derives its
(expert, m-tile) map from the same counters. That makes a decode step with MoE layers capturable in a hipGraph,
unlike a per-expert Python loop which must read the counts back to the host.

Host tensors (CPU plumbing path) use the fp32 PyTorch oracle below, which is also what the kernel tests compare to.
"""
import torch
import torch.nn.functional as F

from .native import hip_ops


# ------------------------------------------------------------------------------------------------ oracles
def topk_gating_reference(logits, k, renormalize=False):
    """(scores fp32 [T, k], experts int64 [T, k], counts int64 [E]) — softmax over all experts, then top-k."""
    probs = torch.softmax(logits.float(), dim=-1)
    w, e = torch.topk(probs, k, dim=-1)
    if renormalize:
        w = w / w.sum(-1, keepdim=True)
    return w, e, torch.bincount(e.reshape(-1), minlength=logits.shape[-1])


def moe_block_reference(x, router_w, fc1_w, fc2_w, k, act, renormalize=False, routing=None, fc1_b=None, fc2_b=None):
    """out[t] = sum_j w[t, j] * fc2_e(act(fc1_e(x[t]))) with e = experts[t, j]; fp32 accumulation. Optional
    per-expert biases fc1_b [E, N1] / fc2_b [E, H] (Megatron-style experts).
    `routing=(w, e)` replaces the router (tests feed the device gating's choice to isolate the expert math)."""
    t = x.reshape(-1, x.shape[-1])
    if routing is None:
        w, e, counts = topk_gating_reference(F.linear(t, router_w), k, renormalize)
    else:
        w, e = routing[0].float(), routing[1].long()
        counts = torch.bincount(e.reshape(-1), minlength=router_w.shape[0])
    out = torch.zeros(t.shape, dtype=torch.float32, device=t.device)
    flat = e.reshape(-1)
    order = torch.argsort(flat, stable=True)
    tok = order // k
    wts = w.reshape(-1)[order]
    s = 0
    for ex, c in enumerate(counts.tolist()):
        if c == 0:
            continue
        rows, ww = tok[s:s + c], wts[s:s + c]
        s += c
        h = act(F.linear(t.index_select(0, rows), fc1_w[ex], None if fc1_b is None else fc1_b[ex]))
        y = F.linear(h, fc2_w[ex], None if fc2_b is None else fc2_b[ex])
        out.index_add_(0, rows, y.float() * ww[:, None])
    return out.to(x.dtype).view(x.shape)


# ------------------------------------------------------------------------------------------------ kernels
def topk_gating(logits, k, renormalize=False):
    """Device: (scores fp32 [T, k], experts int32 [T, k], slots int32 [T, k], counts int32 [E])."""
    return hip_ops().topk_gating(logits.contiguous(), int(k), bool(renormalize))


def moe_scatter(x, experts, slots, counts):
    """x [T, H] -> (xs [T*k, H] expert-contiguous, rows [T, k] where each (t, j) landed, inclusive cumsum [E])."""
    return hip_ops().moe_scatter(x.contiguous(), experts, slots, counts)


def moe_gather(y, scores, rows):
    return hip_ops().moe_gather(y.contiguous(), scores, rows)


# Rows at which the library grouped GEMM (hipBLASLt-backed `torch._grouped_mm`, offsets on device, so still
# sync-free) overtakes the in-tree 128x128 MFMA kernel on gfx950: measured at Mixtral shapes (N 28672, K 4096) the
# kernel is faster up to ~512 rows (decode / small batches: 0.39 vs 0.50 ms), the library from ~4k rows
# (0.97 vs 1.90 ms at 4096, 1.33 PF/s at 16k) — profiles/moe_grouped_gemm_r1.jsonl.
GROUPED_LIBRARY_MIN_ROWS = int(__import__("os").environ.get("DS_MOE_LIBRARY_MIN_ROWS", "1024"))


def grouped_gemm(x, w, counts):
    """Y[rows of e] = X[rows of e] . W[e]^T for expert-contiguous X [R, K], W [E, N, K], counts [E] int32."""
    if x.shape[0] >= GROUPED_LIBRARY_MIN_ROWS and hasattr(torch, "_grouped_mm"):
        offs = torch.cumsum(counts, 0, dtype=torch.int32)
        return torch._grouped_mm(x.contiguous(), w.transpose(1, 2), offs=offs)
    return hip_ops().grouped_gemm(x.contiguous(), w.contiguous(), counts)


def grouped_gemm_ok(n, k):
    return n % 128 == 0 and k % 128 == 0


def native_moe_ok(x, router_w, fc1_w, fc2_w, k):
    E = router_w.shape[0]
    return (x.is_cuda and x.dtype == torch.bfloat16 and fc1_w.dtype == torch.bfloat16 and fc1_w.dim() == 3
            and 1 <= E <= 256 and 1 <= k <= min(8, E) and x.shape[-1] % 8 == 0
            and grouped_gemm_ok(fc1_w.shape[1], fc1_w.shape[2]) and grouped_gemm_ok(fc2_w.shape[1], fc2_w.shape[2]))


def moe_block(x, router_w, fc1_w, fc2_w, k, act, renormalize=False, fc1_b=None, fc2_b=None):
    """Routed expert MLP of a ragged token batch. `act` maps fc1 output [R, G*I] -> [R, I] (gated or plain).
    fc1_b [E, G*I] / fc2_b [E, H]: optional per-expert biases.

    Device path: gating -> scatter -> grouped GEMM -> act -> grouped GEMM -> weighted gather (bf16 out); expert
    biases are added to the expert-contiguous rows through a sync-free row -> expert map.
    """
    if not native_moe_ok(x, router_w, fc1_w, fc2_w, k):
        return moe_block_reference(x, router_w, fc1_w, fc2_w, k, act, renormalize, fc1_b=fc1_b, fc2_b=fc2_b)
    shp = x.shape
    t = x.reshape(-1, shp[-1]).contiguous()
    scores, experts, slots, counts = topk_gating(F.linear(t, router_w), k, renormalize)
    xs, rows, _ = moe_scatter(t, experts, slots, counts)
    h = grouped_gemm(xs, fc1_w, counts)
    row_expert = None
    if fc1_b is not None or fc2_b is not None:
        row_expert = torch.repeat_interleave(torch.arange(counts.numel(), device=counts.device), counts.long(),
                                             output_size=xs.shape[0])
    if fc1_b is not None:
        h = h + fc1_b.index_select(0, row_expert)
    y = grouped_gemm(act(h), fc2_w, counts)
    if fc2_b is not None:
        y = y + fc2_b.index_select(0, row_expert)
    return moe_gather(y, scores, rows).view(shp)


# ------------------------------------------------------------------------------------------------ row gathers
def embed_gather(table, ids, pos_table=None, pos=None):
    """out[i] = table[ids[i]] (+ pos_table[pos[i]]) (reference `ragged_ops/embed/embed.cu:19`)."""
    ids = ids.reshape(-1).long()
    if table.is_cuda and table.dtype == torch.bfloat16 and table.shape[1] % 8 == 0:
        if pos_table is not None:
            return hip_ops().embed_gather(table, ids, pos_table.contiguous(), pos.reshape(-1).long())
        return hip_ops().embed_gather(table, ids, None, None)
    out = table.index_select(0, ids)
    if pos_table is not None:
        out = out + pos_table.index_select(0, pos.reshape(-1).long())
    return out


def rows_gather(x, idx):
    """out[i] = x[idx[i]] over rows of the last dim (reference `logits_gather.cu:19`, random-LTD gather)."""
    x2 = x.reshape(-1, x.shape[-1])
    idx = idx.reshape(-1).long()
    if x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return hip_ops().rows_gather(x2.contiguous(), idx)
    return x2.index_select(0, idx)


def rows_scatter(part, idx, full):
    """full[idx[i]] = part[i] in place (random-LTD scatter back, `gather_scatter.cu`)."""
    f2 = full.view(-1, full.shape[-1])
    idx = idx.reshape(-1).long()
    if full.is_cuda and full.dtype == torch.bfloat16 and full.shape[-1] % 8 == 0 and full.is_contiguous():
        hip_ops().rows_scatter(part.reshape(-1, part.shape[-1]).contiguous(), idx, f2)
    else:
        f2.index_copy_(0, idx, part.reshape(-1, part.shape[-1]).to(f2.dtype))
    return full
