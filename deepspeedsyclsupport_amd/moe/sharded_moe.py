"""Top-k gating + expert-parallel dispatch (reference `moe/sharded_moe.py:95-554`).

MI355X-first dispatch: the reference builds dense one-hot [S, E, C] dispatch/combine masks and moves tokens with
`einsum("sec,sm->ecm")` — O(S·E·C·M) work and memory. Here each routed (token, slot) gets a flat destination index
e*C + loc computed from a per-expert prefix count, tokens are moved with one `index_copy` into the [E, C, M] send
buffer and combined back with `index_select` + weighted `index_add` — O(S·k·M). The two all-to-alls over the EP group
run on RCCL; with EP inside one node they are xGMI full-mesh exchanges.
"""
import math
from typing import Any, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from .. import comm as dist
from ..parallel import groups
from ..utils.logging import logger
from . import mappings
from .mappings import tensor_parallel_world_size

uniform_map = {}
gumbel_map = {}


def multiplicative_jitter(x, device, epsilon=1e-2):
    if epsilon == 0:
        return x
    uniform = uniform_map.get(device)
    if uniform is None:
        uniform = torch.distributions.uniform.Uniform(low=torch.tensor(1.0 - epsilon, device=device),
                                                      high=torch.tensor(1.0 + epsilon, device=device)).rsample
        uniform_map[device] = uniform
    return x * uniform(x.shape)


def gumbel_rsample(shape, device):
    gumbel = gumbel_map.get(device)
    if gumbel is None:
        gumbel = torch.distributions.gumbel.Gumbel(torch.tensor(0.0, device=device),
                                                   torch.tensor(1.0, device=device)).rsample
        gumbel_map[device] = gumbel
    return gumbel(shape)


class _AllToAll(torch.autograd.Function):

    @staticmethod
    def forward(ctx, group, input):
        ctx.group = group
        input = input.contiguous()
        if dist.get_world_size(group) == 1:
            return input
        out = torch.empty_like(input)
        dist.all_to_all_single(out, input, group=group)
        return out

    @staticmethod
    def backward(ctx, grad):
        return None, _AllToAll.apply(ctx.group, grad)


def _capacity(num_tokens, num_experts, capacity_factor, min_capacity, k=1):
    cap = math.ceil(k * num_tokens / num_experts * capacity_factor)
    return max(cap, min_capacity)


def _route(logits, k, capacity_factor, min_capacity, noisy_gate_policy, drop_tokens, use_rts, ep_group,
           top2_2nd_expert_sampling=True, training=True):
    """Returns (l_aux, expert_idx [S,k], loc [S,k] (-1 = dropped), gate_w [S,k], capacity, exp_counts)."""
    S, E = logits.shape
    if noisy_gate_policy == "RSample" and training:
        logits_w_noise = logits + gumbel_rsample(logits.shape, device=logits.device)
    else:
        logits_w_noise = logits
    gates = F.softmax(logits, dim=1)
    idx1 = torch.argmax(logits_w_noise if noisy_gate_policy == "RSample" else gates, dim=1)
    mask1 = F.one_hot(idx1, E)
    if k == 2:
        l2 = logits + gumbel_rsample(logits.shape, device=logits.device) if (top2_2nd_expert_sampling and training) \
            else logits
        idx2 = torch.argmax(l2.masked_fill(mask1.bool(), float("-inf")), dim=1)
        mask2 = F.one_hot(idx2, E)
    # load-balancing loss (GShard): E * sum_e mean(gates_e) * frac_tokens_e (top-1 assignment)
    me = gates.mean(dim=0)
    ce = mask1.float().mean(dim=0)
    l_aux = (me * ce).sum() * E
    exp_counts = mask1.sum(0).detach() + (mask2.sum(0).detach() if k == 2 else 0)
    # capacity
    if drop_tokens:
        capacity = _capacity(S, E, capacity_factor, min_capacity, k)
    else:
        cap_local = int(exp_counts.max())
        t = torch.tensor([cap_local], device=logits.device)
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        capacity = max(int(t), 1)
    if groups._get_expert_model_parallel_world_size() == 1:
        # the layer keeps 1/TP of the capacity slots per tensor-parallel rank (`mappings.drop_tokens`)
        tp = tensor_parallel_world_size()
        capacity = -(-capacity // tp) * tp
    # token priority inside an expert: random (RTS) or arrival order
    if use_rts and drop_tokens and training:
        prio = torch.rand(S, device=logits.device)
        order = torch.argsort(prio)
    else:
        order = torch.arange(S, device=logits.device)
    inv = torch.empty_like(order)
    inv[order] = torch.arange(S, device=logits.device)

    def locations(mask, base=None):
        m = mask[order]
        loc = torch.cumsum(m, dim=0) - 1
        if base is not None:
            loc = loc + base
        loc = (loc * m).sum(1)[inv]  # location of each token in its expert, original order
        return loc

    loc1 = locations(mask1)
    keep1 = loc1 < capacity
    idx = [idx1]
    loc = [torch.where(keep1, loc1, torch.full_like(loc1, -1))]
    g1 = (gates * mask1).sum(1)
    w = [g1]
    if k == 2:
        base = mask1.sum(0, keepdim=True)  # second choices queue behind every first choice of that expert
        loc2 = locations(mask2, base)
        keep2 = loc2 < capacity
        idx.append(idx2)
        loc.append(torch.where(keep2, loc2, torch.full_like(loc2, -1)))
        g2 = (gates * mask2).sum(1)
        g1k = g1 * keep1
        g2k = g2 * keep2
        denom = (g1k + g2k).clamp(min=torch.finfo(gates.dtype).eps)
        w = [g1k / denom, g2k / denom]
    return l_aux, torch.stack(idx, 1), torch.stack(loc, 1), torch.stack(w, 1), capacity, exp_counts


def top1gating(logits, capacity_factor, min_capacity, used_token=None, noisy_gate_policy=None, drop_tokens=True,
               use_rts=True, ep_group=None, use_tutel=False):
    return _route(logits, 1, capacity_factor, min_capacity, noisy_gate_policy, drop_tokens, use_rts, ep_group)


def top2gating(logits, capacity_factor, min_capacity, drop_tokens=True, ep_group=None, top2_2nd_expert_sampling=True):
    return _route(logits, 2, capacity_factor, min_capacity, None, drop_tokens, False, ep_group,
                  top2_2nd_expert_sampling)


class TopKGate(torch.nn.Module):

    def __init__(self, model_dim, num_experts, k=1, capacity_factor=1.0, eval_capacity_factor=1.0, min_capacity=8,
                 noisy_gate_policy=None, drop_tokens=True, use_rts=True, ep_group=None,
                 top2_2nd_expert_sampling=True):
        super().__init__()
        if k not in (1, 2):
            raise ValueError("Only top-1 and top-2 gatings are supported.")
        self.wg = torch.nn.Linear(model_dim, num_experts, bias=False).float()
        self.ep_group = ep_group
        self.k = k
        self.capacity_factor = capacity_factor
        self.eval_capacity_factor = eval_capacity_factor
        self.min_capacity = min_capacity
        self.noisy_gate_policy = noisy_gate_policy
        self.drop_tokens = drop_tokens
        self.use_rts = use_rts
        self.top2_2nd_expert_sampling = top2_2nd_expert_sampling
        self.wall_clock_breakdown = False
        self.gate_time = 0.0

    def _set_ep_group(self, ep_group):
        self.ep_group = ep_group

    def forward(self, input, used_token=None, use_tutel=False):
        x = input.float()
        if self.noisy_gate_policy == "Jitter" and self.training:
            x = multiplicative_jitter(x, device=x.device)
        logits = F.linear(x, self.wg.weight.float())
        cf = self.capacity_factor if self.training else self.eval_capacity_factor
        return _route(logits, self.k, cf, self.min_capacity, self.noisy_gate_policy if self.training else None,
                      self.drop_tokens, self.use_rts, self.ep_group, self.top2_2nd_expert_sampling, self.training)


class MOELayer(torch.nn.Module):

    def __init__(self, gate, experts, ep_group_name, ep_size, num_local_experts, use_tutel=False):
        super().__init__()
        self.gate = gate
        self.experts = experts
        self.ep_group = None
        self.ep_size = ep_size
        self.ep_group_name = ep_group_name
        self.num_local_experts = num_local_experts
        self.time_falltoall = self.time_salltoall = self.time_moe = 0.0
        self.wall_clock_breakdown = False
        self.l_aux = None
        self.exp_counts = None

    def _set_ep_group(self, ep_group):
        self.ep_group = ep_group
        self.gate._set_ep_group(ep_group)

    def forward(self, *input, **kwargs):
        x = input[0]
        d_model = x.shape[-1]
        tokens = x.reshape(-1, d_model)
        S = tokens.shape[0]
        l_aux, eidx, loc, w, C, exp_counts = self.gate(tokens, input[1] if len(input) > 1 else None)
        E = self.ep_size * self.num_local_experts
        k = eidx.shape[1]
        flat_dst = (eidx * C + loc.clamp(min=0)).reshape(-1)           # [S*k]
        kept = (loc >= 0).reshape(-1)
        src_tok = torch.arange(S, device=x.device).repeat_interleave(k)
        kept_idx = kept.nonzero(as_tuple=True)[0]
        dispatched = tokens.new_zeros(E * C, d_model)
        dispatched = dispatched.index_copy(0, flat_dst[kept_idx], tokens.index_select(0, src_tok[kept_idx]))
        dispatched = dispatched.view(E, C, d_model)
        full_C = C
        drop = groups._get_expert_model_parallel_world_size() == 1 and tensor_parallel_world_size() > 1
        if drop:
            # tensor-parallel ranks hold the same tokens and the experts are not tensor parallel: each rank sends
            # only its share of the capacity slots (reference `sharded_moe.py:505-512`)
            dispatched = mappings.drop_tokens(dispatched, dim=1)
            C = dispatched.shape[1]
        # [E, C, M] grouped by destination rank: experts e = r*L + l live on EP rank r
        dispatched = _AllToAll.apply(self.ep_group, dispatched)
        # now [ep, L, C, M] of tokens from every rank for my L local experts -> [L, ep*C, M]
        L = self.num_local_experts
        local_in = dispatched.view(self.ep_size, L, C, d_model).transpose(0, 1).reshape(L * self.ep_size * C, d_model)
        expert_out = self._run_experts(local_in, L, C, d_model)
        back = expert_out.view(L, self.ep_size, C, d_model).transpose(0, 1).contiguous().view(E, C, d_model)
        back = _AllToAll.apply(self.ep_group, back)
        if drop:
            back = mappings.gather_tokens(back, dim=1)  # every tensor-parallel rank needs all tokens again
            C = full_C
        back = back.reshape(E * C, d_model)
        gathered = back.index_select(0, flat_dst[kept_idx]) * w.reshape(-1)[kept_idx].unsqueeze(1).to(back.dtype)
        out = tokens.new_zeros(S, d_model).index_add(0, src_tok[kept_idx], gathered)
        self.l_aux = l_aux
        self.exp_counts = exp_counts
        return out.view_as(x)

    def _run_experts(self, local_in, L, C, d_model):
        per = local_in.view(L, self.ep_size * C, d_model)
        outs = []
        for i, e in enumerate(self.experts.deepspeed_experts):
            o = e(per[i])
            outs.append(o[0] if isinstance(o, tuple) else o)
        return torch.stack(outs, 0).reshape(L * self.ep_size * C, d_model)
