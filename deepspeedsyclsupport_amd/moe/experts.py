"""Local experts of an MoE layer (reference `moe/experts.py`)."""
import copy

import torch


class Experts(torch.nn.Module):

    def __init__(self, expert, num_local_experts=1, expert_group_name=None):
        super().__init__()
        self.deepspeed_experts = torch.nn.ModuleList([copy.deepcopy(expert) for _ in range(num_local_experts)])
        self.num_local_experts = num_local_experts
        for e in self.deepspeed_experts:
            for p in e.parameters():
                p.allreduce = False
                p.group_name = expert_group_name

    def forward(self, inputs):
        # inputs [num_local_experts, T, M] -> same shape
        chunks = inputs.chunk(self.num_local_experts, dim=0)
        outs = []
        for chunk, expert in zip(chunks, self.deepspeed_experts):
            out = expert(chunk)
            if isinstance(out, tuple):
                out = out[0]
            outs.append(out)
        return torch.cat(outs, dim=0)
