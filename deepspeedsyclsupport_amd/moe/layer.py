"""MoE layer (reference `moe/layer.py:16-126`): same constructor and (output, l_aux, exp_counts) return."""
import typing

import torch

from ..parallel import groups
from ..utils.logging import log_dist
from .experts import Experts
from .sharded_moe import MOELayer, TopKGate


class MoE(torch.nn.Module):

    def __init__(self, hidden_size, expert, num_experts=1, ep_size=1, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, min_capacity=4, use_residual=False,
                 noisy_gate_policy: typing.Optional[str] = None, drop_tokens: bool = True, use_rts=True,
                 use_tutel: bool = False, enable_expert_tensor_parallelism: bool = False,
                 top2_2nd_expert_sampling=True):
        super().__init__()
        self.use_residual = use_residual
        self.enable_expert_tensor_parallelism = enable_expert_tensor_parallelism
        assert num_experts % ep_size == 0, \
            f"Number of experts ({num_experts}) should be divisible by expert parallel size ({ep_size})"
        self.ep_size = ep_size
        self.expert_group_name = f"ep_size_{self.ep_size}"
        self.num_experts = num_experts
        self.num_local_experts = num_experts // self.ep_size
        log_dist(f"Creating MoE layer with num_experts: {num_experts} | num_local_experts: {self.num_local_experts} | "
                 f"expert_parallel_size: {self.ep_size}", [0])
        assert noisy_gate_policy is None or noisy_gate_policy in ["None", "Jitter", "RSample"], \
            "Unsupported noisy_gate_policy: " + str(noisy_gate_policy)
        experts = Experts(expert, self.num_local_experts, self.expert_group_name)
        self.deepspeed_moe = MOELayer(TopKGate(hidden_size, num_experts, k, capacity_factor, eval_capacity_factor,
                                               min_capacity, noisy_gate_policy, drop_tokens, use_rts, None,
                                               top2_2nd_expert_sampling), experts, self.expert_group_name,
                                      self.ep_size, self.num_local_experts, use_tutel=use_tutel)
        if self.use_residual:
            self.mlp = expert
            self.coefficient = torch.nn.Linear(hidden_size, 2)
        self._create_process_groups()

    def set_deepspeed_parallelism(self, use_data_before_expert_parallel_=False):
        self._create_process_groups(use_data_before_expert_parallel_=use_data_before_expert_parallel_)

    def _create_process_groups(self, use_data_before_expert_parallel_=False):
        from .. import comm as dist
        if not dist.is_initialized():
            return
        if self.expert_group_name not in groups._get_expert_parallel_group_dict():
            if groups.mpu is None or not self.enable_expert_tensor_parallelism:
                # no tensor parallelism, or experts deliberately kept whole: expert groups span the world and the
                # MoE layer drops the tokens duplicated over tensor-parallel ranks (`moe/mappings.py`)
                groups._create_expert_and_data_parallel(
                    self.ep_size, use_data_before_expert_parallel_=use_data_before_expert_parallel_)
            else:
                groups._create_expert_data_and_model_parallel(
                    self.ep_size, mpu=groups.mpu, use_data_before_expert_parallel_=use_data_before_expert_parallel_)
        self.deepspeed_moe._set_ep_group(groups._get_expert_parallel_group(self.expert_group_name))

    def forward(self, hidden_states, used_token=None):
        output = self.deepspeed_moe(hidden_states, used_token)
        if self.use_residual:
            out_mlp = self.mlp(hidden_states)
            if isinstance(out_mlp, tuple):
                out_mlp = out_mlp[0]
            coef = torch.nn.functional.softmax(self.coefficient(hidden_states), dim=-1)
            output = output * coef[..., 0:1] + out_mlp * coef[..., 1:]
        return output, self.deepspeed_moe.l_aux, self.deepspeed_moe.exp_counts
