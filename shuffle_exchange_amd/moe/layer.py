"""``MoE`` layer (parity: reference deepspeed/moe/layer.py:17-132).

``MoE(hidden_size, expert, num_experts, ep_size, k, capacity_factor, eval_capacity_factor,
min_capacity, use_residual, noisy_gate_policy, drop_tokens, use_rts, ...)`` returns
``(output, l_aux, exp_counts)`` like the reference. Expert-parallel groups are created lazily on
first forward (``set_deepspeed_parallelism``) from ``parallel.groups``; on one 8-GPU MI355X node the
EP all-to-all is a full-mesh exchange over the 7 xGMI links of each GPU.
"""
import torch
import torch.nn as nn

from ..parallel import groups
from .experts import Experts, GroupedSwiGLUExperts
from .sharded_moe import MOELayer, TopKGate


class MoE(nn.Module):
    def __init__(self, hidden_size, expert=None, num_experts=1, ep_size=1, k=1, capacity_factor=1.0,
                 eval_capacity_factor=1.0, min_capacity=4, use_residual=False, noisy_gate_policy=None,
                 drop_tokens=True, use_rts=True, use_tutel=False, enable_expert_tensor_parallelism=False,
                 top2_2nd_expert_sampling=True, intermediate_size=None, drop_policy="probs"):
        super().__init__()
        assert num_experts % ep_size == 0, f"num_experts ({num_experts}) must be divisible by ep_size ({ep_size})"
        self.use_residual = use_residual
        self.enable_expert_tensor_parallelism = enable_expert_tensor_parallelism
        self.ep_size = ep_size
        self.num_experts = num_experts
        self.num_local_experts = num_experts // ep_size
        self.expert_group_name = f"ep_size_{ep_size}"
        if expert is None:
            assert intermediate_size is not None, "either an expert module or intermediate_size (SwiGLU experts)"
            experts = GroupedSwiGLUExperts(hidden_size, intermediate_size, self.num_local_experts,
                                           self.expert_group_name)
        else:
            experts = Experts(expert, self.num_local_experts, self.expert_group_name)
        self.deepspeed_moe = MOELayer(
            TopKGate(hidden_size, num_experts, k, capacity_factor, eval_capacity_factor, min_capacity,
                     noisy_gate_policy, drop_tokens, use_rts, None, top2_2nd_expert_sampling, drop_policy),
            experts, self.expert_group_name, self.ep_size, self.num_local_experts)
        if self.use_residual:
            self.mlp = expert
            self.coefficient = nn.Linear(hidden_size, 2)
        self._groups_ready = False

    def set_deepspeed_parallelism(self, use_data_before_expert_parallel_=False):
        """Create (once) this layer's expert-parallel / expert-data-parallel groups and wire the
        TP token drop/gather (reference layer.py:98-111, groups.py:240 / :383). With tensor
        parallelism and ``enable_expert_tensor_parallelism`` the experts are sharded over the TP
        group here (GroupedSwiGLUExperts: gate/up columns, down rows); without it the EP group
        spans the TP ranks. The engine calls this after AutoTP and before the model broadcast."""
        if self._groups_ready:
            return
        tp = groups.get_tensor_model_parallel_world_size()
        expert_tp = self.enable_expert_tensor_parallelism and tp > 1
        name = groups.create_expert_and_data_parallel(self.ep_size, self.expert_group_name,
                                                      span_tp=tp > 1 and not expert_tp)
        tp_group = groups.get_tensor_model_parallel_group() if tp > 1 else None
        self.deepspeed_moe._set_ep_group(groups.get_expert_parallel_group(name), tp_group, expert_tp)
        if expert_tp:
            experts = self.deepspeed_moe.experts
            if hasattr(experts, "expert_tp_shard_"):
                experts.expert_tp_shard_(tp_group)
            for p in experts.parameters():  # user expert modules shard themselves (reference semantics)
                p.tensor_model_parallel = True
        self._groups_ready = True

    @property
    def expert_tp_rank(self):
        """Model-parallel index of this rank's expert shards in checkpoint file names (0 when the
        experts are not TP-sharded: they are then independent of the TP degree)."""
        if self.deepspeed_moe.expert_tp:
            return groups.get_tensor_model_parallel_rank()
        return 0

    def forward(self, hidden_states, used_token=None):
        if not self._groups_ready:
            self.set_deepspeed_parallelism()
        out = self.deepspeed_moe(hidden_states, used_token)
        if self.use_residual:
            mlp_out = self.mlp(hidden_states)
            if isinstance(mlp_out, tuple):
                mlp_out = mlp_out[0]
            coef = torch.softmax(self.coefficient(hidden_states), dim=-1)
            out = out * coef[..., 0:1] + mlp_out * coef[..., 1:]
        return out, self.deepspeed_moe.l_aux, self.deepspeed_moe.exp_counts
