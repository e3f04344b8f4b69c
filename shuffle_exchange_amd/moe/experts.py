"""Expert containers (parity: reference deepspeed/moe/experts.py:13 ``Experts``).

``Experts``        generic: deep copies of any expert module, run one after another on their
                   capacity block (the reference's behaviour).
``GroupedSwiGLUExperts`` MI355X fast path for Llama/Mixtral experts: the E_local experts' weights
                   are stacked, so gate|up and down are each ONE batched hipBLASLt GEMM over
                   [E_local, tokens, H] with the HIP SwiGLU kernel between them.
Every expert parameter is tagged ``allreduce = False`` and ``group_name`` (reference convention)
so the ZeRO optimizers reduce its gradient over the expert-data-parallel group only.
"""
import copy

import torch
import torch.nn as nn

from ..ops.activation import swiglu


class Experts(nn.Module):
    def __init__(self, expert, num_local_experts=1, expert_group_name=None):
        super().__init__()
        self.deepspeed_experts = nn.ModuleList([copy.deepcopy(expert) for _ in range(num_local_experts)])
        self.num_local_experts = num_local_experts
        for e in self.deepspeed_experts:
            for p in e.parameters():
                p.allreduce = False
                p.group_name = expert_group_name

    def forward(self, inputs):
        # inputs: [E_local, tokens, H]
        outs = [e(chunk) for chunk, e in zip(inputs.unbind(0), self.deepspeed_experts)]
        out = []
        for o in outs:
            out.append(o[0] if isinstance(o, tuple) else o)
        return torch.stack(out, dim=0)


class GroupedSwiGLUExperts(nn.Module):
    def __init__(self, hidden_size, intermediate_size, num_local_experts, expert_group_name=None, init_std=0.02):
        super().__init__()
        self.num_local_experts = num_local_experts
        self.w_gate_up = nn.Parameter(torch.empty(num_local_experts, hidden_size, 2 * intermediate_size))
        self.w_down = nn.Parameter(torch.empty(num_local_experts, intermediate_size, hidden_size))
        with torch.no_grad():
            self.w_gate_up.normal_(0.0, init_std)
            self.w_down.normal_(0.0, init_std)
        for p in (self.w_gate_up, self.w_down):
            p.allreduce = False
            p.group_name = expert_group_name

    def forward(self, x):
        # x: [E_local, C, H] -> per expert [C, H] @ [H, 2I] -> SwiGLU (one HIP launch over all
        # experts) -> [C, I] @ [I, H]. Plain 2-D GEMMs per expert rather than torch.bmm: at
        # Mixtral-8x7B sizes (C = 1280 tokens, H = 4096, I = 14336) each GEMM is 30-150 GFLOP, so
        # batching buys nothing, and the strided-batched backward of bmm under the TunableOp
        # lookup-only GEMM path faulted on MI355X (illegal address in the autograd thread).
        gu = torch.stack([torch.matmul(x[e], self.w_gate_up[e]) for e in range(self.num_local_experts)])
        h = swiglu(gu)
        return torch.stack([torch.matmul(h[e], self.w_down[e]) for e in range(self.num_local_experts)])
