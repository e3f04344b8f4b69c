"""Domino: tensor parallelism with the TP all-reduces hidden behind compute.

Parity: reference runtime/domino/transformer.py -- ``DominoTransformerLayer`` :250 (input split
into two micro-batches along the batch dim, ``intra_layer_overlap_forward`` :591: attention of
micro-batch 1 runs while micro-batch 0's attention all-reduce is in flight, then the same for the
MLP), ``ShardedAttention`` :108, ``NoOper`` :54 (backward-side wait), and
runtime/domino/async_linear.py (``DominoAsyncColumnParallelLinear`` whose backward launches the
input-grad all-reduce asynchronously and computes the weight grad under it).

MI355X design: instead of a separate Megatron-style transformer implementation, Domino is a
*schedule* applied to this repo's AutoTP-sharded decoder layers (``apply_domino`` re-classes
each ``LlamaDecoderLayer`` in place, so parameter names, ZeRO units and checkpoints are
unchanged). Forward row-parallel all-reduces are launched with ``async_op=True`` (RCCL's own
stream; the compute stream only waits where the reduced value is consumed); backward
column-parallel input-grad all-reduces are parked and waited one node later
(``wait_grad_handles``). With 8 GPUs of one node in a TP group every all-reduce is a ring over
the xGMI mesh, ~2 x (tp-1)/tp x activation bytes per link -- exactly the traffic that two
micro-batches can hide behind each other's GEMMs.
"""
import torch

from ... import comm as dist
from ...models.llama import LlamaDecoderLayer
from ...module_inject.layers import LinearAllreduce, LinearLayer, wait_grad_handles
from ...ops.activation import swiglu
from ...ops.attention import attention_qkv_rope


class _AsyncAllReduce(torch.autograd.Function):
    """Launch an in-place async SUM all-reduce; the Work goes into ``box``. Identity backward
    (row-parallel output)."""

    @staticmethod
    def forward(ctx, x, group, box):
        x = x.contiguous()
        box.append(dist.all_reduce(x, group=group, async_op=True))
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None, None


class _WaitAllReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, box):
        box.pop(0).wait()
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


def _split(t, n):
    return [None] * n if t is None else list(t.chunk(n, dim=0))


class DominoLlamaDecoderLayer(LlamaDecoderLayer):
    """Two-micro-batch overlapped schedule of a TP-sharded Llama decoder layer."""

    domino_micro_batches = 2
    overlapped_calls = 0  # forward calls that took the overlapped schedule (observability / tests)

    def forward(self, x, residual, rope, position_ids=None):
        attn, mlp = self.self_attn, self.mlp
        group = attn.o_proj.tp_group
        n = self.domino_micro_batches
        if x.shape[0] < n or group is None or dist.get_world_size(group) == 1:
            return super().forward(x, residual, rope, position_ids)
        DominoLlamaDecoderLayer.overlapped_calls += 1
        xs, rs, ps = _split(x, n), _split(residual, n), _split(position_ids, n)
        gh = [[] for _ in range(n)]  # backward input-grad all-reduce handles per micro-batch
        fbox = [[] for _ in range(n)]  # forward all-reduce handles per micro-batch
        # ---- attention: micro-batch i+1's QKV/flash/o_proj GEMMs run under i's all-reduce
        pend = []
        for i in range(n):
            if rs[i] is None:
                a, h = self.input_layernorm(xs[i]), xs[i]
            else:
                a, h = self.input_layernorm(xs[i], rs[i])
            a = wait_grad_handles(a, gh[i])
            B, S = a.shape[0], a.shape[1]
            qkv = attn.qkv_proj(a, grad_handles=gh[i]).view(B, S, attn.nq + 2 * attn.nkv, attn.d)
            o = attention_qkv_rope(qkv, attn.nq, attn.nkv, rope, ps[i], causal=True)
            y = attn.o_proj.forward_partial(o.reshape(B, S, attn.nq * attn.d))
            pend.append((_AsyncAllReduce.apply(y, group, fbox[i]), h))
        # ---- MLP: consume micro-batch i's reduced attention output, overlap its MLP with the rest
        outs = []
        for i in range(n):
            y, h = pend[i]
            y = _WaitAllReduce.apply(y, fbox[i])
            if attn.o_proj.bias is not None:
                y = y + attn.o_proj.bias
            m, h2 = self.post_attention_layernorm(y, h)
            m = wait_grad_handles(m, gh[i])
            z = mlp.down_proj.forward_partial(swiglu(mlp.gate_up_proj(m, grad_handles=gh[i])))
            outs.append((_AsyncAllReduce.apply(z, group, fbox[i]), h2))
        ys, hs = [], []
        for i in range(n):
            z, h2 = outs[i]
            z = _WaitAllReduce.apply(z, fbox[i])
            if mlp.down_proj.bias is not None:
                z = z + mlp.down_proj.bias
            ys.append(z)
            hs.append(h2)
        return torch.cat(ys, dim=0), torch.cat(hs, dim=0)


def apply_domino(model, micro_batches=2):
    """Switch every AutoTP-sharded Llama decoder layer of ``model`` to the Domino schedule.
    The model must already be tensor-parallel (``tp_model_init`` / engine ``tensor_parallel``)."""
    n = 0
    for m in model.modules():
        if type(m) is LlamaDecoderLayer:
            assert isinstance(m.self_attn.qkv_proj, LinearLayer) and isinstance(m.self_attn.o_proj, LinearAllreduce), \
                "apply_domino needs a tensor-parallel model (run AutoTP first)"
            m.__class__ = DominoLlamaDecoderLayer
            m.domino_micro_batches = micro_batches
            n += 1
    model._sxe_domino = n
    return model
