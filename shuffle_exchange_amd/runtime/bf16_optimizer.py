"""``BF16_Optimizer``: bf16 parameters, fp32 gradient accumulation, ZeRO-1 partitioned fp32 state.

Parity: reference runtime/bf16_optimizer.py:35 and its routing in runtime/engine.py:1384-1386
(bf16 + ZeRO stage 1 + ``data_types.grad_accum_dtype == "fp32"`` and no CPU offload), plus the
``bf16_zero_pp_rank_*`` checkpoint file prefix (engine.py:2927).

Here it is the stage-1 flat-unit optimizer (runtime/zero/stage12.py) with ``fp32_accum``: every
micro-step's bit16 gradient is added into a full-size fp32 buffer per unit as soon as autograd
produces it (the bit16 ``.grad`` never accumulates across micro-steps), and at the accumulation
boundary ONE reduce-scatter per unit -- in fp32 unless ``communication_data_type`` is set -- lands the
averaged fp32 chunk at its owner, whose fused HIP AdamW updates the fp32 master and writes the bf16
chunk; one all-gather per unit rebuilds the bf16 parameters. The reference instead all-reduces the
fp32 gradients of every rank (``get_grads_for_reduction``) and keeps fp32 copies of ALL gradients.
"""
from .fp16.loss_scaler import LossScaler
from .zero.stage12 import ZeroStage12Optimizer


class BF16_Optimizer(ZeroStage12Optimizer):

    def __init__(self, init_optimizer, param_names=None, bfloat16_config=None, mpu=None, clip_grad=0.0, norm_type=2,
                 allgather_bucket_size=5000000000, dp_process_group=None, timers=None, grad_acc_dtype=None,
                 graph_harvesting=False, immediate_grad_update=False, has_moe_layers=False, *, dp_ranks=None,
                 communication_data_type=None, overlap_comm=True, mp_group=None, loss_scaler=None,
                 shuffle_exchange_cfg=None):
        from ..parallel import groups
        if norm_type != 2:
            raise NotImplementedError("BF16_Optimizer clips by the global L2 norm only")
        if dp_ranks is None:
            dp_ranks = groups.group_ranks("seq_data")
        if dp_process_group is None:
            dp_process_group = groups.get_sequence_data_parallel_group()
        super().__init__(init_optimizer, stage=1, loss_scaler=loss_scaler or LossScaler(1.0), clip_grad=clip_grad,
                         dp_ranks=dp_ranks, dp_group=dp_process_group,
                         reduce_bucket_size=min(int(allgather_bucket_size), 500_000_000),
                         communication_data_type=communication_data_type, overlap_comm=overlap_comm,
                         shuffle_exchange_cfg=shuffle_exchange_cfg, mp_group=mp_group, timers=timers, fp32_accum=True)
        self.param_names = param_names or {}
        self.grad_acc_dtype = grad_acc_dtype

    # reference accessors (bf16_optimizer.py: fp32 master groups / their gradients)
    @property
    def fp32_groups_flat_partition(self):
        return list(self.master)

    @property
    def fp32_groups_gradients_flat(self):
        return list(self.grads)

    def state_dict(self):
        sd = super().state_dict()
        sd["bf16_optimizer"] = True
        return sd
