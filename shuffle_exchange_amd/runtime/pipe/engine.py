"""Pipeline-parallel training engine: executes a per-stage instruction schedule (1F1B).

Parity: reference runtime/pipe/engine.py -- ``PipelineEngine`` :61, ``train_batch`` :338,
``eval_batch`` :427, ``_exec_schedule`` :1409 with ``_INSTRUCTION_MAP`` :1396, instruction
handlers (``_exec_load_micro_batch`` :775, ``_exec_forward_pass`` :640, ``_exec_backward_pass``
:716, ``_exec_send_activations`` :982, ``_exec_recv_activations`` :1052, ``_exec_send_grads``
:1008, ``_exec_recv_grads`` :1103, ``_exec_reduce_tied_grads`` :278, ``_exec_reduce_grads`` :286,
``_exec_optimizer_step`` :1163), ``_aggregate_total_loss`` :548. ZeRO-2/3 are rejected as in the
reference (:77-78); ZeRO-0/1 are supported.

Gradient flow per batch: all micro-batch backwards accumulate into ``param.grad`` (the optimizer's
accumulation boundary is held off), tied-weight grads are summed over their stage group, then the
ZeRO optimizer reduces everything in one epilogue and steps.
"""
import torch

from ... import comm as dist
from ...utils.logging import log_dist
from ..engine import SXEEngine
from . import schedule as S
from .p2p import P2PChannel


class PipelineError(Exception):
    pass


def _tuple(x):
    return x if isinstance(x, tuple) else ((x,) if torch.is_tensor(x) else tuple(x))


class PipelineEngine(SXEEngine):
    def __init__(self, *args, has_bool_tensors=False, **kwargs):
        super().__init__(*args, **kwargs)
        assert self.zero_optimization_stage() < 2, "ZeRO-2 and ZeRO-3 are incompatible with pipeline parallelism"
        self.grid = self.module.mpu()
        self.num_stages = self.grid.pipe_parallel_size
        self.stage_id = self.grid.get_stage_id()
        self.prev_stage, self.next_stage = self.stage_id - 1, self.stage_id + 1
        self.micro_batches = self.gradient_accumulation_steps()
        self.p2p = P2PChannel(self.grid, self.device)
        self.batch_fn = None
        self.data_iterator = None
        self.total_loss = None
        self.agg_train_loss = None
        self.loss = None
        self._force_grad_boundary = False
        if self.training_dataloader is not None:
            from ..dataloader import RepeatingLoader
            self.data_iterator = iter(RepeatingLoader(self.training_dataloader))
        # tied weights are summed across stages before the ZeRO reduction: keep their grads in .grad
        for p in self.module.tied_parameters():
            for a in ("_sxe_grad_target", "_sxe_grad_done"):
                if hasattr(p, a):
                    delattr(p, a)
        n_local = sum(p.numel() for p in self.module.parameters())
        log_dist(f"pipeline: {self.num_stages} stages, micro_batches={self.micro_batches}, stage {self.stage_id} "
                 f"holds {n_local} params", ranks=[0])

    def _norm_group(self):
        grid = self.module.mpu()
        if grid.get_slice_parallel_world_size() > 1:
            return grid.get_slice_parallel_group()
        return super()._norm_group()

    # ------------------------------------------------------------------------------- public API
    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.num_stages - 1

    def set_batch_fn(self, fn):
        self.batch_fn = fn

    def set_dataiterator(self, iterator):
        self.data_iterator = iterator

    def forward(self, *a, **k):
        raise PipelineError("Only train_batch() / eval_batch() are accessible with pipeline parallelism")

    def backward(self, *a, **k):
        raise PipelineError("Only train_batch() / eval_batch() are accessible with pipeline parallelism")

    def step(self, *a, **k):
        raise PipelineError("Only train_batch() / eval_batch() are accessible with pipeline parallelism")

    def train_batch(self, data_iter=None):
        if data_iter is not None:
            self.data_iterator = data_iter
        self.module.train()
        self.total_loss = None
        sched = S.TrainSchedule(self.micro_batches, self.num_stages, self.stage_id)
        self._exec_schedule(sched)
        self.agg_train_loss = self._aggregate_total_loss()
        return self.agg_train_loss

    def eval_batch(self, data_iter, return_logits=False, compute_loss=True, reduce_output="avg",
                   num_micro_batches=None):
        self.module.eval()
        self.data_iterator = data_iter
        self.total_loss = None
        self._eval_outputs = []
        self._eval_compute_loss = compute_loss
        sched = S.InferenceSchedule(num_micro_batches or self.micro_batches, self.num_stages, self.stage_id)
        with torch.no_grad():
            self._exec_schedule(sched)
        if compute_loss:
            out = self._aggregate_total_loss(reduce_output == "avg")
        else:
            out = None
        if return_logits:
            return out, self._eval_outputs if self.is_last_stage() else None
        return out

    # ------------------------------------------------------------------------------ execution
    def _exec_schedule(self, sched):
        nb = sched.num_pipe_buffers()
        self.buffers = {k: [None] * nb for k in ("inputs", "labels", "outputs", "loss", "grads")}
        self._sent_meta = False
        self._recv_meta = None
        self._n_micro = sched.micro_batches
        self.optimizer.set_gradient_accumulation_boundary(False)
        self.optimizer.backward_prologue()
        try:
            for step in sched.steps():
                for cmd in step:
                    getattr(self, "_exec_" + _HANDLER[type(cmd)])(**cmd.kwargs)
        finally:
            self.p2p.wait_sends()

    def _next_batch(self):
        batch = next(self.data_iterator)
        if self.batch_fn is not None:
            batch = self.batch_fn(batch)
        return batch

    def _to_dev(self, x):
        if torch.is_tensor(x):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (tuple, list)):
            return type(x)(self._to_dev(t) for t in x)
        return x

    def _exec_load_micro_batch(self, buffer_id):
        batch = self._next_batch()
        inputs, labels = (batch[0], batch[1]) if isinstance(batch, (tuple, list)) and len(batch) == 2 else (batch, None)
        if self.is_first_stage():
            self.buffers["inputs"][buffer_id] = self._to_dev(inputs)
        if self.is_last_stage():
            self.buffers["labels"][buffer_id] = self._to_dev(labels)

    def _exec_forward_pass(self, buffer_id):
        x = self.buffers["inputs"][buffer_id]
        out = self.module(x)
        self.buffers["outputs"][buffer_id] = out
        if self.is_last_stage():
            labels = self.buffers["labels"][buffer_id]
            loss_fn = self.module.loss_fn
            compute = getattr(self, "_eval_compute_loss", True) or self.module.training
            if loss_fn is not None and compute:
                loss = loss_fn(out, labels)
            else:
                loss = out
            if not self.module.training:
                self._eval_outputs.append(out.detach() if torch.is_tensor(out) else out)
            self.buffers["loss"][buffer_id] = loss
            if torch.is_tensor(loss) and loss.dim() == 0:
                l = loss.detach().float()
                self.total_loss = l.clone() if self.total_loss is None else self.total_loss + l
        if not self.module.training:
            self.buffers["inputs"][buffer_id] = None

    def _exec_backward_pass(self, buffer_id):
        opt = self.optimizer
        if self.is_last_stage():
            loss = self.buffers["loss"][buffer_id]
            scaled = loss / self._n_micro
            if self.fp16_enabled():
                scaled = scaled * opt.loss_scale
            scaled.backward()
        else:
            outs = _tuple(self.buffers["outputs"][buffer_id])
            grads = self.buffers["grads"][buffer_id]
            ts = [t for t in outs if torch.is_tensor(t) and t.requires_grad]
            assert len(ts) == len(grads), "gradient count does not match activations requiring grad"
            torch.autograd.backward(ts, grads)
        self.buffers["outputs"][buffer_id] = None
        self.buffers["grads"][buffer_id] = None
        self.buffers["loss"][buffer_id] = None

    def _exec_send_activations(self, buffer_id):
        out = _tuple(self.buffers["outputs"][buffer_id])
        if not self._sent_meta:
            self.p2p.send_meta(out, self.next_stage)
            self._sent_meta = True
        self.p2p.send(out, self.next_stage)

    def _exec_recv_activations(self, buffer_id):
        if self._recv_meta is None:
            self._recv_meta = self.p2p.recv_meta(self.prev_stage)
        ts = self.p2p.recv(self._recv_meta, self.prev_stage)
        for t, (dt, rg, _) in zip(ts, self._recv_meta):
            if rg and t.is_floating_point() and self.module.training:
                t.requires_grad_(True)
        self.buffers["inputs"][buffer_id] = ts[0] if len(ts) == 1 else tuple(ts)

    def _exec_send_grads(self, buffer_id):
        ins = _tuple(self.buffers["inputs"][buffer_id])
        gs = []
        for t in ins:
            if torch.is_tensor(t) and t.requires_grad:
                gs.append(t.grad if t.grad is not None else torch.zeros_like(t))
        self.p2p.send(gs, self.prev_stage)
        self.buffers["inputs"][buffer_id] = None

    def _exec_recv_grads(self, buffer_id):
        outs = _tuple(self.buffers["outputs"][buffer_id])
        meta = [(t.dtype, False, tuple(t.shape)) for t in outs if torch.is_tensor(t) and t.requires_grad]
        self.buffers["grads"][buffer_id] = self.p2p.recv(meta, self.next_stage)

    def _exec_reduce_tied_grads(self):
        self.module.allreduce_tied_weight_gradients()

    def _exec_reduce_grads(self):
        opt = self.optimizer
        opt.set_gradient_accumulation_boundary(True)
        opt.backward_prologue()
        opt.reduce_gradients()

    def _exec_optimizer_step(self):
        self._take_model_step()
        self.micro_steps += self._n_micro

    # ------------------------------------------------------------------------------ loss
    def _aggregate_total_loss(self, average=True):
        """Mean loss over micro-batches (and data-parallel replicas), known on every rank."""
        last = self.grid.stage_to_global(self.num_stages - 1)
        if self.is_last_stage():
            loss = (self.total_loss if self.total_loss is not None else torch.zeros((), device=self.device))
            loss = (loss / self._n_micro if average else loss).reshape(1).float()
            dpg = self.grid.get_data_parallel_group()
            if self.grid.get_data_parallel_world_size() > 1:
                dist.all_reduce(loss, group=dpg)
                loss /= self.grid.get_data_parallel_world_size()
        else:
            loss = torch.zeros(1, device=self.device)
        if self.num_stages > 1:
            dist.broadcast(loss, src=last, group=self.grid.get_pipe_parallel_group())
        return loss.squeeze(0)

    # --------------------------------------------------------------------------- checkpoints
    def module_state_dict(self, exclude_frozen_parameters=False):
        return None  # layer files are written by save_checkpoint via the PipelineModule

    def save_checkpoint(self, save_dir, tag=None, client_state=None, save_latest=True,
                        exclude_frozen_parameters=False):
        import os
        tag = str(tag if tag is not None else f"global_step{self.global_steps}")
        self.module.save_state_dict(os.path.join(save_dir, tag), exclude_frozen_params=exclude_frozen_parameters)
        return super().save_checkpoint(save_dir, tag=tag, client_state=client_state, save_latest=save_latest,
                                       exclude_frozen_parameters=exclude_frozen_parameters)

    def _ckpt_names(self, save_dir, tag):
        import os
        d = os.path.join(save_dir, str(tag))
        pp = self.stage_id
        dp = self.grid.get_data_parallel_rank()
        model = os.path.join(d, f"mp_rank_{pp:02d}_model_states.pt")
        optim = os.path.join(d, f"zero_pp_rank_{dp}_mp_rank_{pp:02d}_optim_states.pt")
        return d, model, optim

    def load_checkpoint(self, load_dir, tag=None, **kw):
        import os
        if tag is None:
            with open(os.path.join(load_dir, "latest")) as f:
                tag = f.read().strip()
        self.module.load_state_dir(os.path.join(load_dir, str(tag)))
        return super().load_checkpoint(load_dir, tag=tag, **kw)


_HANDLER = {
    S.OptimizerStep: "optimizer_step",
    S.ReduceGrads: "reduce_grads",
    S.ReduceTiedGrads: "reduce_tied_grads",
    S.LoadMicroBatch: "load_micro_batch",
    S.ForwardPass: "forward_pass",
    S.BackwardPass: "backward_pass",
    S.SendActivation: "send_activations",
    S.RecvActivation: "recv_activations",
    S.SendGrad: "send_grads",
    S.RecvGrad: "recv_grads",
}
