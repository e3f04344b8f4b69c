"""Pipeline schedules as per-stage instruction streams.

Parity: reference runtime/pipe/schedule.py -- ``PipeSchedule`` :10, ``InferenceSchedule`` :135,
``TrainSchedule`` :189 (1F1B), ``DataParallelSchedule`` and the instruction set (``LoadMicroBatch``,
``ForwardPass``, ``BackwardPass``, ``SendActivation``, ``RecvActivation``, ``SendGrad``,
``RecvGrad``, ``ReduceGrads``, ``ReduceTiedGrads``, ``OptimizerStep``) :327-487.

The 1F1B order here is generated directly: stage ``s`` of ``S`` runs ``min(S-s-1, M)`` warm-up
forwards, then alternates one forward / one backward, then drains the remaining backwards. Each
yielded step is the list of instructions for one slot; buffer ids cycle over
``num_pipe_buffers()`` = the peak number of in-flight micro-batches on that stage (S - s).
"""


class PipeInstruction:
    def __init__(self, **kwargs):
        self.name = self.__class__.__name__
        self.kwargs = kwargs
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __repr__(self):
        args = ", ".join(f"{k}={v}" for k, v in self.kwargs.items())
        return f"{self.name}({args})"

    def __eq__(self, other):
        return type(self) is type(other) and self.kwargs == other.kwargs


class OptimizerStep(PipeInstruction):
    pass


class ReduceGrads(PipeInstruction):
    pass


class ReduceTiedGrads(PipeInstruction):
    pass


class BufferOpInstruction(PipeInstruction):
    def __init__(self, buffer_id, **kwargs):
        super().__init__(buffer_id=buffer_id, **kwargs)


class LoadMicroBatch(BufferOpInstruction):
    pass


class ForwardPass(BufferOpInstruction):
    pass


class BackwardPass(BufferOpInstruction):
    pass


class SendActivation(BufferOpInstruction):
    pass


class RecvActivation(BufferOpInstruction):
    pass


class SendGrad(BufferOpInstruction):
    pass


class RecvGrad(BufferOpInstruction):
    pass


class PipeSchedule:
    def __init__(self, micro_batches, stages, stage_id):
        self.micro_batches = int(micro_batches)
        self.stages = int(stages)
        self.stage_id = int(stage_id)
        self.prev_stage = self.stage_id - 1
        self.next_stage = self.stage_id + 1

    def steps(self):
        raise NotImplementedError

    def num_pipe_buffers(self):
        return self.micro_batches

    @property
    def is_first_stage(self):
        return self.stage_id == 0

    @property
    def is_last_stage(self):
        return self.stage_id == self.stages - 1

    def _buffer_idx(self, micro_batch_id):
        return micro_batch_id % self.num_pipe_buffers()

    def __iter__(self):
        return iter(self.steps())


class InferenceSchedule(PipeSchedule):
    """Forward only; two buffers alternate so the recv of i+1 can overlap the compute of i."""

    def num_pipe_buffers(self):
        return 2

    def steps(self):
        out = []
        for mb in range(self.micro_batches):
            buf = mb % 2
            cmds = []
            if self.is_first_stage or self.is_last_stage:
                cmds.append(LoadMicroBatch(buf))
            if not self.is_first_stage:
                cmds.append(RecvActivation(buf))
            cmds.append(ForwardPass(buf))
            if not self.is_last_stage:
                cmds.append(SendActivation(buf))
            out.append(cmds)
        return out


class TrainSchedule(PipeSchedule):
    """1F1B with a trailing gradient reduction and optimizer step."""

    def num_pipe_buffers(self):
        return max(2, min(self.stages - self.stage_id, self.micro_batches))

    def order(self):
        """[(kind, micro_batch)] with kind in {'F', 'B'} -- the per-stage 1F1B sequence."""
        M = self.micro_batches
        warm = min(self.stages - self.stage_id - 1, M)
        seq = [("F", i) for i in range(warm)]
        f, b = warm, 0
        while f < M:
            seq.append(("F", f))
            f += 1
            seq.append(("B", b))
            b += 1
        while b < M:
            seq.append(("B", b))
            b += 1
        return seq

    def steps(self):
        out = []
        for kind, mb in self.order():
            buf = self._buffer_idx(mb)
            cmds = []
            if kind == "F":
                if self.is_first_stage or self.is_last_stage:
                    cmds.append(LoadMicroBatch(buf))
                if not self.is_first_stage:
                    cmds.append(RecvActivation(buf))
                cmds.append(ForwardPass(buf))
                if not self.is_last_stage:
                    cmds.append(SendActivation(buf))
            else:
                if not self.is_last_stage:
                    cmds.append(RecvGrad(buf))
                cmds.append(BackwardPass(buf))
                if not self.is_first_stage:
                    cmds.append(SendGrad(buf))
            out.append(cmds)
        out.append([ReduceTiedGrads(), ReduceGrads(), OptimizerStep()])
        return out


class DataParallelSchedule(PipeSchedule):
    """Single stage: plain gradient accumulation."""

    def num_pipe_buffers(self):
        return 1

    def steps(self):
        out = []
        for mb in range(self.micro_batches):
            out.append([LoadMicroBatch(0), ForwardPass(0), BackwardPass(0)])
        out.append([ReduceTiedGrads(), ReduceGrads(), OptimizerStep()])
        return out
