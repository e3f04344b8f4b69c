"""Pipeline parallelism (parity: reference runtime/pipe/)."""
from .module import LayerSpec, PipelineModule, TiedLayerSpec  # noqa: F401
from .schedule import (BackwardPass, DataParallelSchedule, ForwardPass, InferenceSchedule,  # noqa: F401
                       LoadMicroBatch, OptimizerStep, PipeInstruction, PipeSchedule, RecvActivation, RecvGrad,
                       ReduceGrads, ReduceTiedGrads, SendActivation, SendGrad, TrainSchedule)
from ...parallel.topology import PipeDataParallelTopology, PipeModelDataParallelTopology, ProcessTopology  # noqa: F401,E501
