"""Public pipeline API (reference ``deepspeed.pipe``)."""
from ..runtime.pipe import (LayerSpec, PipeDataParallelTopology, PipeModelDataParallelTopology,  # noqa: F401
                            PipelineModule, ProcessTopology, TiedLayerSpec)
