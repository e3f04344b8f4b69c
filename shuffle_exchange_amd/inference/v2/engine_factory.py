"""Build a ragged inference engine from a Hugging Face model or checkpoint directory.

Parity: reference inference/v2/engine_factory.py:69-133 ``build_hf_engine(path, engine_config,
debug_level)`` -- reads the checkpoint's ``config.json``, picks the model implementation by
``model_type`` (llama / mistral / mixtral / opt / falcon / phi / phi3 / qwen2 / qwen2_moe) and
returns an ``InferenceEngineV2``. No hub access here: ``path`` is a local directory (or an
already-instantiated transformers model); weights are read with safetensors / ``weights_only``.
"""
import torch

from .engine_v2 import InferenceEngineV2, RaggedInferenceEngineConfig
from .model_implementations.hf_decoder import load_hf_decoder


def build_hf_engine(path_or_model, engine_config: RaggedInferenceEngineConfig = None, dtype=torch.bfloat16,
                    device=None, debug_level=None, weight_quant=None):
    """``weight_quant='fp8'``: row-scaled e4m3 projection / LM-head weights (ops/fp_quantizer.FP8Weight)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    tp = int(((engine_config.tensor_parallel if engine_config is not None else None) or {}).get("tp_size", 1))
    tp_group = None
    if tp > 1:  # every rank loads the checkpoint and keeps its shard (reference sharding/*.py)
        from .engine_v2 import _tp_group
        tp_group = _tp_group(tp)
    model = load_hf_decoder(path_or_model, dtype=dtype, device=device, weight_quant=weight_quant, tp_group=tp_group,
                            tp_size=tp)
    return InferenceEngineV2(model, engine_config)


def build_engine_from_ds_checkpoint(path, engine_config: RaggedInferenceEngineConfig = None, debug_level=None):
    """Rebuild an engine from ``InferenceEngineV2.serialize`` output (reference engine_factory.py:32-66);
    see serialization.py."""
    from .serialization import build_engine_from_ds_checkpoint as _build
    return _build(path, engine_config, debug_level)
