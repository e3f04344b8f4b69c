"""Ragged model implementations (reference inference/v2/model_implementations/)."""
from .llama import RaggedLlama  # noqa: F401


def ragged_model_for(model):
    """Pick the ragged implementation for a framework model (Llama-family incl. Mixtral)."""
    if hasattr(model, "layers") and hasattr(model.layers[0], "self_attn") and hasattr(model, "embed_tokens"):
        return RaggedLlama(model)
    raise NotImplementedError(f"no ragged inference implementation for {type(model).__name__}")
