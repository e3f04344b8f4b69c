"""Ragged model implementations (reference inference/v2/model_implementations/).

* ``RaggedLlama``: serves this framework's own LlamaForCausalLM / MixtralForCausalLM training
  modules in place (no weight copy);
* ``RaggedDecoder`` (hf_decoder.py): Hugging Face checkpoints of the FastGen families -- Llama-2/3,
  Mistral, Mixtral, Qwen2, Qwen2-MoE, Phi, Phi-3, Falcon, OPT -- converted once into the packed
  layout of the gfx950 kernels.
"""
from .hf_decoder import RaggedDecoder, load_hf_decoder, spec_from_hf_config  # noqa: F401
from .llama import RaggedLlama  # noqa: F401


def ragged_model_for(model, weight_quant=None, tp_group=None, tp_size=1, pins=None):
    """Pick the ragged implementation for a model object (``weight_quant='fp8'``: row-scaled e4m3
    projection / LM-head weights for the decode GEMMs; ``tp_group``: tensor-parallel sharding)."""
    if isinstance(model, (RaggedDecoder, RaggedLlama)):
        if getattr(model, "tp", 1) != tp_size:
            raise ValueError(f"model was sharded for tp={getattr(model, 'tp', 1)}, engine tp_size={tp_size}: "
                             "build it with the same tensor_parallel config (build_hf_engine does)")
        return model
    if hasattr(model, "config") and hasattr(model.config, "model_type") and hasattr(model.config, "to_dict"):
        p = next(model.parameters())
        dtype = p.dtype if p.dtype in (__import__("torch").bfloat16, __import__("torch").float16,
                                       __import__("torch").float32) else None
        return load_hf_decoder(model, dtype=dtype, device=p.device, weight_quant=weight_quant, tp_group=tp_group,
                               tp_size=tp_size)
    if hasattr(model, "layers") and hasattr(model.layers[0], "self_attn") and hasattr(model, "embed_tokens"):
        return RaggedLlama(model, weight_quant=weight_quant, tp_group=tp_group, tp_size=tp_size, pins=pins)
    raise NotImplementedError(f"no ragged inference implementation for {type(model).__name__}")
