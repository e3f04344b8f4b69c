from .evoformer_attn import DS4Sci_EvoformerAttention, EvoformerFusedAttention  # noqa: F401
