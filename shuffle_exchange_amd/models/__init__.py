from .llama import LlamaConfig, LlamaForCausalLM, llama_config  # noqa: F401
from .gpt2 import GPT2Config, GPT2LMHeadModel, gpt2_config  # noqa: F401
from .mixtral import MixtralConfig, MixtralForCausalLM, mixtral_config  # noqa: F401
