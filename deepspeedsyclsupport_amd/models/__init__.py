from .llama import LlamaConfig, LlamaForCausalLM, llama2_7b_config  # noqa: F401
