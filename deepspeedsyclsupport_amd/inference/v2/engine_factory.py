"""Build a ragged engine from a HF checkpoint directory or model (reference `inference/v2/engine_factory.py:65`)."""
import torch

from ..config import to_dtype
from ..model_implementations import convert
from .config_v2 import RaggedInferenceEngineConfig
from .engine_v2 import InferenceEngineV2


def build_hf_engine(path_or_model, engine_config: RaggedInferenceEngineConfig = None, debug_level=0,
                    dtype=torch.bfloat16, device=None):
    """`path_or_model`: a local HF checkpoint directory (loaded with safetensors/transformers, no network) or an
    already-instantiated HF / native model."""
    engine_config = engine_config or RaggedInferenceEngineConfig()
    if isinstance(path_or_model, str):
        import transformers
        model = transformers.AutoModelForCausalLM.from_pretrained(path_or_model, torch_dtype=torch.float32,
                                                                  local_files_only=True)
    else:
        model = path_or_model
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
            torch.device("cpu")
    tp = engine_config.tensor_parallel.tp_size
    group, rank = None, 0
    if tp > 1:
        from ... import comm as dist
        from ..engine import InferenceEngine
        group = InferenceEngine.inference_mp_group
        if group is None:
            world, me = dist.get_world_size(), dist.get_rank()
            for s in range(0, world, tp):
                g = dist.new_group(list(range(s, s + tp)))
                if s <= me < s + tp:
                    group = g
        rank = dist.get_rank(group)
    ds_model = convert.from_model(model, group, tp, rank, to_dtype(dtype), device,
                                  max_positions=engine_config.state_manager.max_context)
    q = engine_config.quantization.quantization_mode
    if q in ("int8", "int4"):
        ds_model.quantize_weights(8 if q == "int8" else 4)
    return InferenceEngineV2(ds_model, engine_config)
