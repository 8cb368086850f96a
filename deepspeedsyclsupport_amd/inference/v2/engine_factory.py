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
        import os
        if os.path.exists(os.path.join(path_or_model, "ds_model_config.json")):
            return build_engine_from_ds_checkpoint(path_or_model, engine_config, debug_level, device)
        from .checkpoint import HuggingFaceCheckpointEngine
        from .model_implementations import POLICIES
        ckpt = HuggingFaceCheckpointEngine(path_or_model)
        policy_cls = POLICIES.get(ckpt.model_config.model_type)
        if policy_cls is not None:
            # streamed load: checkpoint tensors go layer by layer into the sharded device model
            return _engine_from_policy(policy_cls(ckpt.model_config, checkpoint_engine=ckpt), engine_config, dtype)
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
    else:
        _apply_decode_layout(ds_model, engine_config.decode_layout, tp, device)
    return InferenceEngineV2(ds_model, engine_config)


def _tp_group(tp):
    """The tensor-parallel group of this rank (consecutive ranks), created on first use."""
    from ... import comm as dist
    from ..engine import InferenceEngine
    group = InferenceEngine.inference_mp_group
    if group is None:
        world, me = dist.get_world_size(), dist.get_rank()
        for s in range(0, world, tp):
            g = dist.new_group(list(range(s, s + tp)))
            if s <= me < s + tp:
                group = g
    return group


def _engine_from_policy(policy, engine_config, dtype=torch.bfloat16):
    """Policy (checkpoint engine + containers) -> model -> engine (reference `engine_factory.py:65-129`)."""
    tp = engine_config.tensor_parallel.tp_size
    policy.dtype = dtype
    ds_model = policy.build_model(engine_config, _tp_group(tp) if tp > 1 else None)
    q = engine_config.quantization.quantization_mode
    if q in ("int8", "int4"):
        ds_model.quantize_weights(8 if q == "int8" else 4)
    else:
        _apply_decode_layout(ds_model, engine_config.decode_layout, tp, torch.device(ds_model.device))
    return InferenceEngineV2(ds_model, engine_config)


def _apply_decode_layout(ds_model, mode, tp, device):
    """Same policy as `InferenceEngine._apply_decode_layout` (a shuffled copy of the bf16 projection weights)."""
    if mode == "row_major" or tp != 1 or device.type != "cuda" or ds_model.dtype != torch.bfloat16:
        return
    if mode == "shuffled":
        ds_model.quantize_weights(16)
    elif mode == "both" or ds_model.projection_bytes() <= torch.cuda.get_device_properties(device).total_memory // 4:
        ds_model.add_decode_layout()


def build_engine_from_ds_checkpoint(path, engine_config: RaggedInferenceEngineConfig = None, debug_level=0,
                                    device=None):
    """Rebuild an engine from `InferenceEngineV2.serialize(path)` output (reference `engine_factory.py:28`): the
    model spec JSON plus this rank's safetensors shard — no HF checkpoint or transformers model needed. The job's
    tensor-parallel degree must match the one the shards were written at."""
    import json
    import os

    from safetensors.torch import load_file

    from ..model_implementations.transformer import DSInferenceModel, DSModelSpec
    engine_config = engine_config or RaggedInferenceEngineConfig()
    with open(os.path.join(path, "ds_model_config.json")) as f:
        fields = json.load(f)
    fields["layer_windows"] = tuple(fields.get("layer_windows", ()))
    spec = DSModelSpec(**fields)
    meta_path = os.path.join(path, "ds_model_meta.json")
    meta = json.load(open(meta_path)) if os.path.exists(meta_path) else {"dtype": "bfloat16", "tp_size": 1}
    tp = engine_config.tensor_parallel.tp_size
    if tp != meta["tp_size"]:
        raise ValueError(f"checkpoint was serialized at tp={meta['tp_size']}, engine asks for tp={tp}")
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
            torch.device("cpu")
    group, rank = None, 0
    if tp > 1:
        from ... import comm as dist
        world, me = dist.get_world_size(), dist.get_rank()
        for s in range(0, world, tp):
            g = dist.new_group(list(range(s, s + tp)))
            if s <= me < s + tp:
                group = g
        rank = dist.get_rank(group)
    model = DSInferenceModel(spec, group, tp, rank, to_dtype(meta["dtype"]), device)
    sd = load_file(os.path.join(path, f"params_rank_{rank}.safetensors"), device=str(device))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    if unexpected or any(not k.startswith(("rope_", "alibi")) for k in missing):
        raise ValueError(f"serialized weights do not match the spec: missing {missing[:4]}, unexpected "
                         f"{unexpected[:4]}")
    q = engine_config.quantization.quantization_mode
    if q in ("int8", "int4"):
        model.quantize_weights(8 if q == "int8" else 4)
    else:
        _apply_decode_layout(model, engine_config.decode_layout, tp, device)
    return InferenceEngineV2(model, engine_config)
