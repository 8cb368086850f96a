"""`init_inference` configuration (reference `inference/config.py:15-300`, same keys and aliases)."""
from typing import Dict, Optional, Union

import torch
from pydantic import Field, field_validator

from ..runtime.config_utils import DeepSpeedConfigModel
from ..runtime.zero.config import DeepSpeedZeroConfig

_DTYPES = {
    "fp16": torch.float16, "float16": torch.float16, "half": torch.float16, "torch.float16": torch.float16,
    "bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "bfloat": torch.bfloat16, "torch.bfloat16": torch.bfloat16,
    "fp32": torch.float32, "float32": torch.float32, "float": torch.float32, "torch.float32": torch.float32,
    "int8": torch.int8, "torch.int8": torch.int8,
}


def to_dtype(d):
    if isinstance(d, torch.dtype):
        return d
    if isinstance(d, str) and d in _DTYPES:
        return _DTYPES[d]
    raise ValueError(f"unsupported inference dtype {d!r}")


class DeepSpeedTPConfig(DeepSpeedConfigModel):
    enabled: bool = True
    tp_size: int = 1
    mpu: object = None
    tp_group: object = None
    tp_grain_size: int = 64


class DeepSpeedMoEConfig(DeepSpeedConfigModel):
    enabled: bool = True
    ep_size: int = 1
    moe_experts: list = Field([1], alias="num_experts")
    type: str = "standard"
    ep_mp_group: object = None
    ep_group: object = Field(None, alias="expert_group")


class BaseQuantConfig(DeepSpeedConfigModel):
    enabled: bool = True
    num_bits: int = 8
    q_type: str = "symmetric"
    q_groups: int = 1


class WeightQuantConfig(BaseQuantConfig):
    enabled: bool = True
    quantized_initialization: Dict = {}
    post_init_quant: Dict = {}
    group_size: int = 64


class ActivationQuantConfig(BaseQuantConfig):
    enabled: bool = True


class QKVQuantConfig(DeepSpeedConfigModel):
    enabled: bool = True


class QuantizationConfig(DeepSpeedConfigModel):
    enabled: bool = True
    activation: ActivationQuantConfig = ActivationQuantConfig()
    weight: WeightQuantConfig = WeightQuantConfig()
    qkv: QKVQuantConfig = QKVQuantConfig()


class InferenceCheckpointConfig(DeepSpeedConfigModel):
    checkpoint_dir: Optional[str] = None
    save_mp_checkpoint_path: Optional[str] = None
    base_dir: Optional[str] = None


class DeepSpeedInferenceConfig(DeepSpeedConfigModel):
    replace_with_kernel_inject: bool = Field(False, alias="kernel_inject")
    dtype: object = torch.float16
    tensor_parallel: DeepSpeedTPConfig = Field(DeepSpeedTPConfig(), alias="tp")
    enable_cuda_graph: bool = False
    # bf16 projection weights for decode (`ops/bf16_gemv.py`): "row_major" = the parameters only; "both" = plus a
    # copy in MFMA operand order for steps of 2 - 16 token rows (twice the weight memory); "shuffled" = operand
    # order only (prefill un-shuffles per GEMM); "auto" = "both" when the copy fits in a quarter of the device memory
    decode_layout: str = "auto"
    use_triton: bool = False
    triton_autotune: bool = False
    zero: DeepSpeedZeroConfig = DeepSpeedZeroConfig()
    triangular_masking: bool = Field(True, alias="tm")
    moe: Union[bool, DeepSpeedMoEConfig] = DeepSpeedMoEConfig()
    quant: QuantizationConfig = QuantizationConfig(enabled=False)
    checkpoint: Union[str, Dict, None] = None
    base_dir: str = ""
    set_empty_params: bool = False
    save_mp_checkpoint_path: Optional[str] = None
    checkpoint_config: InferenceCheckpointConfig = Field(InferenceCheckpointConfig(), alias="ckpt_config")
    return_tuple: bool = True
    training_mp_size: int = 1
    replace_method: str = "auto"
    injection_policy: Optional[Dict] = Field(None, alias="injection_dict")
    injection_policy_tuple: Optional[tuple] = None
    config: Optional[Dict] = Field(None, alias="args")
    max_out_tokens: int = Field(1024, alias="max_tokens")
    min_out_tokens: int = Field(1, alias="min_tokens")
    transposed_mode: bool = False
    # MI355X additions: paged KV cache geometry for the injected decoder
    kv_block_size: int = 64
    max_batch_size: int = 64
    # deprecated aliases (reference keeps them for older scripts)
    mp_size: int = 1
    mpu: object = None
    ep_size: int = 1
    ep_group: object = Field(None, alias="expert_group")
    ep_mp_group: object = Field(None, alias="expert_mp_group")
    moe_experts: list = [1]
    moe_type: str = "standard"

    @field_validator("dtype", mode="before")
    @classmethod
    def _dtype(cls, v):
        return to_dtype(v)

    @field_validator("moe", mode="before")
    @classmethod
    def _moe(cls, v):
        if isinstance(v, bool):
            return DeepSpeedMoEConfig(enabled=v)
        return v

    def model_post_init(self, __ctx):
        # deprecated mp_size -> tensor_parallel.tp_size (reference config.py:277)
        if self.mp_size != 1 and self.tensor_parallel.tp_size == 1:
            self.tensor_parallel.tp_size = self.mp_size
        if self.mpu is not None and self.tensor_parallel.mpu is None:
            self.tensor_parallel.mpu = self.mpu


from enum import Enum  # noqa: E402

from .v2.inference_utils import DtypeEnum  # noqa: E402,F401  (the multi-spelling dtype enum)


class MoETypeEnum(str, Enum):
    residual = "residual"
    standard = "standard"


class QuantTypeEnum(str, Enum):
    asym = "asymmetric"
    sym = "symmetric"

