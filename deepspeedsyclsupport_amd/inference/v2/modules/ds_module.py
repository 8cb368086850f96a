"""Base of the configurable inference v2 building blocks (reference `inference/v2/modules/ds_module.py`): a module
has a name (its registry key), a config class, says which configs it supports, and is built from
(config, implementation_config)."""
from abc import ABC, abstractstaticmethod
from typing import Any, Dict, Type

import torch

from ....runtime.config_utils import DeepSpeedConfigModel


class DSModuleConfig(DeepSpeedConfigModel):
    max_tokens: int


class DSModuleBase(torch.nn.Module, ABC):

    @abstractstaticmethod
    def name() -> str:
        ...

    @abstractstaticmethod
    def config_class() -> Type[DSModuleConfig]:
        ...

    @abstractstaticmethod
    def supports_config(config: DSModuleConfig) -> bool:
        ...

    def __init__(self, config: DSModuleConfig, implementation_config: Dict[str, Any] = {}) -> None:
        super().__init__()
        self._config = config
        self._implementation_config = implementation_config

    @property
    def config(self):
        return self._config
