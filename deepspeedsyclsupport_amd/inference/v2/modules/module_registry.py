"""Per-interface registries of module implementations (reference `inference/v2/modules/module_registry.py`)."""
from abc import ABC, abstractstaticmethod
from typing import Any, Dict, Type

from ....runtime.config_utils import DeepSpeedConfigModel
from .ds_module import DSModuleBase


class ConfigBundle(DeepSpeedConfigModel):
    """Which implementation (`name`), its interface config, and implementation-specific options."""
    name: str
    config: DeepSpeedConfigModel
    implementation_config: Dict[str, Any] = {}


class DSModuleRegistryBase(ABC):
    """Subclasses set `registry = {}` and name the interface class; implementations register with
    `@Registry.register_module`."""

    @classmethod
    def instantiate_config(cls, config_bundle: ConfigBundle) -> DSModuleBase:
        impl = cls.registry.get(config_bundle.name)
        if impl is None:
            raise KeyError(f"Unknown DSModule: {config_bundle.name}, cls.registry={cls.registry}")
        if not impl.supports_config(config_bundle.config):
            raise ValueError(f"Config {config_bundle.config} is not supported by {impl}")
        return impl(config_bundle.config, config_bundle.implementation_config)

    @abstractstaticmethod
    def associated_class() -> Type[DSModuleBase]:
        raise NotImplementedError("Must associated a DSModule class with its registry.")

    @classmethod
    def register_module(cls, child_class):
        base = cls.associated_class()
        if not issubclass(child_class, base):
            raise TypeError(f"Can only register subclasses of {base}, {child_class} does not inherit from {base}")
        cls.registry[child_class.name()] = child_class
        return child_class
