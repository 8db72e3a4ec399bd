"""Registry of inference-v2 compute modules (reference inference/v2/modules/module_registry.py :13-60).

Every interface (attention, linear, MoE, pre/post norm, embedding, unembed) owns a registry mapping an
implementation name to a class. ``instantiate_config(ConfigBundle)`` checks ``supports_config`` and builds the
module; the heuristics in :mod:`.heuristics` choose the name from the layer config and the engine config, so a new
kernel is added by registering a class, never by editing the model.
"""
from dataclasses import dataclass, field
from typing import Any, Dict


@dataclass
class ConfigBundle:
    name: str
    config: Any
    implementation_config: Dict[str, Any] = field(default_factory=dict)


class DSModuleBase:
    """A stateless compute module: weights are passed to ``forward``; ``transform_param`` converts a checkpoint
    tensor to the layout / precision the implementation consumes (done once at load)."""

    def __init__(self, config, implementation_config=None):
        self._config = config
        self._implementation_config = dict(implementation_config or {})

    @staticmethod
    def name() -> str:
        raise NotImplementedError

    @staticmethod
    def supports_config(config) -> bool:
        return True

    def transform_param(self, param):
        return param

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)


class DSModuleRegistryBase:
    registry: Dict[str, type] = {}

    @staticmethod
    def associated_class():
        return DSModuleBase

    @classmethod
    def register_module(cls, child_class):
        if not issubclass(child_class, cls.associated_class()):
            raise TypeError(f"Can only register subclasses of {cls.associated_class().__name__}, "
                            f"{child_class.__name__} is not one")
        cls.registry[child_class.name()] = child_class
        return child_class

    @classmethod
    def instantiate_config(cls, bundle: ConfigBundle):
        if bundle.name not in cls.registry:
            raise KeyError(f"Unknown DSModule: {bundle.name}, registry={sorted(cls.registry)}")
        impl = cls.registry[bundle.name]
        if not impl.supports_config(bundle.config):
            raise ValueError(f"Config {bundle.config} is not supported by {impl.__name__}")
        return impl(bundle.config, bundle.implementation_config)

    @classmethod
    def supporting(cls, config):
        """Names of the registered implementations that accept ``config`` (registration order)."""
        return [n for n, impl in cls.registry.items() if impl.supports_config(config)]
