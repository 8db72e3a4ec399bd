"""Inference-v2 compute modules: interfaces, registries, MI355X implementations and the selection heuristics
(reference deepspeed/inference/v2/modules)."""
from .configs import (DSEmbeddingsConfig, DSLinearConfig, DSMoEConfig, DSNormConfig, DSSelfAttentionConfig,
                      DSUnembedConfig)
from .heuristics import (instantiate_attention, instantiate_embed, instantiate_linear, instantiate_moe,
                         instantiate_post_norm, instantiate_pre_norm, instantiate_unembed)
from .interfaces import (DSEmbeddingBase, DSEmbeddingRegistry, DSLinearBase, DSLinearRegistry, DSMoEBase,
                         DSMoERegistry, DSPostNormBase, DSPostNormRegistry, DSPreNormBase, DSPreNormRegistry,
                         DSSelfAttentionBase, DSSelfAttentionRegistry, DSUnembedBase, DSUnembedRegistry)
from .module_registry import ConfigBundle, DSModuleBase, DSModuleRegistryBase
