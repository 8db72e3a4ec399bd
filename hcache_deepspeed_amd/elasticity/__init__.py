from .elasticity import (ElasticityConfig, ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize,
                         compute_elastic_config, elasticity_enabled, ensure_immutable_elastic_config)
from .elastic_agent import DSElasticAgent

__all__ = ["compute_elastic_config", "elasticity_enabled", "ensure_immutable_elastic_config", "ElasticityConfig",
           "ElasticityError", "ElasticityConfigError", "ElasticityIncompatibleWorldSize", "DSElasticAgent"]
