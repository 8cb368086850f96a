from .elasticity import compute_elastic_config, elasticity_enabled, ensure_immutable_elastic_config
from .config import ElasticityConfig, ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize
from .elastic_agent import DSElasticAgent, WorkerSpec
