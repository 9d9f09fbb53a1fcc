from .elasticity import compute_elastic_config, elasticity_enabled, ensure_immutable_elastic_config  # noqa: F401
from .config import ElasticityConfig, ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize  # noqa
