"""Elastic batch sizing (reference elasticity/)."""
from .elasticity import (ElasticityConfigError, ElasticityError, ElasticityIncompatibleWorldSize,  # noqa: F401
                         compute_elastic_config, elasticity_enabled)
