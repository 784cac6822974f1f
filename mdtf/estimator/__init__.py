"""Estimator-style front ends: ``Estimator``/``DistributeEstimator``, ``DistributeExperiment``, ``RunConfig``."""
from .run_config import RunConfig  # noqa: F401
from .estimator import Estimator, EstimatorSpec, ModeKeys, metrics  # noqa: F401
from .distribute import DistributeEstimator, DistributeExperiment, current_input  # noqa: F401
