"""Compat shim: reference import path ``fedml_core/robustness/robust_aggregation.py`` -> ``neuroimagedisttraining_amd.core.robustness``."""
from neuroimagedisttraining_amd.core.robustness import (  # noqa: F401
    RobustAggregator, coordinate_median, is_weight_param, krum, load_model_weight_diff, robust_aggregate,
    trimmed_mean, vectorize_weight)
