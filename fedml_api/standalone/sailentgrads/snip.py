"""Compat shim: reference import path ``fedml_api/standalone/sailentgrads/snip.py``."""
from neuroimagedisttraining_amd.algorithms.snip import global_threshold, mask_from_scores, mean_scores, snip_scores  # noqa: F401
