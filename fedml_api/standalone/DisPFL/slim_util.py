"""Compat shim: reference import path ``fedml_api/standalone/DisPFL/slim_util.py``."""
from neuroimagedisttraining_amd.algorithms.sparse import hamming_distance, model_difference  # noqa: F401
