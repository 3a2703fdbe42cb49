"""Compat shim: reference import path ``fedml_api/standalone/DisPFL/dispfl_api.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import DisPFLAPI  # noqa: F401
