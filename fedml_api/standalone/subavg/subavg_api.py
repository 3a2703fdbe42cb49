"""Compat shim: reference import path ``fedml_api/standalone/subavg/subavg_api.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import SubAvgAPI  # noqa: F401
