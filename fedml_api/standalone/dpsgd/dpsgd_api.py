"""Compat shim: reference import path ``fedml_api/standalone/dpsgd/dpsgd_api.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import DPSGDAPI  # noqa: F401
