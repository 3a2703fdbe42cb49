"""Compat shim: reference import path ``fedml_api/standalone/ditto/ditto_api.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import DittoAPI  # noqa: F401
