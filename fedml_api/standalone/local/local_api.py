"""Compat shim: reference import path ``fedml_api/standalone/local/local_api.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import LocalAPI  # noqa: F401
