"""Compat shim: reference import path ``fedml_api/standalone/sailentgrads/sailentgrads_api.py``."""
from neuroimagedisttraining_amd.algorithms.salientgrads import SailentGradsAPI  # noqa: F401
