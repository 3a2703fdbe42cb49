"""Compat shim: reference import path ``fedml_api/standalone/sailentgrads/set_client.py``."""
from neuroimagedisttraining_amd.algorithms.common import client_sampling  # noqa: F401
