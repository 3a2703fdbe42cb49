"""Compat shim: reference import path ``fedml_api/standalone/ditto/client.py``."""
from neuroimagedisttraining_amd.algorithms.common import Client  # noqa: F401
