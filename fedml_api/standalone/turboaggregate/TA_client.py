"""Compat shim: reference import path ``fedml_api/standalone/turboaggregate/TA_client.py``."""
from neuroimagedisttraining_amd.algorithms.turboaggregate import TA_Client  # noqa: F401
