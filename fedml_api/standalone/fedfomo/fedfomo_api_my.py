"""Compat shim: reference import path ``fedml_api/standalone/fedfomo/fedfomo_api_my.py``."""
from neuroimagedisttraining_amd.algorithms.personalized import FedFomoAPI  # noqa: F401
