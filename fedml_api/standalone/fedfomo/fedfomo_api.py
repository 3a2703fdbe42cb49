"""Compat shim: reference import path ``fedml_api/standalone/fedfomo/fedfomo_api.py`` (class ``FEDFOMOAPI``,
``fedfomo_api.py:13``)."""
from neuroimagedisttraining_amd.algorithms.personalized import FedFomoAPI  # noqa: F401

FEDFOMOAPI = FedFomoAPI
