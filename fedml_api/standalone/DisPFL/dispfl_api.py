"""Compat shim: reference import path ``fedml_api/standalone/DisPFL/dispfl_api.py`` (class ``dispflAPI``,
``dispfl_api.py:17``)."""
from neuroimagedisttraining_amd.algorithms.personalized import DisPFLAPI  # noqa: F401

dispflAPI = DisPFLAPI
