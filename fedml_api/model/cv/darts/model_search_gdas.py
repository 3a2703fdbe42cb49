"""Compat shim: reference ``fedml_api/model/cv/darts/model_search_gdas.py``."""
from neuroimagedisttraining_amd.nas.search import Cell, MixedOp, Network_GumbelSoftmax  # noqa: F401
