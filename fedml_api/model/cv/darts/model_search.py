"""Compat shim: reference ``fedml_api/model/cv/darts/model_search.py``."""
from neuroimagedisttraining_amd.nas.search import Cell, MixedOp, ModelForModelSizeMeasure, Network  # noqa: F401
