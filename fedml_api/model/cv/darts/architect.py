"""Compat shim: reference ``fedml_api/model/cv/darts/architect.py``."""
from neuroimagedisttraining_amd.nas.architect import Architect  # noqa: F401
