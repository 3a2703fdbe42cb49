"""Compat shim: reference ``fedml_api/model/cv/darts/operations.py``."""
from neuroimagedisttraining_amd.nas.ops import *  # noqa: F401,F403
from neuroimagedisttraining_amd.nas.ops import OPS, PRIMITIVES  # noqa: F401
