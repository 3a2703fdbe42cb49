"""Compat shim: reference ``fedml_api/model/cv/darts/utils.py``."""
from neuroimagedisttraining_amd.nas.utils import *  # noqa: F401,F403
