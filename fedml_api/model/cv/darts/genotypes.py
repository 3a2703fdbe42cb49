"""Compat shim: reference ``fedml_api/model/cv/darts/genotypes.py``."""
from neuroimagedisttraining_amd.nas.genotypes import *  # noqa: F401,F403
