"""Compat shim: reference ``fedml_api/model/cv/darts/visualize.py`` -> ``neuroimagedisttraining_amd.nas.visualize``."""
from neuroimagedisttraining_amd.nas.visualize import plot, to_dot  # noqa: F401
