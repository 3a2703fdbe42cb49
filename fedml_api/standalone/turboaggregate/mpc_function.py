"""Compat shim: reference import path ``fedml_api/standalone/turboaggregate/mpc_function.py``."""
from neuroimagedisttraining_amd.algorithms.turboaggregate import *  # noqa: F401,F403
