"""Compat shim: reference import path ``fedml_core/distributed/client/client_manager.py`` -> ``neuroimagedisttraining_amd.comm.managers``."""
from neuroimagedisttraining_amd.comm.managers import ClientManager  # noqa: F401
