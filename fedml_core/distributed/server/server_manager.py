"""Compat shim: reference import path ``fedml_core/distributed/server/server_manager.py`` -> ``neuroimagedisttraining_amd.comm.managers``."""
from neuroimagedisttraining_amd.comm.managers import ServerManager  # noqa: F401
