"""Compat shim: reference import path ``fedml_core/distributed/communication/mpi/com_manager.py`` -> ``neuroimagedisttraining_amd.comm.managers``."""
from neuroimagedisttraining_amd.comm.managers import MpiCommunicationManager  # noqa: F401
