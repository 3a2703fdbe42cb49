"""Compat shim: reference import path ``fedml_core/distributed/communication/base_com_manager.py`` -> ``neuroimagedisttraining_amd.comm.message``."""
from neuroimagedisttraining_amd.comm.message import BaseCommunicationManager  # noqa: F401
