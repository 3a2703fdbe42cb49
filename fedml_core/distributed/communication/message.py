"""Compat shim: reference import path ``fedml_core/distributed/communication/message.py`` -> ``neuroimagedisttraining_amd.comm.message``."""
from neuroimagedisttraining_amd.comm.message import Message  # noqa: F401
