"""Compat shim: reference import path ``fedml_core/distributed/communication/observer.py`` -> ``neuroimagedisttraining_amd.comm.message``."""
from neuroimagedisttraining_amd.comm.message import Observer  # noqa: F401
