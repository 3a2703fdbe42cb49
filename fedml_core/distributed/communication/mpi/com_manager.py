"""Compat shim: reference import path ``fedml_core/distributed/communication/mpi/com_manager.py`` ->
``neuroimagedisttraining_amd.comm.mpi_threads`` (send/receive threads over an mpi4py-like ``comm``)."""
from neuroimagedisttraining_amd.comm.mpi_threads import MpiCommunicationManager, TorchP2PComm  # noqa: F401
