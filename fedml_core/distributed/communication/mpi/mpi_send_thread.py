"""Compat shim: reference ``fedml_core/distributed/communication/mpi/mpi_send_thread.py`` ->
``neuroimagedisttraining_amd.comm.mpi_threads``."""
from neuroimagedisttraining_amd.comm.mpi_threads import MPISendThread  # noqa: F401
