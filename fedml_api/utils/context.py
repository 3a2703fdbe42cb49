"""Compat shim: reference import path ``fedml_api/utils/context.py`` -> ``neuroimagedisttraining_amd.utils.context``."""
from neuroimagedisttraining_amd.utils.context import get_lock, raise_MPI_error, raise_error_without_process  # noqa: F401
