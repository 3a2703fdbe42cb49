"""Compat shim: reference import path ``fedml_api/utils/logger.py`` -> ``neuroimagedisttraining_amd.utils.logger``."""
from neuroimagedisttraining_amd.utils.logger import logging_config  # noqa: F401
