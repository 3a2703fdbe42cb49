"""Compat shim: reference import path ``fedml_api/data_preprocessing/synthetic/data_loader.py`` -> ``neuroimagedisttraining_amd.data.images``."""
from neuroimagedisttraining_amd.data.images import load_partition_data_synthetic_tabular  # noqa: F401
from neuroimagedisttraining_amd.data.abcd import load_partition_data_abcd_synthetic  # noqa: F401
