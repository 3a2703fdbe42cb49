"""Compat shim: reference import path ``fedml_api/data_preprocessing/ABCD/data_loader.py`` -> ``neuroimagedisttraining_amd.data.abcd``."""
from neuroimagedisttraining_amd.data.abcd import (  # noqa: F401
    load_partition_data_abcd, load_partition_data_abcd_rescale, load_partition_data_abcd_synthetic)
