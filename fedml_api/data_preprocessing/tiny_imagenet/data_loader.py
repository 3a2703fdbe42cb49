"""Compat shim: reference import path ``fedml_api/data_preprocessing/tiny_imagenet/data_loader.py`` -> ``neuroimagedisttraining_amd.data.images``."""
from neuroimagedisttraining_amd.data.images import load_partition_data_tiny, partition_data  # noqa: F401
