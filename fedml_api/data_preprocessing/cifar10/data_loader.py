"""Compat shim: reference import path ``fedml_api/data_preprocessing/cifar10/data_loader.py`` -> ``neuroimagedisttraining_amd.data.images``."""
from neuroimagedisttraining_amd.data.images import load_partition_data_cifar10, partition_data  # noqa: F401
