"""Compat shim: reference import path ``fedml_api/data_preprocessing/cifar100/data_loader.py`` -> ``neuroimagedisttraining_amd.data.images``."""
from neuroimagedisttraining_amd.data.images import load_partition_data_cifar100, partition_data  # noqa: F401
