"""Compat shim: reference ``fedml_api/data_preprocessing/cifar100/datasets.py`` -> ``neuroimagedisttraining_amd.data.datasets``."""
from neuroimagedisttraining_amd.data.datasets import CIFAR100_truncated  # noqa: F401
