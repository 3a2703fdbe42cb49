"""Compat shim: reference ``fedml_api/data_preprocessing/ABCD/datasets.py`` -> ``neuroimagedisttraining_amd.data.datasets``."""
from neuroimagedisttraining_amd.data.datasets import CIFAR10_truncated  # noqa: F401
