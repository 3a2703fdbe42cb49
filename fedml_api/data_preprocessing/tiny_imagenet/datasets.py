"""Compat shim: reference ``fedml_api/data_preprocessing/tiny_imagenet/datasets.py`` -> ``neuroimagedisttraining_amd.data.datasets``."""
from neuroimagedisttraining_amd.data.datasets import tiny, tiny_truncated  # noqa: F401
