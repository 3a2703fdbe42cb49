"""Compat shim: reference import path ``fedml_api/model/cv/cnn_cifar10.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import cnn_cifar10, cnn_cifar100  # noqa: F401
