"""Compat shim: reference import path ``fedml_api/model/cv/lenet5.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import LeNet5, LeNet5_cifar  # noqa: F401
