"""Compat shim: reference import path ``fedml_api/model/cv/cnn.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import CNN_DropOut, CNN_OriginalFedAvg, cnn_cifar10  # noqa: F401
