"""Compat shim: reference import path ``fedml_api/model/cv/cnn_meta.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import Meta_net, cnn_cifar10_meta  # noqa: F401
