"""Compat shim: reference import path ``fedml_api/model/cv/vgg.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import VGG, make_layers, vgg11, vgg16  # noqa: F401
