"""Compat shim: reference import path ``fedml_api/model/cv/resnet.py`` -> ``neuroimagedisttraining_amd.models.zoo2d``."""
from neuroimagedisttraining_amd.models.zoo2d import (  # noqa: F401
    BasicBlock, ResNet, customized_resnet18, original_resnet18, tiny_ResNet, tiny_resnet18)
