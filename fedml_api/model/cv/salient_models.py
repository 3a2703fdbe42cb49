"""Compat shim: reference import path ``fedml_api/model/cv/salient_models.py`` -> ``neuroimagedisttraining_amd.models``."""
from neuroimagedisttraining_amd.models.alexnet3d import (  # noqa: F401
    AlexNet3D_Deeper_Dropout, AlexNet3D_Dropout, AlexNet3D_Dropout_Regression)
from neuroimagedisttraining_amd.models.resnet3d import BasicBlock, Bottleneck, ResNet_l3, conv3x3  # noqa: F401
