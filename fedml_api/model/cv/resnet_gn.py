"""Compat shim: reference import path ``fedml_api/model/cv/resnet_gn.py`` -> ``neuroimagedisttraining_amd.models.norm_resnets``."""
from neuroimagedisttraining_amd.models.norm_resnets import (  # noqa: F401
    GNBasicBlock as BasicBlock, GNBottleneck as Bottleneck, ResNetGN as ResNet, resnet18_gn as resnet18,
    resnet34_gn as resnet34, resnet50_gn as resnet50, resnet101_gn as resnet101, resnet152_gn as resnet152)
