"""Compat shim: reference import path ``fedml_api/model/cv/resnet_ip.py`` -> ``neuroimagedisttraining_amd.models.norm_resnets``."""
from neuroimagedisttraining_amd.models.norm_resnets import ResNet_ip, resnet29_ip, resnet56_ip, resnet110_ip  # noqa: F401
