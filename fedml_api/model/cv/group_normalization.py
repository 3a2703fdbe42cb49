"""Compat shim: reference import path ``fedml_api/model/cv/group_normalization.py`` -> ``neuroimagedisttraining_amd.models.norm_resnets``."""
from neuroimagedisttraining_amd.models.norm_resnets import GroupNorm2d, GroupNorm3d  # noqa: F401
