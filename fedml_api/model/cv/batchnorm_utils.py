"""Compat shim: reference import path ``fedml_api/model/cv/batchnorm_utils.py`` -> ``neuroimagedisttraining_amd.models.norm_resnets``."""
from neuroimagedisttraining_amd.models.norm_resnets import (  # noqa: F401
    DataParallelWithCallback, SynchronizedBatchNorm1d, SynchronizedBatchNorm2d, SynchronizedBatchNorm3d,
    convert_sync_batchnorm, patch_replication_callback)
