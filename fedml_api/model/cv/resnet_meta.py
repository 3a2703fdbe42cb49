"""Compat shim: reference ``fedml_api/model/cv/resnet_meta.py`` (broken upstream) -> working PruningNet."""
from neuroimagedisttraining_amd.models.meta_resnet import CHANNEL_SCALE as channel_scale  # noqa: F401
from neuroimagedisttraining_amd.models.meta_resnet import MetaResNet20 as ResNet20  # noqa: F401
from neuroimagedisttraining_amd.models.meta_resnet import MetaBasicBlock, MetaStem, resnet20_meta  # noqa: F401
