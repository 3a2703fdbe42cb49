"""Model zoo (reference ``fedml_api/model/cv``) plus the new LR and 3D ResNet-50 models.

:func:`create_model` mirrors the entry points' ``create_model(args, model_name, class_num)``
(``main_sailentgrads.py:164-178``, ``main_dispfl.py:163-177`` ...).
"""
from __future__ import annotations

from .alexnet3d import (AlexNet3D_Deeper_Dropout, AlexNet3D_Dropout, AlexNet3D_Dropout_Regression, alexnet3d,
                        feature_shape)
from .norm_resnets import (GroupNorm2d, GroupNorm3d, ResNet_ip, ResNetGN, SynchronizedBatchNorm1d,
                           SynchronizedBatchNorm2d, SynchronizedBatchNorm3d, convert_sync_batchnorm, resnet18_gn,
                           resnet29_ip, resnet34_gn, resnet50_gn, resnet56_ip, resnet101_gn, resnet110_ip,
                           resnet152_gn)
from .resnet3d import ResNet3D, ResNet_l3, resnet3d_18, resnet3d_50, resnet_l3
from .zoo2d import (CNN_DropOut, CNN_OriginalFedAvg, LeNet5, LeNet5_cifar, LogisticRegression, Meta_net, ResNet,
                    VGG, cnn_cifar10, cnn_cifar10_meta, cnn_cifar100, customized_resnet18, original_resnet18,
                    tiny_resnet18, vgg11, vgg16)

__all__ = [n for n in dir() if not n.startswith("_")]


def create_model(model_name, dataset="ABCD", class_num=1, in_shape=None, input_dim=None, logger=None):
    """Build a model by the reference CLI name (``--model``)."""
    name = model_name.lower()
    if name in ("3dcnn", "alexnet3d", "alexnet3d_dropout"):
        return AlexNet3D_Dropout(num_classes=class_num, in_shape=in_shape)
    if name in ("3dcnn_deeper", "alexnet3d_deeper"):
        return AlexNet3D_Deeper_Dropout(num_classes=class_num)
    if name in ("3dcnn_regression",):
        return AlexNet3D_Dropout_Regression(num_classes=class_num)
    if name in ("resnet_l3", "3dresnet"):
        return resnet_l3(num_classes=class_num, in_shape=in_shape or (121, 145, 121))
    if name in ("resnet3d_50", "3dresnet50"):
        return resnet3d_50(num_classes=class_num, checkpoint_stages=True)
    if name in ("resnet3d_18", "3dresnet18"):
        return resnet3d_18(num_classes=class_num)
    if name == "resnet18":
        if dataset == "tiny":
            return tiny_resnet18(class_num=class_num)
        return customized_resnet18(class_num=class_num)
    if name == "resnet18_bn":
        return original_resnet18(class_num=class_num)
    if name == "vgg11":
        return vgg11(class_num)
    if name == "vgg16":
        return vgg16(class_num)
    if name == "lenet5":
        return LeNet5(class_num) if dataset in ("mnist", "emnist", "fmnist") else LeNet5_cifar(class_num)
    if name in ("cnn_cifar10", "cnn"):
        return cnn_cifar10(n_cls=class_num)
    if name == "cnn_cifar100":
        return cnn_cifar100(n_cls=class_num)
    if name == "cnn_meta":
        return cnn_cifar10_meta(n_cls=class_num)
    if name in ("lr", "logistic_regression"):
        return LogisticRegression(input_dim, class_num)
    if name in ("resnet20_meta", "resnet_meta"):
        from .meta_resnet import resnet20_meta
        return resnet20_meta(class_num)
    if name == "resnet56_ip":
        return resnet56_ip(class_num)
    if name in ("resnet18_gn", "resnet50_gn"):
        return {"resnet18_gn": resnet18_gn, "resnet50_gn": resnet50_gn}[name](class_num)
    raise ValueError("unknown model %r" % model_name)
