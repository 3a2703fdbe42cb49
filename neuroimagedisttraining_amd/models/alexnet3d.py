"""3D AlexNet family for structural MRI (reference ``fedml_api/model/cv/salient_models.py:142-297``).

State-dict keys are identical to the reference (``features.{0,4,8,11,14}`` convs,
``features.{1,5,9,12,15}`` BatchNorm3d, ``classifier.{1,4}`` linears) because SalientGrads masks
and SNIP scores are keyed by parameter name.

The reference's weight-init loop targets ``nn.Conv2d`` and therefore never fires for these 3D
layers; only BatchNorm3d gets weight=1/bias=0 (which is also PyTorch's default).  We keep that
behaviour: convs and linears use PyTorch's default kaiming-uniform init.

At input 1x121x145x121 the flattened feature size is 128x1x2x1 = 256.
"""
from __future__ import annotations

import torch
import torch.nn as nn

ABCD_SHAPE = (121, 145, 121)


def _bn_defaults(module):
    for m in module.modules():
        if isinstance(m, nn.BatchNorm3d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)


def _flat_features(features, in_shape):
    was = features.training
    with torch.no_grad():
        n = int(features.eval()(torch.zeros(1, 1, *in_shape)).flatten(1).shape[1])
    features.train(was)
    return n


def _conv_bn_relu(cin, cout, k, stride=1, pad=0):
    return [nn.Conv3d(cin, cout, kernel_size=k, stride=stride, padding=pad),
            nn.BatchNorm3d(cout), nn.ReLU(inplace=True)]


class AlexNet3D_Dropout(nn.Module):
    """Headline model: 5 conv/BN/ReLU blocks, 3 max-pools, dropout MLP head (256 -> 64 -> C)."""

    def __init__(self, num_classes=2, in_shape=None):
        super().__init__()
        layers = []
        layers += _conv_bn_relu(1, 64, 5, stride=2) + [nn.MaxPool3d(3, 3)]          # 0..3
        layers += _conv_bn_relu(64, 128, 3) + [nn.MaxPool3d(3, 3)]                  # 4..7
        layers += _conv_bn_relu(128, 192, 3, pad=1)                                  # 8..10
        layers += _conv_bn_relu(192, 192, 3, pad=1)                                  # 11..13
        layers += _conv_bn_relu(192, 128, 3, pad=1) + [nn.MaxPool3d(3, 3)]          # 14..17
        self.features = nn.Sequential(*layers)
        nfeat = 256 if in_shape is None else _flat_features(self.features, in_shape)
        self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(nfeat, 64), nn.ReLU(inplace=True),
                                        nn.Dropout(), nn.Linear(64, num_classes))
        _bn_defaults(self)

    def forward(self, x):
        x = self.features(x)
        return self.classifier(x.flatten(1))


class AlexNet3D_Deeper_Dropout(nn.Module):
    """Six-conv variant (-> 384 -> 256 -> 256), ``Linear(512, 64)`` head; returns ``[x, x]``
    (``salient_models.py:194-246``)."""

    def __init__(self, num_classes=2):
        super().__init__()
        layers = []
        layers += _conv_bn_relu(1, 64, 5, stride=2) + [nn.MaxPool3d(3, 3)]
        layers += _conv_bn_relu(64, 128, 3) + [nn.MaxPool3d(3, 3)]
        layers += _conv_bn_relu(128, 192, 3, pad=1)
        layers += _conv_bn_relu(192, 384, 3, pad=1)
        layers += _conv_bn_relu(384, 256, 3, pad=1)
        layers += _conv_bn_relu(256, 256, 3, pad=1) + [nn.MaxPool3d(3, 3)]
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(512, 64), nn.ReLU(inplace=True),
                                        nn.Dropout(), nn.Linear(64, num_classes))
        _bn_defaults(self)

    def forward(self, x):
        x = self.classifier(self.features(x).flatten(1))
        return [x, x]


class AlexNet3D_Dropout_Regression(nn.Module):
    """Regression head variant; returns ``[x.squeeze(), features]`` (``salient_models.py:248-297``)."""

    def __init__(self, num_classes=1):
        super().__init__()
        base = AlexNet3D_Dropout(num_classes)
        self.features = base.features
        self.regressor = base.classifier

    def forward(self, x):
        f = self.features(x).flatten(1)
        return [self.regressor(f).squeeze(), f]


def alexnet3d(num_classes=1, in_shape=None, **kw):
    return AlexNet3D_Dropout(num_classes=num_classes, in_shape=in_shape)


def min_alexnet3d_shape():
    """Smallest cubic input that AlexNet3D_Dropout accepts (one voxel after the last pool)."""
    return (69, 69, 69)


def feature_shape(model: nn.Module, in_shape=ABCD_SHAPE):
    """Flattened feature size of ``model.features`` for a single-channel volume."""
    with torch.no_grad():
        return model.features(torch.zeros(1, 1, *in_shape)).flatten(1).shape[1]
