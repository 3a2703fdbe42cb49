"""Client-batched AlexNet3D_Dropout: one forward/backward trains C clients with C weight sets.

Layout ("folded groups"): the C lockstep clients of a step are folded into the channel axis —
activations are ``[B, C*ch, D, H, W]`` so that

* every Conv3d is a grouped convolution with ``groups=C`` (weights ``[C*Cout, Cin, k, k, k]``),
* BatchNorm3d over ``C*ch`` channels is exactly per-(client, channel) batch statistics,
* ReLU / MaxPool3d are layout-agnostic,
* the classifier is a batched matmul over the client axis.

Two backends share this module:

``"torch"`` — PyTorch-ROCm ops (MIOpen grouped conv3d); used as the oracle and as fallback.
``"hip"``   — the hand-written CDNA4 kernels of :mod:`neuroimagedisttraining_amd.ops`
              (fused conv1+BN+ReLU+pool, MFMA implicit-GEMM conv2..5, fused BN/ReLU/pool,
              fused backward).  Selected per layer; see ``ops.available()``.

Reference model: ``fedml_api/model/cv/salient_models.py:142-191`` (keys identical).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..models.alexnet3d import AlexNet3D_Dropout
from .flat import ParamLayout

CONV_IDX = (0, 4, 8, 11, 14)
BN_IDX = (1, 5, 9, 12, 15)
POOL_AFTER = {0: True, 4: True, 8: False, 11: False, 14: True}
CONV_CFG = {0: (5, 2, 0), 4: (3, 1, 0), 8: (3, 1, 1), 11: (3, 1, 1), 14: (3, 1, 1)}  # k, stride, pad
BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def template_model(num_classes=1, in_shape=None):
    return AlexNet3D_Dropout(num_classes=num_classes, in_shape=in_shape)


def layouts(model):
    params = ParamLayout.from_tensors(list(model.named_parameters()))
    buffers = ParamLayout.from_tensors(list(model.named_buffers()))
    return params, buffers


class BatchedAlexNet3D:
    """Functional client-batched forward over ``[C, P]`` parameter and ``[C, Q]`` buffer rows."""

    def __init__(self, num_classes=1, in_shape=None, dropout=0.5):
        self.template = template_model(num_classes, in_shape)
        self.players, self.blayers = layouts(self.template)
        self.num_classes = num_classes
        self.dropout = dropout

    # ---------------------------------------------------------------------------------
    def forward(self, theta, bufs, x, training, compute_dtype=torch.bfloat16, update_stats=True):
        """``theta`` [C,P] fp32 (may require grad); ``bufs`` [C,Q] fp32 (updated in place when
        ``training and update_stats``); ``x`` [B, C, D, H, W] (B-major so the channel fold is
        free).  Returns logits ``[C, B, num_classes]`` fp32."""
        C = theta.shape[0]
        B = x.shape[0]
        pv = self.players.views(theta)
        bv = self.blayers.views(bufs)
        h = x.to(compute_dtype)
        for ci, bi in zip(CONV_IDX, BN_IDX):
            k, s, p = CONV_CFG[ci]
            w = pv["features.%d.weight" % ci]
            cout, cin = w.shape[1], w.shape[2]
            w = w.reshape(C * cout, cin, k, k, k).to(compute_dtype)
            b = pv["features.%d.bias" % ci].reshape(C * cout).to(compute_dtype)
            h = F.conv3d(h, w, b, stride=s, padding=p, groups=C)
            rm = bv["features.%d.running_mean" % bi].reshape(C * cout)
            rv = bv["features.%d.running_var" % bi].reshape(C * cout)
            gamma = pv["features.%d.weight" % bi].reshape(C * cout)
            beta = pv["features.%d.bias" % bi].reshape(C * cout)
            if training and update_stats:
                # F.batch_norm updates running stats in place on the (contiguous) views
                rm_c, rv_c = rm.clone(), rv.clone()
                h = F.batch_norm(h, rm_c, rv_c, gamma.to(h.dtype), beta.to(h.dtype), True, BN_MOMENTUM, BN_EPS)
                with torch.no_grad():
                    bv["features.%d.running_mean" % bi].copy_(rm_c.view(C, cout))
                    bv["features.%d.running_var" % bi].copy_(rv_c.view(C, cout))
                    bv["features.%d.num_batches_tracked" % bi].add_(1)
            else:
                h = F.batch_norm(h, rm, rv, gamma.to(h.dtype), beta.to(h.dtype), False, 0.0, BN_EPS)
            h = F.relu(h)
            if POOL_AFTER[ci]:
                h = F.max_pool3d(h, 3, 3)
        feat = h.reshape(B, C, -1).transpose(0, 1).float()          # [C, B, 256]
        if training and self.dropout > 0:
            feat = F.dropout(feat, self.dropout, True)
        w1 = pv["classifier.1.weight"]                                # [C, 64, 256]
        z = torch.baddbmm(pv["classifier.1.bias"].unsqueeze(1), feat, w1.transpose(1, 2))
        z = F.relu(z)
        if training and self.dropout > 0:
            z = F.dropout(z, self.dropout, True)
        w2 = pv["classifier.4.weight"]
        return torch.baddbmm(pv["classifier.4.bias"].unsqueeze(1), z, w2.transpose(1, 2))

    # ---------------------------------------------------------------------------------
    def state_to_rows(self, sd, device):
        return (self.players.flatten_state(sd, device), self.blayers.flatten_state(sd, device))

    def rows_to_state(self, prow, brow):
        out = dict(self.players.unflatten(prow))
        out.update(self.blayers.unflatten(brow))
        return {k: out[k] for k in self.template.state_dict().keys()}
