"""PyTorch reference implementations (fp32) of the fused HIP ops — the numerics oracle and the CPU path.

Everything here follows the reference model's semantics exactly (``salient_models.py:142-191`` and the
SalientGrads trainer ``sailentgrads/my_model_trainer.py:201-235``): Conv3d -> BatchNorm3d(train) -> ReLU ->
MaxPool3d, dropout MLP head, BCEWithLogits loss averaged over the client's batch.

Layouts shared with the HIP path:
* volumes are stored as uint8 in the polyphase layout ``[N, 61, 73, 61, 8]`` (see ``csrc/kernels/conv1.hip``);
  :func:`unpolyphase` recovers ``[N, 121, 145, 121]``;
* dropout masks come from the same counter hash as ``csrc/kernels/head.hip`` (:func:`dropout_keep`).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

VOL = (121, 145, 121)
PPH = (61, 73, 61)
M64 = (1 << 64) - 1


def polyphase(vol_u8: torch.Tensor) -> torch.Tensor:
    """``[N, 121, 145, 121]`` uint8 -> ``[N, 61, 73, 61, 8]`` (phase r = (d&1)<<2 | (h&1)<<1 | (w&1))."""
    N, D, H, W = vol_u8.shape
    assert (D, H, W) == VOL
    pad = torch.zeros((N, 2 * PPH[0], 2 * PPH[1], 2 * PPH[2]), dtype=vol_u8.dtype, device=vol_u8.device)
    pad[:, :D, :H, :W] = vol_u8
    x = pad.view(N, PPH[0], 2, PPH[1], 2, PPH[2], 2)          # n z rd y rh x rw
    return x.permute(0, 1, 3, 5, 2, 4, 6).reshape(N, PPH[0], PPH[1], PPH[2], 8).contiguous()


def unpolyphase(x8: torch.Tensor) -> torch.Tensor:
    N = x8.shape[0]
    x = x8.view(N, PPH[0], PPH[1], PPH[2], 2, 2, 2).permute(0, 1, 4, 2, 5, 3, 6)
    x = x.reshape(N, 2 * PPH[0], 2 * PPH[1], 2 * PPH[2])
    return x[:, :VOL[0], :VOL[1], :VOL[2]].contiguous()


def _mix(z):
    z = z & M64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def hash4_np(seed, a, b, c):
    """numpy twin of ``hash4`` in head.hip (uint64 wrap-around arithmetic)."""
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    c = np.asarray(c, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = (a << np.uint64(40)) ^ (b << np.uint64(20)) ^ c
        z = np.uint64(seed & M64) ^ (np.uint64(0x9e3779b97f4a7c15) * key)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(32)).astype(np.uint32)


def dropout_keep(seed, G, B, nfeat, keep, layer=0, cids=None):
    """Boolean keep-mask ``[G, B, nfeat]`` identical to the HIP head kernel's (streams keyed by global client id)."""
    if keep >= 1.0:
        return np.ones((G, B, nfeat), dtype=bool)
    s = seed if layer == 0 else (seed ^ 0x5bd1e995)
    cid = np.arange(G) if cids is None else np.asarray(cids)
    g, b, f = np.meshgrid(cid, np.arange(B), np.arange(nfeat), indexing="ij")
    thr = np.uint64(int(keep * 4294967296.0))
    return hash4_np(s, g, b, f).astype(np.uint64) < thr


# ------------------------------------------------------------------------------------------------
# functional AlexNet3D_Dropout over a flat parameter row
CONV_IDX = (0, 4, 8, 11, 14)
BN_IDX = (1, 5, 9, 12, 15)
CONV_CFG = {0: (2, 0), 4: (1, 0), 8: (1, 1), 11: (1, 1), 14: (1, 1)}  # stride, pad
POOL_AFTER = {0: True, 4: True, 8: False, 11: False, 14: True}


def alexnet_forward(p, bufs, x, training, keep=0.5, masks=None, momentum=0.1, eps=1e-5):
    """``p``/``bufs``: dicts name -> tensor (views, modified in place for running stats when training).
    ``x``: ``[B, 1, D, H, W]`` float.  ``masks``: (m1 [B,256], m2 [B,64]) keep masks or None."""
    h = x
    for ci, bi in zip(CONV_IDX, BN_IDX):
        s, pd = CONV_CFG[ci]
        h = F.conv3d(h, p["features.%d.weight" % ci], p["features.%d.bias" % ci], s, pd)
        rm, rv = bufs["features.%d.running_mean" % bi], bufs["features.%d.running_var" % bi]
        if training:
            rm_c, rv_c = rm.detach().to(h.dtype).clone(), rv.detach().to(h.dtype).clone()
            h = F.batch_norm(h, rm_c, rv_c, p["features.%d.weight" % bi], p["features.%d.bias" % bi], True,
                             momentum, eps)
            with torch.no_grad():
                rm.copy_(rm_c)
                rv.copy_(rv_c)
                bufs["features.%d.num_batches_tracked" % bi].add_(1)
        else:
            h = F.batch_norm(h, rm, rv, p["features.%d.weight" % bi], p["features.%d.bias" % bi], False, 0.0, eps)
        h = F.relu(h)
        if POOL_AFTER[ci]:
            h = F.max_pool3d(h, 3, 3)
    f = h.flatten(1)
    if training and masks is not None:
        f = f * masks[0].to(f.dtype) / keep
    z = F.relu(F.linear(f, p["classifier.1.weight"], p["classifier.1.bias"]))
    if training and masks is not None:
        z = z * masks[1].to(z.dtype) / keep
    return F.linear(z, p["classifier.4.weight"], p["classifier.4.bias"])


def train_step_reference(layout, blayout, theta, bufs, vols, labels, B, keep=0.5, seed=0, dtype=torch.float32):
    """Reference local step for G clients (sequential loop, autograd).

    ``theta`` ``[G,P]`` fp32 (not modified), ``bufs`` ``[G,Q]`` (running stats updated in place),
    ``vols`` ``[G*B, 121,145,121]`` uint8, ``labels`` ``[G*B]``.  Returns (grads [G,P], losses [G], logits [G*B]).
    """
    G = theta.shape[0]
    grads = torch.zeros_like(theta)
    losses = torch.zeros(G, dtype=torch.float32, device=theta.device)
    logits = torch.zeros(G * B, dtype=torch.float32, device=theta.device)
    m1 = torch.from_numpy(dropout_keep(seed, G, B, 256, keep, 0)).to(theta.device)
    m2 = torch.from_numpy(dropout_keep(seed, G, B, 64, keep, 1)).to(theta.device)
    for g in range(G):
        row = theta[g].detach().clone().to(dtype).requires_grad_(True)
        pv = {n: row[o:o + t].view(s) for n, o, t, s in zip(layout.names, layout.offsets,
                                                             [layout.numel(i) for i in range(len(layout.names))],
                                                             layout.shapes)}
        bv = blayout.views(bufs[g:g + 1])
        bv = {k: v[0] for k, v in bv.items()}
        x = (vols[g * B:(g + 1) * B].to(dtype) / 255.0).unsqueeze(1)
        y = labels[g * B:(g + 1) * B].to(dtype).view(B, 1)
        out = alexnet_forward(pv, bv, x, True, keep, (m1[g], m2[g]) if keep < 1 else None)
        loss = F.binary_cross_entropy_with_logits(out, y)
        loss.backward()
        grads[g] = row.grad.to(torch.float32)
        losses[g] = loss.detach()
        logits[g * B:(g + 1) * B] = out.detach().view(-1).float()
    return grads, losses, logits


def eval_logits_reference(layout, blayout, theta, bufs, vols, B, dtype=torch.float32):
    """Eval-mode logits for G clients x B samples (client g uses row g)."""
    G = theta.shape[0]
    out = torch.zeros(G * B, dtype=torch.float32, device=theta.device)
    with torch.no_grad():
        for g in range(G):
            row = theta[g].to(dtype)
            pv = {n: row[o:o + layout.numel(i)].view(s)
                  for i, (n, o, s) in enumerate(zip(layout.names, layout.offsets, layout.shapes))}
            bv = {k: v[0] for k, v in blayout.views(bufs[g:g + 1].clone()).items()}
            x = (vols[g * B:(g + 1) * B].to(dtype) / 255.0).unsqueeze(1)
            out[g * B:(g + 1) * B] = alexnet_forward(pv, bv, x, False).view(-1).float()
    return out


def clip_sgd_mask_reference(theta, grad, mask, lr, wd, max_norm=10.0):
    """clip_grad_norm_(10) -> SGD(weight_decay, momentum 0) -> weights *= mask, per row (in place)."""
    for g in range(theta.shape[0]):
        gn = grad[g].norm()
        coef = min(1.0, max_norm / (float(gn) + 1e-6))
        gg = grad[g] * coef
        theta[g] -= lr * (gg + wd * theta[g])
        if mask is not None:
            theta[g] *= mask
    return theta
