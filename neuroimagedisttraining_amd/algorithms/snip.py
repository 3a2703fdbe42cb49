"""SNIP saliency and global top-k mask selection (reference ``sailentgrads/snip.py``).

The reference patches every Conv3d/Linear to compute ``F.conv3d(x, w*mask)`` and reads
``|dL/dmask|`` at ``mask=1``.  Since ``dL/dmask = w * dL/dw_eff`` and ``w_eff = w`` at mask 1,
this module computes the identical quantity as ``|w ⊙ ∂L/∂w|`` from one ordinary backward pass on a
throwaway copy of the model (train mode, as in the reference) — no monkey-patching.

Mask rule (``snip.py:80-116``): concatenate all scores, divide by their sum, ``k = int(N*keep)``,
threshold = k-th largest, keep ``score >= threshold`` (ties kept, Q7).  Non-conv/linear params
(biases, BN affine) get all-ones masks.  The device path uses the HIP radix-select kernel in
:mod:`neuroimagedisttraining_amd.ops.topk` when available (bit-identical threshold).
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

MASKABLE = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.Linear)


def maskable_weight_names(model):
    return [name + ".weight" for name, m in model.named_modules() if isinstance(m, MASKABLE)]


def snip_scores(model, x, y, loss="bce"):
    """Per-layer ``|w ⊙ ∂L/∂w|`` for one mini-batch; keys are module names (``features.0``)."""
    cp = copy.deepcopy(model)
    cp.train()
    names = [n for n, m in cp.named_modules() if isinstance(m, MASKABLE)]
    mods = dict(cp.named_modules())
    for p in cp.parameters():
        p.requires_grad_(False)
    for n in names:
        mods[n].weight.requires_grad_(True)
    out = cp(x)
    out = out[0] if isinstance(out, (list, tuple)) else out
    if out.dim() == 1 or (out.dim() == 2 and out.shape[1] == 1):
        L = F.binary_cross_entropy_with_logits(out.float(), y.view(-1, 1).float())
    else:
        L = F.cross_entropy(out.float(), y.long())
    L.backward()
    res = {n: (mods[n].weight.detach() * mods[n].weight.grad).abs() for n in names}
    del cp
    return res


def stratified_rng(seed, client, it):
    """RNG of IterSNIP iteration ``it`` of ``client`` under ``--stratified_sampling``: a pure function of
    (run seed, client id, iteration), shared by the eager API and the client-batched runner so both draw the
    same mini-batches (and hence the same global mask) independently of sharding."""
    import numpy as np
    return np.random.RandomState(abs(hash((int(seed), -7, int(client), int(it)))) % (2 ** 31))


def stratified_batch(indices, labels, batch_size, rng):
    """A label-stratified mini-batch of a client's train ``indices`` (``labels[i]`` = label of ``indices[i]``):
    per class round(B * n_class / n) samples with the largest-remainder rule (the counts sum to B), drawn
    without replacement, returned in a random order.  This is the intent of the reference's stratified IterSNIP
    branch (``sailentgrads/client.py:33-43``: StratifiedKFold over the client's samples) at mini-batch size."""
    import numpy as np
    indices = np.asarray(indices)
    y = np.asarray(labels).reshape(-1)
    B = min(int(batch_size), len(indices))
    cls, cnt = np.unique(y, return_counts=True)
    q = B * cnt / cnt.sum()
    take = np.floor(q).astype(int)
    for i in np.argsort(-(q - take), kind="stable")[:B - take.sum()]:
        take[i] += 1
    out = []
    for k, n in zip(cls, take):
        pool = indices[y == k]
        out.append(pool[rng.permutation(len(pool))[:n]])
    b = np.concatenate(out) if out else indices[:0]
    return b[rng.permutation(len(b))]


def mean_scores(score_dicts):
    """Element-wise mean of a list of score dicts (``get_mean_snip_scores`` / ``get_mean_sailency_scores``)."""
    out = {}
    for d in score_dicts:
        for k, v in d.items():
            out[k] = v.clone() if k not in out else out[k].add_(v)
    for k in out:
        out[k].div_(len(score_dicts))
    return out


def global_threshold(all_scores_flat, keep_ratio, use_kernel=True):
    """k-th largest of normalised scores.  Returns ``(threshold, norm_factor)``."""
    norm = all_scores_flat.sum()
    normed = all_scores_flat / norm
    k = int(normed.numel() * keep_ratio)
    k = max(1, k)
    if use_kernel and normed.is_cuda:
        from ..ops import topk as _tk
        thr = _tk.kth_largest(normed, k)
    else:
        thr = torch.topk(normed, k, sorted=True).values[-1]
    return thr, norm


def mask_from_scores(model, scores, keep_ratio, use_kernel=True):
    """Returns ``(keep_masks{module}, final_weight_mask{param name})`` as in the reference."""
    names = list(scores.keys())
    flat = torch.cat([scores[n].flatten() for n in names])
    thr, norm = global_threshold(flat, keep_ratio, use_kernel)
    keep = {n: ((scores[n] / norm) >= thr).float() for n in names}
    final = {}
    wnames = {n + ".weight": n for n in names}
    for pname, p in model.named_parameters():
        final[pname] = keep[wnames[pname]].to(p.device) if pname in wnames else torch.ones_like(p)
    return keep, final


# ------------------------------------------------------------------------------------------------
# The reference's public SNIP functions with their signatures (``sailentgrads/snip.py:9-164``), imported by its
# ``sailentgrads_api.py:16`` and ``client.py:12``.  ``self`` is any object with a ``.model`` (the reference's
# client / trainer).  They delegate to the functions above; the scores are the same |dL/dmask| at mask = 1.

def snip_forward_conv3d(self, x):
    """Forward of a Conv3d whose weight is multiplied by a learnable ``weight_mask`` (``snip.py:9-12``)."""
    return F.conv3d(x, self.weight * self.weight_mask, self.bias, self.stride, self.padding, self.dilation,
                    self.groups)


def snip_forward_linear(self, x):
    """Forward of a Linear whose weight is multiplied by a learnable ``weight_mask`` (``snip.py:15-16``)."""
    return F.linear(x, self.weight * self.weight_mask, self.bias)


def get_snip_scores(self, mini_batch, re_init=False):
    """``snip.py:21-79``: ``mini_batch = (inputs, targets, site_info)`` with channel-less volumes (a channel axis is
    added), BCE-with-logits loss, scores of every Conv3d / Linear as a list of ``(module name, |dL/dmask|)``.
    ``re_init`` re-initialises the scored copy's weights with Xavier-normal first, as the reference does."""
    model = self.model
    device = next(iter(model.parameters())).device
    inputs, targets = mini_batch[0], mini_batch[1]
    inputs = torch.as_tensor(inputs).to(device).unsqueeze(1)
    targets = torch.as_tensor(targets).to(device)
    cp = copy.deepcopy(model)
    if re_init:
        for m in cp.modules():
            if isinstance(m, (nn.Conv3d, nn.Linear)):
                nn.init.xavier_normal_(m.weight)
    scores = snip_scores(cp, inputs.float(), targets.float(), loss="bce")
    del cp
    return [(n, scores[n]) for n in scores]


def get_mask_from_grads(self, grads_abs, keep_ratio, params):
    """``snip.py:84-129``: global top-``keep_ratio`` of the sum-normalised scores (ties kept).  Returns
    ``(keep_masks{module name}, mask_key_layer{module}, final_weight_mask{parameter name})``; biases and norm
    parameters get all-ones masks.  ``params`` is unused, as in the reference."""
    del params
    keep, final = mask_from_scores(self.model, dict(grads_abs), keep_ratio, use_kernel=False)
    mods = dict(self.model.named_modules())
    mask_key_layer = {mods[n]: keep[n] for n in keep if n in mods}
    return keep, mask_key_layer, final


def get_mean_snip_scores(grads_gathered):
    """``snip.py:133-155``: element-wise mean of a list of score dicts (or lists of ``(name, score)`` pairs)."""
    return mean_scores([dict(g) for g in grads_gathered])


def get_mean_sailency_scores(final_sailency_list):
    """``snip.py:158-179`` (IterSNIP): element-wise mean of a list of saliency dicts."""
    return mean_scores([dict(g) for g in final_sailency_list])
