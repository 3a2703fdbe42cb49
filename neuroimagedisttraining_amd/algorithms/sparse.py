"""Sparse-mask utilities shared by DisPFL, SubAvg and SalientGrads (reference
``DisPFL/my_model_trainer.py:31-189``, ``DisPFL/client.py:71-99``, ``DisPFL/slim_util.py:7-19``,
``subavg/prune_func.py:9-87``).

All mask math runs on the masks' device (GPU on MI355X) — the reference sorts on CPU per layer and moves
masks host<->device every step.
"""
from __future__ import annotations

import copy
import math

import numpy as np
import torch


def erk_sparsities(params, dense_ratio, tabu=(), erk_power_scale=1.0, distribution="ERK"):
    """Per-layer sparsity so the total density equals ``dense_ratio`` (ERK: density ~ sum(shape)/prod(shape),
    layers whose probability would exceed 1 become dense)."""
    if distribution == "uniform":
        return {n: (0.0 if n in tabu else 1.0 - dense_ratio) for n in params}
    dense_layers = set(tabu)
    while True:
        divisor = rhs = 0.0
        raw = {}
        for n, p in params.items():
            n_param = float(np.prod(p.shape))
            if n in dense_layers:
                rhs -= n_param * (1 - dense_ratio)
            else:
                rhs += n_param * dense_ratio
                raw[n] = (float(np.sum(p.shape)) / n_param) ** erk_power_scale
                divisor += raw[n] * n_param
        eps = rhs / divisor if divisor > 0 else 0.0
        mx = max(raw.values()) if raw else 0.0
        if raw and mx * eps > 1:
            for n, r in raw.items():
                if r == mx:
                    dense_layers.add(n)
            continue
        return {n: (0.0 if n in dense_layers else 1.0 - eps * raw[n]) for n in params}


def init_masks(params, sparsities, generator=None):
    """Random masks with ``int((1 - s) * numel)`` ones per layer."""
    masks = {}
    for n, p in params.items():
        m = torch.zeros(p.numel(), device=p.device)
        k = int((1 - sparsities[n]) * p.numel())
        if k > 0:
            m[torch.randperm(p.numel(), generator=generator)[:k].to(p.device)] = 1
        masks[n] = m.view_as(p)
    return masks


def cosine_annealing(alpha, round_idx, total_rounds):
    return alpha / 2 * (1 + np.cos(round_idx * np.pi / total_rounds))


def fire_mask(masks, weights, round_idx, anneal_factor, comm_round):
    """Drop the ``ceil(drop_ratio * nnz)`` smallest-|w| active weights per layer (cosine-annealed drop ratio).

    As in ``DisPFL/client.py:71-82``: ``num_non_zeros`` is a float32 tensor, so the product with the drop ratio is
    float32; the sort is stable (ties go to the lowest index, like the device kernel)."""
    drop_ratio = cosine_annealing(anneal_factor, round_idx, comm_round)
    new, num_remove = {}, {}
    for n, m in masks.items():
        nnz = m.float().sum()
        k = int(math.ceil(float(torch.tensor(drop_ratio, dtype=torch.float32) * nnz)))
        num_remove[n] = k
        w = weights[n].to(m.device)
        score = torch.where(m > 0, w.abs(), torch.full_like(w, 1e5))
        out = m.clone().view(-1)
        if k > 0:
            out[torch.sort(score.view(-1), stable=True).indices[:k]] = 0
        new[n] = out.view_as(m)
    return new, num_remove


def regrow_mask(masks, num_remove, gradient=None, generator=None):
    """Re-activate ``num_remove`` inactive weights per layer: top-|g| (gradient regrowth, stable descending sort) or
    uniformly at random (``DisPFL/client.py:86-99``)."""
    new = {}
    for n, m in masks.items():
        out = m.clone().view(-1)
        k = num_remove.get(n, 0)
        if k > 0:
            if gradient is not None:
                g = gradient[n].to(m.device).abs().view(-1)
                score = torch.where(out == 0, g, torch.full_like(g, -1e5))
                out[torch.sort(score, descending=True, stable=True).indices[:k]] = 1
            else:
                inactive = (out == 0).float()
                k = min(k, int(inactive.sum()))
                if k > 0:
                    out[torch.multinomial(inactive, k, replacement=False, generator=generator)] = 1
        new[n] = out.view_as(m)
    return new


def hamming_distance(m1, m2):
    """(differing entries, total entries) over all layers."""
    diff = tot = 0
    for n in m1:
        diff += int((m1[n].bool() != m2[n].to(m1[n].device).bool()).sum())
        tot += m1[n].numel()
    return diff, tot


def model_difference(a, b):
    return sum(float(torch.sum((a[n] - b[n]) ** 2)) for n in a)


# -------------------------------------------------------------------------------------- SubAvg (prune_func)
def fake_prune(each_prune_ratio, param_dict, mask):
    """New mask zeroing weights below the ``each_prune_ratio`` percentile of alive |w| per weight layer
    (``subavg/prune_func.py:9-30``: numpy.percentile on the float32 alive values, float32 interpolation)."""
    new = dict(mask)
    for n, t in param_dict.items():
        if "weight" in n and "bn" not in n and n in mask:
            tt = t.detach().float().cpu().numpy()
            mm = mask[n].detach().float().cpu().numpy()
            alive = tt[np.nonzero(tt * mm)]
            if alive.size == 0:
                continue
            thr = np.percentile(np.abs(alive), each_prune_ratio * 100)
            new[n] = torch.from_numpy(np.where(np.abs(tt) < thr, 0, mm).astype(np.float32)).to(mask[n].device)
    return new


def real_prune(param_dict, mask):
    return {n: (t * mask[n].to(t.device) if n in mask else t.clone()) for n, t in param_dict.items()}


def dist_masks(m1, m2):
    """Mean over layers of the per-layer normalised Hamming distance (scipy ``distance.hamming``)."""
    ds = [float((m1[n].reshape(-1).bool() != m2[n].reshape(-1).to(m1[n].device).bool()).float().mean()) for n in m1]
    return float(np.mean(ds)) if ds else 0.0


def print_pruning(param_dict):
    nz = tot = 0
    for t in param_dict.values():
        nz += int(torch.count_nonzero(t))
        tot += t.numel()
    return nz / max(1, tot), nz


def masked_average(w_server, w_locals):
    """SubAvg aggregation: each coordinate averaged over the clients whose mask keeps it (1/count), keeping
    the server value where no client does (``subavg_api.py:123-139``)."""
    masks = [m for m, _ in w_locals]
    ws = [w for _, w in w_locals]
    out = dict(w_server)
    for n in w_server:
        if n not in masks[0]:
            continue
        count = sum(m[n].to(ws[0][n].device).float() for m in masks)
        avg = sum(w[n].float() for w in ws) / count
        ok = torch.isfinite(avg)
        t = w_server[n].clone().float()
        t[ok] = avg[ok]
        out[n] = t.to(w_server[n].dtype)
    return out


def weight_mask_names(model):
    from .snip import maskable_weight_names
    return maskable_weight_names(model)


def copy_masks(m):
    return {k: v.clone() for k, v in m.items()}


deepcopy = copy.deepcopy
