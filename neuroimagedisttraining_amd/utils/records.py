"""End-of-run records: ``record_information`` and ``record_avg_inference_flops`` of the reference APIs.

``record_information`` (``subavg/subavg_api.py:218-221``, ``fedfomo/fedfomo_api.py:326-329``,
``local/local_api.py:196-199``) pickles ``stat_info`` to ``../../results/<dataset>/<identity>`` and crashes when that
directory is missing (quirk Q13).  Here it is written WITHOUT pickle: ``<identity>.json`` holds every scalar / list /
small array, large arrays (final masks, mask-distance matrices of big federations) go to ``<identity>.npz``
(``numpy.load`` with the default ``allow_pickle=False`` reads it back), and the directory is created.

``record_avg_inference_flops`` (``subavg_api.py:223-235``, ``ditto/ditto_api.py:78,153``) averages the sparse-aware
inference FLOPs of every client's model (``w_global`` under the client's personal mask for SubAvg, ``w_global``
alone for Ditto).  The counter's per-layer cost is affine in the layer's non-zero weight count
(``(2 nnz + bias * C_out) * spatial`` for a conv, ``(2 nnz(weight) + nnz(bias)) * batch`` for a linear layer: the
reference's ``multiply_adds=True``, ``main_flops_counter.py:58-80``; ``utils/flops.py``), so the coefficients are measured with ONE forward of the template model and each client's
count is a dot product with its per-layer non-zero counts — no per-client forward pass.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch
import torch.nn as nn

from .flops import INPUT_SHAPES

_BIG = 4096  # arrays with more elements than this go to the .npz sidecar


def _to_jsonable(v, key, arrays):
    if torch.is_tensor(v):
        v = v.detach().cpu().numpy()
    if isinstance(v, np.ndarray):
        if v.size > _BIG:
            arrays[key] = v
            return {"npz": key}
        return v.tolist()
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, dict):
        return {str(k): _to_jsonable(x, "%s.%s" % (key, k), arrays) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_to_jsonable(x, "%s.%d" % (key, i), arrays) for i, x in enumerate(v)]
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    return str(v)


def record_information(stat_info, results_dir, dataset, identity):
    """Persist ``stat_info`` as ``<results_dir>/<dataset>/<identity>.json`` (+ ``.npz`` for large arrays).
    Returns the JSON path."""
    d = os.path.join(results_dir, str(dataset))
    os.makedirs(d, exist_ok=True)
    arrays = {}
    doc = {str(k): _to_jsonable(v, str(k), arrays) for k, v in stat_info.items()}
    base = os.path.join(d, identity)
    if arrays:
        np.savez_compressed(base + ".npz", **arrays)
        doc["_npz"] = os.path.basename(base + ".npz")
    tmp = base + ".json.tmp"
    with open(tmp, "w") as f:
        json.dump(doc, f)
    os.replace(tmp, base + ".json")
    return base + ".json"


def load_information(path):
    """Inverse of :func:`record_information` (arrays from the sidecar come back as numpy arrays)."""
    with open(path) as f:
        doc = json.load(f)
    npz = doc.pop("_npz", None)
    arrays = np.load(os.path.join(os.path.dirname(path), npz)) if npz else {}

    def back(v):
        if isinstance(v, dict) and set(v) == {"npz"}:
            return arrays[v["npz"]]
        if isinstance(v, dict):
            return {k: back(x) for k, x in v.items()}
        if isinstance(v, list):
            return [back(x) for x in v]
        return v
    return {k: back(v) for k, v in doc.items()}


def flop_coefficients(model, dataset="ABCD", input_shape=None):
    """{parameter name: (a, b)} such that the counter's FLOPs = sum over names of a * nnz(parameter) + b
    (:func:`..utils.flops.count_model_param_flops`: conv weight ``(2 * spatial, bias * Cout * spatial)``, linear weight
    ``(2 * batch, 0)`` and its bias, counted by its non-zeros like the reference, ``(batch, 0)``).  One forward of
    ``model`` on a ``(1,) + input`` tensor (the counter's batch of one)."""
    coef = {}
    names = {m: n for n, m in model.named_modules()}

    def conv_hook(m, inp, out):
        spatial = out.numel() // m.out_channels
        bias = m.out_channels if m.bias is not None else 0
        coef[names[m] + ".weight"] = (2.0 * spatial, float(bias * spatial))

    def linear_hook(m, inp, out):
        batch = out.numel() // m.out_features
        coef[names[m] + ".weight"] = (2.0 * batch, 0.0)
        if m.bias is not None:
            coef[names[m] + ".bias"] = (float(batch), 0.0)

    hs = []
    for m in model.modules():
        if isinstance(m, (nn.Conv1d, nn.Conv2d, nn.Conv3d)):
            hs.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, nn.Linear):
            hs.append(m.register_forward_hook(linear_hook))
    shape = input_shape or INPUT_SHAPES.get(dataset, (3, 32, 32))
    dev = next(model.parameters()).device
    was = model.training
    model.eval()
    with torch.no_grad():
        model(torch.zeros((1,) + tuple(shape), device=dev))
    model.train(was)
    for h in hs:
        h.remove()
    return coef


def sparse_inference_flops(coef, layout, rows):
    """Inference FLOPs of each flat parameter row of ``rows`` [K, >= P] (device or host): sum over the counted
    layers of a * nnz + b, with ``layout`` the flat parameter layout (``engine.flat.ParamLayout``)."""
    out = torch.zeros(rows.shape[0], dtype=torch.float64, device=rows.device)
    for i, n in enumerate(layout.names):
        if n in coef:
            a, b = coef[n]
            o, k = layout.offsets[i], layout.numel(i)
            out += a * torch.count_nonzero(rows[:, o:o + k], dim=1).double() + b
    return out
