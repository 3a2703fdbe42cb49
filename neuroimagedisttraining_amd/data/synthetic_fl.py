"""Synthetic ABCD-shape federated cohorts for the headline configs (BASELINE.json configs 2-3).

Every client's volumes are generated from a client-specific seed, so a client's data is identical no matter
how many ranks the clients are sharded over (1/2/4/8 GPUs see the same cohort).  Labels are non-IID across
clients: each client draws its positive-class probability from a Dirichlet(alpha) prior over the 2 classes
(the ``dir`` partitioner's class prior, ``cifar10/data_loader.py:118-149``), and its "site" (scanner effect)
is ``client % 21`` like the reference's 21 site-clients (``ABCD/data_loader.py:176``).

The store is built directly in the layout the HIP kernels consume: uint8 polyphase volumes
``[N_local, 61, 73, 61, 8]`` plus the per-sample patch moments used by the fused conv1/BN1 kernel.
"""
from __future__ import annotations

import numpy as np
import torch

from .volumes import make_synthetic_abcd
from ..engine.executor import ClientSplit


def client_labels(n_clients, n_per_client, alpha=0.3, seed=0):
    rs = np.random.RandomState(seed + 7)
    p = rs.dirichlet([alpha, alpha], size=n_clients)[:, 1]
    labs = []
    for c in range(n_clients):
        r = np.random.RandomState(seed * 1009 + c)
        labs.append((r.rand(n_per_client) < p[c]).astype(np.float32))
    return labs


def skewed_sizes(n_clients, per_client, alpha, seed=0, minimum=2):
    """Per-client sizes with Dirichlet(alpha) quotas and the same total as ``n_clients * per_client`` (unequal
    sites, like the reference's 270-807-subject ABCD site clients).  ``alpha <= 0``: equal sizes."""
    if alpha <= 0:
        return [per_client] * n_clients
    q = np.random.RandomState(seed + 31).dirichlet([alpha] * n_clients)
    tot = n_clients * per_client
    s = np.maximum(minimum, np.floor(q * (tot - minimum * n_clients)).astype(np.int64) + minimum)
    s[np.argmax(s)] += tot - int(s.sum())
    return [int(x) for x in s]


def build_fl_volumes(local_clients, n_clients, n_train, n_test, device, seed=0, alpha=0.3, shape=(121, 145, 121),
                     label_signal=0.35):
    """Generate the local clients' volumes.  ``n_train`` / ``n_test``: per-client ints or lists (unequal clients).
    Returns (vol_u8 [N_local, D,H,W], labels [N_local] f32 (device), splits dict client -> ClientSplit of indices
    into the local store).  ``label_signal`` sets how separable the classes are (0.35: easy; ~0.05: the fp32
    reference reaches only ~0.8 accuracy, so numerics regressions show in the accuracy trajectory)."""
    ntr = list(n_train) if hasattr(n_train, "__len__") else [n_train] * n_clients
    nte = list(n_test) if hasattr(n_test, "__len__") else [n_test] * n_clients
    maxper = max(a + b for a, b in zip(ntr, nte))
    labs = client_labels(n_clients, maxper, alpha, seed)
    vols, ys, splits = [], [], {}
    off = 0
    for c in local_clients:
        per = ntr[c] + nte[c]
        st = make_synthetic_abcd(per, shape=shape, n_sites=21, seed=seed * 100003 + c, device=device,
                                 labels=labs[c][:per], site=np.full(per, c % 21, dtype=np.float32),
                                 label_signal=label_signal)
        vols.append(st.volumes)
        ys.append(st.labels)
        splits[c] = ClientSplit(train=np.arange(off, off + ntr[c]), test=np.arange(off + ntr[c], off + per))
        off += per
    vol = torch.cat(vols, 0) if vols else torch.zeros((0,) + tuple(shape), dtype=torch.uint8, device=device)
    y = torch.cat(ys, 0) if ys else torch.zeros(0, device=device)
    return vol, y.float(), splits


def to_hip_store(vol_u8, chunk=512):
    """uint8 volumes -> polyphase store + per-sample conv1 patch moments (HIP kernels)."""
    from .. import ops
    m = ops.ext()
    N = vol_u8.shape[0]
    dev = vol_u8.device
    x8 = torch.empty((N, 61, 73, 61, 8), dtype=torch.uint8, device=dev)
    mom = torch.empty((N, 125 + 125 * 125), dtype=torch.float64, device=dev)
    st = ops.stream()
    for s in range(0, N, chunk):
        e = min(N, s + chunk)
        src = vol_u8[s:e].contiguous()
        m.polyphase(src.data_ptr(), x8[s].data_ptr(), e - s, st)
        m.conv1_sample_moments(x8[s].data_ptr(), e - s, mom[s].data_ptr(), st)
    return x8, mom


def conv1_moments_reference(vol_u8):
    """fp64 reference of the per-sample patch moments (sum p, sum p p^T over all 59x71x59 positions)."""
    N = vol_u8.shape[0]
    out = torch.zeros((N, 125 + 125 * 125), dtype=torch.float64)
    for n in range(N):
        v = vol_u8[n].to(torch.float64)
        p = v.unfold(0, 5, 2).unfold(1, 5, 2).unfold(2, 5, 2)  # [59,71,59,5,5,5]
        p = p.reshape(-1, 125)
        out[n, :125] = p.sum(0)
        out[n, 125:] = (p.t() @ p).reshape(-1)
    return out
