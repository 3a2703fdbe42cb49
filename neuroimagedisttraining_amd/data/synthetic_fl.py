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


def build_fl_volumes(local_clients, n_clients, n_train, n_test, device, seed=0, alpha=0.3, shape=(121, 145, 121)):
    """Generate the local clients' volumes.  Returns (vol_u8 [N_local, D,H,W], labels [N_local] f32 (device),
    splits dict client -> ClientSplit of indices into the local store)."""
    per = n_train + n_test
    labs = client_labels(n_clients, per, alpha, seed)
    vols, ys, splits = [], [], {}
    off = 0
    for c in local_clients:
        st = make_synthetic_abcd(per, shape=shape, n_sites=21, seed=seed * 100003 + c, device=device,
                                 labels=labs[c], site=np.full(per, c % 21, dtype=np.float32))
        vols.append(st.volumes)
        ys.append(st.labels)
        splits[c] = ClientSplit(train=np.arange(off, off + n_train), test=np.arange(off + n_train, off + per))
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
    st = torch.cuda.current_stream().cuda_stream
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
