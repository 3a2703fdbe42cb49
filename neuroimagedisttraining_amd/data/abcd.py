"""ABCD federated datasets (reference ``fedml_api/data_preprocessing/ABCD/data_loader.py``).

Returned structures follow the dataset 8-tuple contract:
``[train_num, test_num, train_global, test_global, train_local_num_dict, train_local_dict,
test_local_dict, class_num]`` with the first four ``None`` as in the reference.

Each local "DataLoader" is an :class:`IndexLoader` that yields the reference's
``(x_index, y, site)`` float triples and carries a ``.store`` (:class:`VolumeStore`) and the raw
``.indices`` so device-side trainers / the client-batched engine can gather voxels directly.

* :func:`load_partition_data_abcd` — real HDF5 (``X``,``y``,``site`` keys) when ``h5py`` and the file
  exist (site-as-client, seeded 80/20 split, ``max_clients`` default 21 = quirk Q9); otherwise a
  synthetic cohort of the same shape.
* :func:`load_partition_data_abcd_synthetic` — synthetic ABCD-shape cohort partitioned with any of
  the reference partitioners (``dir``/``hetero``/``homo``/``site``/...) into N clients, each split
  80/20 into train/test like the site split.
* :func:`load_partition_data_abcd_rescale` — merge sites and split into contiguous equal shards
  (``ABCD/data_loader.py:216-315``).
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch

from ..core import partition as P
from .volumes import ABCD_SHAPE, VolumeStore, make_synthetic_abcd, quantize_cohort_volumes

log = logging.getLogger(__name__)


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


class IndexLoader:
    """Minimal DataLoader over subject indices (shuffle per epoch, ``drop_last=False``)."""

    def __init__(self, store: VolumeStore, indices, batch_size, shuffle, seed=None):
        self.store = store
        self.indices = np.asarray(indices, dtype=np.int64)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.dataset = _Len(len(self.indices))
        self._rng = np.random.RandomState(seed) if seed is not None else None
        lab = store.labels.detach().cpu().numpy()
        st = store.site.detach().cpu().numpy()
        self._y = lab[self.indices].astype(np.float32) if len(self.indices) else np.zeros(0, np.float32)
        self._s = st[self.indices].astype(np.float32) if len(self.indices) else np.zeros(0, np.float32)

    def __len__(self):
        n = len(self.indices)
        return (n + self.batch_size - 1) // self.batch_size

    def order(self):
        n = len(self.indices)
        if not self.shuffle:
            return np.arange(n)
        return (self._rng or np.random).permutation(n)

    def __iter__(self):
        o = self.order()
        for s in range(0, len(o), self.batch_size):
            b = o[s:s + self.batch_size]
            yield (torch.from_numpy(self.indices[b].astype(np.float32)),
                   torch.from_numpy(self._y[b]), torch.from_numpy(self._s[b]))


def _assemble(store, train_map, test_map, batch_size, class_num=2, logger=None, seed=None):
    num, trn, tst = {}, {}, {}
    for c in sorted(train_map):
        trn[c] = IndexLoader(store, train_map[c], batch_size, shuffle=True,
                             seed=None if seed is None else seed + 7919 * c)
        tst[c] = IndexLoader(store, test_map[c], batch_size, shuffle=False)
        num[c] = len(train_map[c])
        (logger or log).info("client_idx = %d, local_train_sample_number = %d, local_test_sample_number = %d",
                             c, num[c], len(test_map[c]))
    return [None, None, None, None, num, trn, tst, class_num]


def split_clients_80_20(client_map, test_ratio=0.2, seed=42):
    """Per-client seeded shuffle then 80/20 split (the ABCD per-site rule applied to any map)."""
    train, test = {}, {}
    for c, ix in client_map.items():
        ix = np.asarray(ix, dtype=np.int64).copy()
        np.random.RandomState(seed).shuffle(ix)
        nt = int(len(ix) * test_ratio)
        train[c], test[c] = ix[:len(ix) - nt], ix[len(ix) - nt:]
    return train, test


def load_partition_data_abcd_synthetic(client_number=64, partition_method="dir", partition_alpha=0.3,
                                       batch_size=16, shape=ABCD_SHAPE, n_per_client=180, seed=0,
                                       device="cpu", logger=None, store=None, n_sites=21):
    """Synthetic ABCD-shape federated cohort (headline benchmark data).

    ``n_per_client`` subjects per client (default 180 -> 144 train / 36 test, i.e. the ABCD
    train pool of ≈9.2k subjects spread over 64 clients)."""
    n_total = client_number * n_per_client
    if store is None:
        store = make_synthetic_abcd(n_total, shape, n_sites=n_sites, seed=seed, device=device)
    labels = store.labels.cpu().numpy().astype(np.int64)
    rs = np.random.RandomState(seed)
    if partition_method == "site":
        train, test, _ = P.partition_by_site(store.site.cpu().numpy(), max_clients=client_number)
    else:
        cmap = P.partition_labels(partition_method, labels, client_number, partition_alpha, n_cls=2, rng=rs)
        train, test = split_clients_80_20(cmap)
    return _assemble(store, train, test, batch_size, 2, logger, seed=seed)


def _read_h5(path):
    """``X`` (as uint8, quantised chunk-wise from the stored dtype: :func:`quantize_cohort_volumes`), ``y``, ``site``."""
    import h5py  # optional dependency
    with h5py.File(path, "r") as f:
        y = f["y"][()]
        site = f["site"][()]
        X = quantize_cohort_volumes(f["X"]) if "X" in f else None
    return X, y, site


def _cohort_store(X, y, site, device):
    X = quantize_cohort_volumes(X)  # no-op copy for uint8; refuses non-/255 floats instead of truncating them
    return VolumeStore(torch.from_numpy(X).to(device),
                       torch.from_numpy(np.asarray(y, np.float32)).to(device),
                       torch.from_numpy(np.asarray(site, np.float32)).to(device))


def load_partition_data_abcd(data_dir, partition_method="site", partition_alpha=0.3, client_number=21,
                             batch_size=16, logger=None, max_clients=21, device="cpu", shape=ABCD_SHAPE):
    """Reference entry point.  ``data_dir`` may be an HDF5 file (keys ``X`` volumes — uint8, or the reference's
    float k/255 maps, quantised exactly — ``y``, ``site``) or a directory containing ``alldatain8bitsnormalized.h5``.  Falls back to a synthetic
    cohort (and says so) when ``h5py`` or the file is unavailable."""
    path = data_dir
    if path and os.path.isdir(path):
        nv = os.path.join(path, "alldatain8bitsnormalized.nidtvol")
        path = nv if os.path.exists(nv) else os.path.join(path, "alldatain8bitsnormalized.h5")
    if path and str(path).endswith(".nidtvol"):
        # native NIDTVOL1 cohort (mmap + C++ gather, overlapped H2D when device is a GPU)
        from .volume_file import VolumeFile
        vf = VolumeFile(path)
        store = vf.to_store(device=device)
        train, test, _ = P.partition_by_site(vf.sites, max_clients=max_clients)
        return _assemble(store, train, test, batch_size, 2, logger)
    try:
        X, y, site = _read_h5(path)
    except Exception as e:  # noqa: BLE001 - h5py missing or no file: synthetic fallback
        (logger or log).warning("ABCD HDF5 unavailable (%s); using synthetic ABCD-shape cohort", e)
        return load_partition_data_abcd_synthetic(client_number, "site" if partition_method == "site" else partition_method,
                                                  partition_alpha, batch_size, shape=shape, device=device,
                                                  logger=logger)
    if X is None:
        raise ValueError("HDF5 file has no 'X' volumes")
    store = _cohort_store(X, y, site, device)
    train, test, _ = P.partition_by_site(np.asarray(site), max_clients=max_clients)
    return _assemble(store, train, test, batch_size, 2, logger)


def load_partition_data_abcd_rescale(data_dir, partition_method="site", partition_alpha=0.3, client_number=21,
                                     batch_size=16, logger=None, split_ratio=0.2, seed=42, store=None, device="cpu"):
    """Reference signature (``ABCD/data_loader.py:216``): merge every subject of the cohort at ``data_dir`` (or an
    in-memory ``store``), seeded 80/20 split, then ``client_number`` contiguous equal shards (IID by order); the
    test shards are the matching slices of the test pool."""
    if store is None:
        store = _load_store(data_dir, device, logger)
    n = len(store)
    ix = np.arange(n)
    np.random.RandomState(seed).shuffle(ix)
    nt = int(n * split_ratio)
    tr, te = ix[:n - nt], ix[n - nt:]
    train = {c: s for c, s in enumerate(np.array_split(tr, client_number))}
    test = {c: s for c, s in enumerate(np.array_split(te, client_number))}
    return _assemble(store, train, test, batch_size, 2, logger)


def _load_store(data_dir, device="cpu", logger=None):
    """VolumeStore of a cohort path (NIDTVOL1 file / directory, or HDF5 with h5py); synthetic if absent."""
    path = data_dir
    if path and os.path.isdir(path):
        nv = os.path.join(path, "alldatain8bitsnormalized.nidtvol")
        path = nv if os.path.exists(nv) else os.path.join(path, "alldatain8bitsnormalized.h5")
    if path and str(path).endswith(".nidtvol") and os.path.exists(path):
        from .volume_file import VolumeFile
        return VolumeFile(path).to_store(device=device)
    try:
        X, y, site = _read_h5(path)
    except Exception as e:  # noqa: BLE001
        (logger or log).warning("ABCD cohort unavailable (%s); using a synthetic ABCD-shape cohort", e)
        return make_synthetic_abcd(21 * 40, seed=0, device=device)
    return _cohort_store(X, y, site, device)
