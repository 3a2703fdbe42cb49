"""CIFAR-10 / CIFAR-100 / Tiny-ImageNet / tabular federated loaders (reference
``fedml_api/data_preprocessing/{cifar10,cifar100,tiny_imagenet}/{data_loader,data_val_loader}.py``).

Images come from ``data_dir``: the reference's dataset directories (Tiny-ImageNet list files + JPEGs, the CIFAR
binary batches: ``data/image_files.py``) or an ``.npz`` with ``x_train, y_train, x_test, y_test`` (loaded with
``allow_pickle=False``); uint8 pixels are normalised with the reference loader's mean/std.  Without a
``data_dir`` each loader builds a synthetic dataset of the real shape and class count (class-conditional smooth
patterns + noise, learnable); a ``data_dir`` that holds no dataset files raises.  Partitioning and the
per-client test / validation construction follow the reference exactly:

* train split: ``partition_method`` in {dir, n_cls, my_part, homo, hetero};
* per-client test set: for each class ``c``, ``ceil(train_count_c / train_total * ceil(|test| / C))`` random
  test indices of class c (test sets overlap across clients);
* val loaders (9-tuple): 10 % of *client 0's* size sampled from each client's train indices.

Every loader returns the reference's 8-tuple ``[None, None, None, None, train_num_dict, train_dict, test_dict,
class_num]`` (val variant: + ``val_dict``).
"""
from __future__ import annotations

import logging
import math
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, TensorDataset

from ..core import partition as P

log = logging.getLogger(__name__)

SPECS = {"cifar10": ((3, 32, 32), 10, 50000, 10000), "cifar100": ((3, 32, 32), 100, 50000, 10000),
         "tiny": ((3, 64, 64), 200, 100000, 10000), "mnist": ((1, 28, 28), 10, 60000, 10000),
         "emnist": ((1, 28, 28), 62, 60000, 10000)}


def synthetic_images(n, shape, n_cls, seed=0, noise=0.6, template_seed=12345):
    """Class-conditional images: a random low-frequency template per class + per-sample noise.

    The class templates depend only on ``template_seed`` so train and test splits share them."""
    c, h, w = shape
    gt = torch.Generator().manual_seed(template_seed)
    coarse = torch.randn(n_cls, c, max(2, h // 8), max(2, w // 8), generator=gt)
    g = torch.Generator().manual_seed(seed)
    templ = torch.nn.functional.interpolate(coarse, size=(h, w), mode="bilinear", align_corners=False)
    y = torch.randint(0, n_cls, (n,), generator=g)
    x = templ[y] + noise * torch.randn(n, c, h, w, generator=g)
    return x.float(), y.long()


def _as_hwc(x):
    x = np.asarray(x)
    if x.ndim == 4 and x.shape[1] in (1, 3) and x.shape[-1] not in (1, 3):
        x = np.transpose(x, (0, 2, 3, 1))
    return np.ascontiguousarray(x)


def load_raw(dataset, data_dir, n_train=None, n_test=None, seed=0, ref_pixel_order=False):
    """``(x_train, y_train, x_test, y_test, n_cls)`` of ``dataset`` as the files hold them: uint8 ``[N, H, W, C]``
    pixels for the reference's dataset directories (``data/image_files.py``) and uint8 ``.npz`` files; normalised
    float ``[N, C, H, W]`` for a float ``.npz`` and for the synthetic images, which are only made when no
    ``data_dir`` is given — a ``data_dir`` without dataset files raises."""
    shape, n_cls, ntr, nte = SPECS[dataset]
    if data_dir:
        if os.path.isfile(data_dir) and data_dir.endswith(".npz"):
            d = np.load(data_dir, allow_pickle=False)
            xs = [d["x_train"], d["x_test"]]
            if xs[0].dtype == np.uint8:
                xs = [torch.from_numpy(_as_hwc(x)) for x in xs]
            else:
                xs = [torch.from_numpy(np.asarray(x)).float() for x in xs]
            return xs[0], torch.from_numpy(d["y_train"]).long(), xs[1], torch.from_numpy(d["y_test"]).long(), n_cls
        from .image_files import read_image_split
        xtr, ytr = read_image_split(dataset, data_dir, True, ref_pixel_order)
        xte, yte = read_image_split(dataset, data_dir, False, ref_pixel_order)
        return torch.from_numpy(xtr), torch.from_numpy(ytr), torch.from_numpy(xte), torch.from_numpy(yte), n_cls
    ntr = n_train or ntr
    nte = n_test or nte
    xtr, ytr = synthetic_images(ntr, shape, n_cls, seed)
    xte, yte = synthetic_images(nte, shape, n_cls, seed + 1)
    log.info("%s: no --data_dir, using synthetic %s images (%d train / %d test)", dataset, shape, ntr, nte)
    return xtr, ytr, xte, yte, n_cls


def normalise_u8(x, dataset):
    """uint8 ``[N, H, W, C]`` pixels -> float ``[N, C, H, W]``: ``ToTensor`` (/255) then the reference loader's
    ``Normalize(mean, std)`` (``NORM``; datasets without one stop after ``ToTensor``)."""
    f = x.permute(0, 3, 1, 2).float().div_(255.0)
    if dataset in NORM:
        mean, std = NORM[dataset]
        f.sub_(torch.tensor(mean).view(1, -1, 1, 1)).div_(torch.tensor(std).view(1, -1, 1, 1))
    return f.contiguous()


def _load_arrays(dataset, data_dir, n_train=None, n_test=None, seed=0, ref_pixel_order=False):
    """The eager loaders' arrays: normalised float NCHW images (uint8 pixels are normalised here, as the HIP image
    engine normalises them on device) and int64 labels."""
    xtr, ytr, xte, yte, n_cls = load_raw(dataset, data_dir, n_train, n_test, seed, ref_pixel_order)
    if xtr.dtype == torch.uint8:
        xtr, xte = normalise_u8(xtr, dataset), normalise_u8(xte, dataset)
    return xtr, ytr, xte, yte, n_cls


# Normalize constants of the reference loaders (cifar10/data_loader.py:43-44, cifar100/data_loader.py:30-31,
# tiny_imagenet/data_loader.py:49-50); the images handled here are already normalised with them
NORM = {"cifar10": ((0.49139968, 0.48215827, 0.44653124), (0.24703233, 0.24348505, 0.26158768)),
        "cifar100": ((0.5071, 0.4865, 0.4409), (0.2673, 0.2564, 0.2762)),
        "tiny": ((0.5, 0.5, 0.5), (0.5, 0.5, 0.5))}
AUG_PAD = 4


class AugmentedTensorDataset(Dataset):
    """Train-time augmentation of the reference image loaders on normalised CHW tensors: RandomCrop(size, padding=4)
    then RandomHorizontalFlip(0.5) (``cifar10/data_loader.py:46-52``, ``tiny_imagenet/data_loader.py:51-57``).
    The reference pads the uint8 PIL image with 0 before normalising, so the padding here is the normalised value of
    a black pixel, -mean/std per channel.  Draws follow torchvision: top, then left, each ``torch.randint(0, 2 pad +
    1)``, then ``torch.rand(1) < 0.5`` for the flip (global torch RNG, as the reference's DataLoader workers)."""

    def __init__(self, x, y, mean, std, pad=AUG_PAD):
        self.x, self.y, self.pad = x, y, int(pad)
        self.fill = (-torch.tensor(mean, dtype=x.dtype) / torch.tensor(std, dtype=x.dtype)).view(-1, 1, 1)

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        img = self.x[i]
        C, H, W = img.shape
        p = self.pad
        top = int(torch.randint(0, 2 * p + 1, (1,)))
        left = int(torch.randint(0, 2 * p + 1, (1,)))
        padded = self.fill[:C].expand(C, H + 2 * p, W + 2 * p).clone()
        padded[:, p:p + H, p:p + W] = img
        out = padded[:, top:top + H, left:left + W]
        if float(torch.rand(1)) < 0.5:
            out = out.flip(-1)
        return out.contiguous(), self.y[i]


def _loader(x, y, idx, bs, shuffle, augment=None):
    """``augment``: (mean, std) of the dataset -> train-time RandomCrop + RandomHorizontalFlip."""
    idx = torch.as_tensor(np.asarray(idx, dtype=np.int64))
    ds = AugmentedTensorDataset(x[idx], y[idx], *augment) if augment is not None else TensorDataset(x[idx], y[idx])
    return DataLoader(ds, batch_size=bs, shuffle=shuffle, drop_last=False)


def partition_data(y_train, partition, n_clients, alpha, n_cls, rng=None):
    return P.partition_labels(partition, np.asarray(y_train), n_clients, alpha, n_cls=n_cls, rng=rng)


def load_partition_data(dataset, data_dir, partition_method, partition_alpha, client_number, batch_size,
                        logger=None, n_train=None, n_test=None, seed=0, with_val=False, augment=True,
                        ref_pixel_order=False):
    """``augment``: the reference's train-time RandomCrop(pad 4) + RandomHorizontalFlip on the train loaders of the
    image datasets.  Test loaders are not augmented, as in the reference; validation loaders are not either, which
    deviates from the reference's FedFomo validation loader (built with ``transform_train``,
    ``cifar10/data_val_loader.py:248,309``) — see PARITY.md §2.5."""
    logger = logger or log
    aug = NORM.get(dataset) if augment else None
    xtr, ytr, xte, yte, n_cls = _load_arrays(dataset, data_dir, n_train, n_test, seed, ref_pixel_order)
    rng = np.random.RandomState(seed)
    train_map = partition_data(ytr.numpy(), partition_method, client_number, partition_alpha, n_cls, rng)
    test_map = P.per_client_test_indices(ytr.numpy(), yte.numpy(), train_map, n_cls=n_cls, rng=rng)
    val_map = {}
    if with_val:
        nval = int(0.1 * len(train_map[0]))
        for c in range(client_number):
            ix = np.asarray(train_map[c])
            pick = rng.choice(len(ix), min(nval, len(ix)), replace=False)
            val_map[c] = ix[pick]
            train_map[c] = np.delete(ix, pick)
    num, trn, tst, val = {}, {}, {}, {}
    for c in range(client_number):
        num[c] = len(train_map[c])
        trn[c] = _loader(xtr, ytr, train_map[c], batch_size, True, aug)
        tst[c] = _loader(xte, yte, test_map[c], batch_size, False)
        if with_val:
            val[c] = _loader(xtr, ytr, val_map[c], batch_size, False)
        logger.info("client_idx = %d, local_train_sample_number = %d", c, num[c])
    if with_val:  # reference 9-tuple order: (..., num, train, val, test, class_num) (cifar10/data_val_loader.py:325)
        return [None, None, None, None, num, trn, val, tst, n_cls]
    return [None, None, None, None, num, trn, tst, n_cls]


def load_partition_data_cifar10(data_dir, partition_method, partition_alpha, client_number, batch_size, logger=None,
                                **kw):
    return load_partition_data("cifar10", data_dir, partition_method, partition_alpha, client_number, batch_size,
                               logger, **kw)


def load_partition_data_cifar100(data_dir, partition_method, partition_alpha, client_number, batch_size,
                                 logger=None, **kw):
    return load_partition_data("cifar100", data_dir, partition_method, partition_alpha, client_number, batch_size,
                               logger, **kw)


def load_partition_data_tiny(data_dir, partition_method, partition_alpha, client_number, batch_size, logger=None,
                             **kw):
    return load_partition_data("tiny", data_dir, partition_method, partition_alpha, client_number, batch_size,
                               logger, **kw)


def load_partition_data_with_val(dataset, data_dir, partition_method, partition_alpha, client_number, batch_size,
                                 logger=None, **kw):
    return load_partition_data(dataset, data_dir, partition_method, partition_alpha, client_number, batch_size,
                               logger, with_val=True, **kw)


# ------------------------------------------------------------------------------------------------ tabular
def synthetic_tabular(n_clients=2, n_per_client=500, dim=60, n_cls=10, alpha=1.0, beta=1.0, seed=0):
    """FedProx-style synthetic(alpha, beta) non-IID tabular data: client-specific model and feature shift."""
    rs = np.random.RandomState(seed)
    xs, ys = [], []
    for c in range(n_clients):
        u = rs.normal(0, alpha)
        b = rs.normal(0, beta)
        W = rs.normal(u, 1, (dim, n_cls))
        bias = rs.normal(u, 1, n_cls)
        v = rs.normal(b, 1, dim)
        cov = np.diag(np.power(np.arange(1, dim + 1, dtype=np.float64), -1.2))
        x = rs.multivariate_normal(v, cov, n_per_client)
        y = np.argmax(x @ W + bias, 1)
        xs.append(x.astype(np.float32))
        ys.append(y.astype(np.int64))
    return xs, ys


def load_partition_data_synthetic_tabular(client_number=2, batch_size=32, n_per_client=500, dim=60, n_cls=10,
                                          alpha=1.0, beta=1.0, seed=0, test_ratio=0.2):
    xs, ys = synthetic_tabular(client_number, n_per_client, dim, n_cls, alpha, beta, seed)
    num, trn, tst = {}, {}, {}
    for c in range(client_number):
        n = len(ys[c])
        nt = int(math.floor(n * test_ratio))
        x = torch.from_numpy(xs[c])
        y = torch.from_numpy(ys[c])
        num[c] = n - nt
        trn[c] = DataLoader(TensorDataset(x[nt:], y[nt:]), batch_size=batch_size, shuffle=True)
        tst[c] = DataLoader(TensorDataset(x[:nt], y[:nt]), batch_size=batch_size, shuffle=False)
    return [None, None, None, None, num, trn, tst, n_cls]
