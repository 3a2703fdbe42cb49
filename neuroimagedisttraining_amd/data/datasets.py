"""Index-subset ("truncated") datasets (reference ``fedml_api/data_preprocessing/{cifar10,cifar100,ABCD}/
datasets.py:36-92`` ``CIFAR10_truncated`` / ``CIFAR100_truncated`` and ``tiny_imagenet/datasets.py:20-270``
``tiny`` / ``tiny_truncated``).

The reference wraps torchvision datasets and decodes Tiny-ImageNet JPEGs into a pickle cache.  Here (no
network, no torchvision, nothing unpickled) the backing arrays come from, in order: an explicit
``cache_data_set`` object with ``.data`` / ``.targets`` (the reference's in-memory cache argument), an ``.npz``
at ``root`` (``x_train, y_train, x_test, y_test``, loaded with ``allow_pickle=False``), the reference's dataset
directory at ``root`` (CIFAR binary batches, Tiny-ImageNet list files + JPEGs: ``data/image_files.py``), or —
only when ``root`` is empty — the synthetic class-conditional images of ``data/images.py``.  ``.data`` is HWC like torchvision's, so transforms written for the reference keep
working; without a transform an item is a CHW float tensor.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch.utils.data import Dataset

from .images import SPECS, synthetic_images


class ArrayData:
    """Minimal stand-in for a torchvision dataset object: ``.data`` (N,H,W,C) and ``.targets``."""

    def __init__(self, data, targets):
        self.data = data
        self.targets = list(np.asarray(targets).tolist())


def load_arrays(name, root, train=True, n=None, seed=0, ref_pixel_order=False):
    """(data [N,H,W,C], targets [N] int64) for ``name`` in {cifar10, cifar100, tiny}: uint8 pixels from the
    reference's dataset directories (``data/image_files.py``) or an ``.npz``; synthetic float images only without a
    ``root`` (a ``root`` with no dataset files raises)."""
    shape, n_cls, ntr, nte = SPECS[name]
    if root and os.path.isfile(root) and root.endswith(".npz"):
        d = np.load(root, allow_pickle=False)
        x = d["x_train" if train else "x_test"]
        y = d["y_train" if train else "y_test"]
        if x.ndim == 4 and x.shape[1] in (1, 3) and x.shape[-1] not in (1, 3):
            x = np.transpose(x, (0, 2, 3, 1))
        return np.ascontiguousarray(x), np.asarray(y, dtype=np.int64)
    if root:
        from .image_files import read_image_split
        return read_image_split(name, root, train, ref_pixel_order)
    n = n or (ntr if train else nte)
    x, y = synthetic_images(n, shape, n_cls, seed=seed + (0 if train else 1))
    return x.permute(0, 2, 3, 1).contiguous().numpy(), y.numpy()


def _to_item(img):
    return torch.as_tensor(np.asarray(img, dtype=np.float32)).permute(2, 0, 1)


class TruncatedDataset(Dataset):
    """``dataidxs``-subset of an array dataset with optional ``transform`` / ``target_transform``."""

    dataset_name = "cifar10"

    def __init__(self, root, cache_data_set=None, dataidxs=None, train=True, transform=None,
                 target_transform=None, download=False, n=None):
        self.root = root
        self.dataidxs = dataidxs
        self.train = train
        self.transform = transform
        self.target_transform = target_transform
        self.download = download  # accepted for signature parity; nothing is ever downloaded
        self.data, self.target = self.__build_truncated_dataset__(cache_data_set, n)

    def __build_truncated_dataset__(self, cache_data_set, n=None):
        if cache_data_set is None:
            data, target = load_arrays(self.dataset_name, self.root, self.train, n=n)
        else:
            data, target = cache_data_set.data, np.array(cache_data_set.targets)
        if self.dataidxs is not None:
            idx = np.asarray(self.dataidxs, dtype=np.int64)
            data, target = data[idx], target[idx]
        return data, target

    def __getitem__(self, index):
        img, target = self.data[index], self.target[index]
        img = self.transform(img) if self.transform is not None else _to_item(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, int(target)

    def __len__(self):
        return len(self.data)


class CIFAR10_truncated(TruncatedDataset):  # noqa: N801 (reference class name)
    dataset_name = "cifar10"


class CIFAR100_truncated(TruncatedDataset):  # noqa: N801
    dataset_name = "cifar100"


class tiny_truncated(TruncatedDataset):  # noqa: N801
    dataset_name = "tiny"


class tiny(Dataset):  # noqa: N801
    """Whole Tiny-ImageNet split (``tiny_imagenet/datasets.py:20-210``): 200 classes of 3x64x64.  The reference
    decodes ``root/tiny-imagenet-200/{train,val}_list.txt`` JPEGs once and caches a pickle; here the same files are
    decoded with PIL and cached as an ``.npz`` (``data/image_files.py``), or the split comes from an ``.npz`` at
    ``root`` or is synthesised (empty ``root``)."""

    def __init__(self, root, train=True, transform=None, target_transform=None, n=None):
        self.root, self.train = root, train
        self.transform, self.target_transform = transform, target_transform
        self.data, t = load_arrays("tiny", root, train, n=n)
        self.targets = list(t.tolist())

    def __getitem__(self, index):
        img, target = self.data[index], self.targets[index]
        img = self.transform(img) if self.transform is not None else _to_item(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target

    def __len__(self):
        return len(self.data)
