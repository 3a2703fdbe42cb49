"""Readers of the reference's on-disk image datasets (no network, no torchvision, nothing unpickled).

* **Tiny-ImageNet** (``tiny_imagenet/datasets.py:46-105``): ``<root>/tiny-imagenet-200/{train,val}_list.txt`` lists
  ``<relative jpeg path> <label>`` per line; every JPEG is decoded with PIL (``.convert('RGB')``).  The reference
  stacks the HWC decodes, then ``reshape(-1, 3, 64, 64).transpose(0, 2, 3, 1)`` — a reinterpretation of each
  image's HWC bytes as CHW, which scrambles the pixels.  ``ref_pixel_order=True`` reproduces that scramble
  (PARITY.md §2.5); the default keeps the decoded images intact.  The decode is cached next to the lists as
  ``tiny{True,False}[_refpix].npz`` (the reference caches a pickle; here an ``.npz`` read with
  ``allow_pickle=False``).
* **CIFAR-10 / CIFAR-100** (``cifar10/datasets.py:49-60`` reads torchvision's ``CIFAR10(root)``): the binary
  distribution — ``cifar-10-batches-bin/data_batch_{1..5}.bin`` + ``test_batch.bin`` (records of 1 label byte +
  3072 CHW pixel bytes) and ``cifar-100-binary/{train,test}.bin`` (coarse label byte, fine label byte, 3072
  pixels; the fine label is the class, as torchvision's ``CIFAR100``).  torchvision's python layout
  (``cifar-10-batches-py``) is pickles and is refused with a pointer to the binary one.

Every reader returns ``(uint8 [N, H, W, 3], int64 [N])``, the ``.data`` / ``.targets`` layout of the reference's
dataset objects.  A ``data_dir`` that holds none of the expected files raises: images are synthesised only when
no ``data_dir`` is given (``data_dir=""``).
"""
from __future__ import annotations

import logging
import os

import numpy as np

log = logging.getLogger(__name__)

_CIFAR = {
    "cifar10": ("cifar-10-batches-bin", ["data_batch_%d.bin" % i for i in range(1, 6)], ["test_batch.bin"], 1),
    "cifar100": ("cifar-100-binary", ["train.bin"], ["test.bin"], 2),
}


def _cifar_dir(name, root):
    sub, trn, tst, _ = _CIFAR[name]
    for d in (os.path.join(root, sub), root):
        if all(os.path.isfile(os.path.join(d, f)) for f in trn + tst):
            return d
    return None


def read_cifar_bin(name, root, train):
    """CIFAR-10/100 binary batches under ``root`` (or ``root/<cifar-*-bin>``) -> (uint8 [N,32,32,3], int64 [N])."""
    d = _cifar_dir(name, root)
    if d is None:
        raise FileNotFoundError(_missing(name, root))
    _, trn, tst, nlab = _CIFAR[name]
    xs, ys = [], []
    for f in (trn if train else tst):
        raw = np.fromfile(os.path.join(d, f), dtype=np.uint8)
        rec = 3072 + nlab
        if raw.size % rec:
            raise ValueError("%s: %s is not a whole number of %d-byte records" % (name, f, rec))
        raw = raw.reshape(-1, rec)
        ys.append(raw[:, nlab - 1].astype(np.int64))  # CIFAR-100: the fine label (second byte)
        xs.append(raw[:, nlab:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return np.ascontiguousarray(np.concatenate(xs)), np.concatenate(ys)


def _tiny_dir(root):
    for d in (os.path.join(root, "tiny-imagenet-200"), root):
        if os.path.isfile(os.path.join(d, "train_list.txt")) and os.path.isfile(os.path.join(d, "val_list.txt")):
            return d
    return None


def _read_list(path):
    names, labels = [], []
    with open(path) as f:
        for line in f:
            if line.strip():
                img, lbl = line.strip().split()
                names.append(img)
                labels.append(int(lbl))
    return names, np.asarray(labels, dtype=np.int64)


def read_tiny_imagenet(root, train, ref_pixel_order=False, cache=True):
    """Tiny-ImageNet split from the reference's list files + JPEGs -> (uint8 [N,64,64,3], int64 [N])."""
    d = _tiny_dir(root)
    if d is None:
        raise FileNotFoundError(_missing("tiny", root))
    cpath = os.path.join(d, "tiny%s%s.npz" % (bool(train), "_refpix" if ref_pixel_order else ""))
    if cache and os.path.isfile(cpath):
        z = np.load(cpath, allow_pickle=False)
        return z["data"], z["targets"]
    from PIL import Image
    names, labels = _read_list(os.path.join(d, "train_list.txt" if train else "val_list.txt"))
    data = np.empty((len(names), 64, 64, 3), dtype=np.uint8)
    for i, n in enumerate(names):
        with Image.open(os.path.join(d, n)) as im:
            a = np.asarray(im.convert("RGB"))
        if a.shape != (64, 64, 3):
            raise ValueError("tiny: %s decodes to %s, expected 64x64 RGB" % (n, a.shape))
        data[i] = a
        if i % 10000 == 9999:
            log.info("tiny: decoded %d / %d %s images", i + 1, len(names), "train" if train else "val")
    if ref_pixel_order:  # the reference's stack + reshape(-1, 3, 64, 64) + transpose(0, 2, 3, 1)
        data = np.ascontiguousarray(data.reshape(-1, 3, 64, 64).transpose(0, 2, 3, 1))
    if cache:
        try:
            tmp = cpath + ".tmp.npz"
            np.savez(tmp, data=data, targets=labels)
            os.replace(tmp, cpath)
        except OSError as e:  # a read-only dataset directory: decode again next time
            log.warning("tiny: could not write the decode cache %s (%s)", cpath, e)
    return data, labels


def _missing(name, root):
    if name == "tiny":
        want = "tiny-imagenet-200/{train,val}_list.txt (+ the JPEGs they list)"
    else:
        sub, trn, tst, _ = _CIFAR[name]
        want = "%s/{%s}" % (sub, ",".join(trn + tst))
        if os.path.isdir(os.path.join(root, sub.replace("-bin", "-py").replace("-binary", "-python"))):
            want += " (torchvision's python layout holds pickles, which are never loaded: use the binary version)"
    return ("%s: --data_dir %r holds no dataset files; expected %s under it, an .npz with x_train/y_train/x_test/"
            "y_test, or --data_dir '' for synthetic images" % (name, root, want))


def read_image_split(name, root, train, ref_pixel_order=False):
    """Dispatch on ``name`` in {cifar10, cifar100, tiny} for a dataset directory ``root`` (raises when absent)."""
    if not os.path.isdir(root):
        raise FileNotFoundError("%s: --data_dir %r does not exist" % (name, root))
    if name == "tiny":
        return read_tiny_imagenet(root, train, ref_pixel_order)
    if name in _CIFAR:
        return read_cifar_bin(name, root, train)
    raise ValueError("no on-disk reader for dataset %r" % name)
