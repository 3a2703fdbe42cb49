"""ABCD cohort preprocessing (reference ``Preprocess_ABCD.ipynb``), producing the uint8 volume store.

The notebook's steps, reproduced on arrays (NIfTI reading needs nibabel, which this image does not ship; pass
the grey-matter maps as a float array, an ``.npy`` memory map, or any iterable of volumes):

1. brain mask = mean grey-matter image > 0.2 (cells 12-16);
2. every subject multiplied by the mask (cell 20);
3. per-subject min-max scaling over the masked volume and 8-bit quantisation by truncation,
   ``uint8((v - min) / (max - min) * 255)`` (cells 33 / 37);
4. labels: sex as pandas category codes of ``female`` (codes follow the sorted categories), site via
   ``LabelEncoder`` (sorted unique site names) (cells 27-28).

The result is written as a NIDTVOL1 file (:func:`data.volume_file.write_volume_file`), which the native
reader memory-maps (the notebook saved an HDF5 with keys ``X``, ``y``, ``site``).  The volumes are quantised and
written one subject at a time, so the cohort is never resident in host memory (the float cohort is 97 GB).

CLI: ``python -m neuroimagedisttraining_amd.data.preprocess <X.npy> <labels.npz> out.nidtvol`` with the float
grey-matter maps ``X`` [N, D, H, W] as a ``.npy`` (memory-mapped, ``mmap_mode='r'``) and ``female`` / ``site``
arrays in the npz (loaded with ``allow_pickle=False``).
"""
from __future__ import annotations

import sys

import numpy as np


def brain_mask(volumes, threshold=0.2):
    """Mean image over subjects > ``threshold`` (one streaming pass)."""
    acc, n = None, 0
    for v in volumes:
        v = np.asarray(v, dtype=np.float64)
        acc = v.copy() if acc is None else acc + v
        n += 1
    if n == 0:
        raise ValueError("brain_mask: no volumes")
    return (acc / n) > threshold


def quantize_subject(volume, mask):
    """Masked per-subject min-max to [0, 1] and 8-bit truncation (``astype(np.uint8)`` of ``x * 255``)."""
    v = np.asarray(volume, dtype=np.float64) * mask
    lo, hi = float(v.min()), float(v.max())
    if hi <= lo:
        return np.zeros(v.shape, dtype=np.uint8)
    return ((v - lo) / (hi - lo) * 255.0).astype(np.uint8)


def category_codes(values):
    """pandas ``astype('category').cat.codes``: index into the sorted unique non-missing values, -1 for missing."""
    vals = np.asarray(values, dtype=object)
    missing = np.array([x is None or (isinstance(x, float) and np.isnan(x)) or x == "" for x in vals])
    cats = sorted({x for x, m in zip(vals, missing) if not m})
    index = {c: i for i, c in enumerate(cats)}
    return np.array([-1 if m else index[x] for x, m in zip(vals, missing)], dtype=np.int64), cats


def label_encode(values):
    """sklearn ``LabelEncoder().fit_transform``: index into the sorted unique values (missing as a value)."""
    vals = np.asarray(["" if v is None else v for v in values], dtype=object).astype(str)
    cats = sorted(set(vals.tolist()))
    index = {c: i for i, c in enumerate(cats)}
    return np.array([index[x] for x in vals], dtype=np.int64), cats


def preprocess_cohort(volumes, female, site, out_path=None, threshold=0.2, drop_missing=True):
    """Mask, quantise and label a cohort.

    ``volumes`` must be re-iterable (array, ``np.load(..., mmap_mode='r')`` memory map, or a sequence of
    per-subject arrays): pass 1 computes the mean-image mask, pass 2 quantises one subject at a time.  With
    ``out_path`` each quantised subject is streamed straight into the NIDTVOL1 file (host memory holds one subject,
    never the cohort) and ``(None, y, site_codes)`` is returned; without it the uint8 cohort is returned.
    ``drop_missing``: subjects whose sex is missing (category code -1) are left out instead of being written with
    label -1, which a BCE loss would consume as a target."""
    mask = brain_mask(volumes, threshold)
    y, _ = category_codes(female)
    s, _ = label_encode(site)
    keep = np.nonzero(y >= 0)[0] if drop_missing else np.arange(len(y))
    if out_path is None:
        q = np.stack([quantize_subject(volumes[i], mask) for i in keep]) if len(keep) else None
        return q, y[keep], s[keep]
    from .volume_file import write_volume_file
    shape = tuple(np.asarray(volumes[int(keep[0])]).shape) if len(keep) else tuple(np.asarray(volumes[0]).shape)

    class _Quantised:  # sliceable view that quantises on demand (the writer streams `chunk` subjects at a time)
        def __init__(self):
            self.shape = (len(keep),) + shape

        def __getitem__(self, sl):
            return np.stack([quantize_subject(volumes[int(i)], mask) for i in keep[sl]])

    write_volume_file(out_path, _Quantised(), y[keep].astype(np.float32), s[keep].astype(np.float32), chunk=1)
    return None, y[keep], s[keep]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 3:
        print(__doc__)
        return 2
    X = np.load(argv[0], mmap_mode="r", allow_pickle=False)
    d = np.load(argv[1], allow_pickle=False)
    _, y, s = preprocess_cohort(X, d["female"], d["site"], out_path=argv[2])
    print("wrote %s: %d subjects (%d dropped: missing sex) %s, %d sites" % (
        argv[2], len(y), X.shape[0] - len(y), tuple(X.shape[1:]), len(set(s.tolist()))))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
