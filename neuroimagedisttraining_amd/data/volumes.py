"""Device-resident uint8 volume store + synthetic ABCD-shape sMRI generator.

The reference keeps only an *index* tensor in its DataLoaders and re-opens an HDF5 file on every
batch to fetch ``X`` (8-bit normalised grey-matter maps) and ``y``
(``ABCD/data_loader.py:119``, ``sailentgrads/my_model_trainer.py:185-199``).  Here the volumes live
once in HBM as uint8 (2.1 MB/subject; the whole 11.5k-subject cohort is ~24 GB, a fraction of one
MI355X's 288 GB) and a batch fetch is a device gather + uint8->float/bf16 convert (/255) —
no host round trip per step.

Batches keep the reference's 3-tuple contract ``(x_index, y, site)`` so algorithm code that walks
``train_data_local_dict[c]`` works unchanged; :meth:`VolumeStore.fetch` turns the index column
into voxels.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

ABCD_SHAPE = (121, 145, 121)


@dataclass
class VolumeStore:
    volumes: torch.Tensor        # uint8 [N, D, H, W] (device or host)
    labels: torch.Tensor         # float32 [N]
    site: torch.Tensor           # float32 [N]

    @property
    def shape(self):
        return tuple(self.volumes.shape[1:])

    def __len__(self):
        return self.volumes.shape[0]

    def to(self, device):
        return VolumeStore(self.volumes.to(device), self.labels.to(device), self.site.to(device))

    def fetch(self, index, device=None, dtype=torch.float32, sort=True):
        """Gather volumes by (float or int) subject index -> ``(x [B,1,D,H,W], y [B])``.

        ``sort=True`` reproduces the reference's sorted fancy-index HDF5 read, which returns
        samples (and labels) in ascending subject order (``my_model_trainer.py:191-196``)."""
        idx = torch.as_tensor(index).to(torch.long).flatten()
        if sort:
            idx, _ = torch.sort(idx)
        dev = self.volumes.device if device is None else torch.device(device)
        idx_v = idx.to(self.volumes.device)
        x = self.volumes.index_select(0, idx_v)
        if x.device != dev:
            x = x.to(dev, non_blocking=True)
        x = (x.to(dtype) * (1.0 / 255.0)).unsqueeze(1)
        y = self.labels.index_select(0, idx_v).to(dev)
        return x, y


def quantize_cohort_volumes(X, chunk=64, atol=1e-3):
    """Cohort volumes ``X`` ([N, D, H, W], numpy array / tensor / h5py dataset) -> uint8 numpy array, without ever
    silently zeroing the data.

    * uint8 is taken as is; other integer dtypes must lie in [0, 255];
    * float volumes are accepted only in the reference's stored form, the 8-bit quantised maps divided by 255
      (``Preprocess_ABCD.ipynb``: ``eight_bit_data = (...).astype(np.uint8) / 255.0``, read back as float32 by
      ``sailentgrads/my_model_trainer.py:194-197``): ``round(X * 255)`` is kept when every ``|X*255 - round(X*255)|``
      is below ``atol`` and the result lies in [0, 255];
    * anything else raises ``ValueError`` naming the dtype and range.
    Processed ``chunk`` subjects at a time, so an HDF5 dataset is never materialised as floats."""
    n = int(X.shape[0])
    out = np.empty(tuple(int(s) for s in X.shape), dtype=np.uint8)
    for s in range(0, n, chunk):
        v = X[s:s + chunk]
        v = v.cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
        if v.dtype == np.uint8:
            out[s:s + len(v)] = v
            continue
        if np.issubdtype(v.dtype, np.integer) or v.dtype == np.bool_:
            lo, hi = int(v.min()), int(v.max())
            if lo < 0 or hi > 255:
                raise ValueError("cohort X (dtype %s) has integer values in [%d, %d], outside uint8" % (v.dtype, lo, hi))
            out[s:s + len(v)] = v.astype(np.uint8)
            continue
        if not np.issubdtype(v.dtype, np.floating):
            raise ValueError("cohort X has unsupported dtype %s" % v.dtype)
        x = v.astype(np.float64) * 255.0
        q = np.rint(x)
        err = float(np.abs(x - q).max()) if x.size else 0.0
        lo, hi = float(v.min()), float(v.max())
        if not np.isfinite(err) or err >= atol or q.min() < 0 or q.max() > 255:
            raise ValueError("cohort X (dtype %s, range [%g, %g]) is not 8-bit data stored as k/255 (max |X*255 - "
                             "round(X*255)| = %g): quantise it like Preprocess_ABCD.ipynb before loading"
                             % (v.dtype, lo, hi, err))
        out[s:s + len(v)] = q.astype(np.uint8)
    return out


def _smooth_field(gen, n, coarse, shape, device):
    """Low-frequency random field: coarse normal noise trilinearly upsampled to ``shape``."""
    z = torch.randn((n, 1) + tuple(coarse), generator=gen, device=device)
    return torch.nn.functional.interpolate(z, size=shape, mode="trilinear", align_corners=False)[:, 0]


def make_synthetic_abcd(n_subjects, shape=ABCD_SHAPE, n_sites=21, seed=0, device="cpu",
                        label_signal=0.35, site_shift=0.08, chunk=64, labels=None, site=None):
    """Synthetic grey-matter-like volumes of ABCD shape with a learnable sex signal.

    * brain: an ellipsoid mask (≈ the reference's mean-image>0.2 mask) filled with a smooth
      random field (folding-like texture) in [0,1];
    * label: class-1 subjects get extra intensity in two bilateral ellipsoidal "regions";
    * site: a per-site global intensity/contrast shift (scanner effect) so site-clients are
      non-IID in their input distribution;
    * quantised to uint8 exactly like the reference's preprocessing (min-max, x255).
    Labels are balanced Bernoulli(0.5); sites are drawn with a skewed (Zipf-like) size profile.
    """
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(int(seed))
    rs = np.random.RandomState(seed)
    lab_draw = rs.randint(0, 2, size=n_subjects).astype(np.float32)
    labels = lab_draw if labels is None else np.asarray(labels, dtype=np.float32)
    w = 1.0 / np.arange(1, n_sites + 1) ** 0.5
    site_draw = rs.choice(n_sites, size=n_subjects, p=w / w.sum()).astype(np.float32)
    site = site_draw if site is None else np.asarray(site, dtype=np.float32)
    if len(site) != n_subjects or len(labels) != n_subjects:
        raise ValueError("labels / site must have one entry per subject")
    if site.size and (site.min() < 0 or site.max() >= n_sites):  # indexes the per-site gain table on device
        raise ValueError("site ids must lie in [0, n_sites=%d)" % n_sites)
    rs = np.random.RandomState(12345)  # scanner effects are a property of the site, shared by all clients
    site_gain = 1.0 + site_shift * rs.randn(n_sites).astype(np.float32)
    site_bias = site_shift * 0.5 * rs.randn(n_sites).astype(np.float32)

    D, H, W = shape
    zz = torch.linspace(-1, 1, D, device=device).view(D, 1, 1)
    yy = torch.linspace(-1, 1, H, device=device).view(1, H, 1)
    xx = torch.linspace(-1, 1, W, device=device).view(1, 1, W)
    r2 = (zz / 0.82) ** 2 + (yy / 0.86) ** 2 + (xx / 0.80) ** 2
    brain = (r2 < 1.0).float() * (1.0 - 0.35 * r2.clamp(max=1.0))
    roi = torch.exp(-(((zz - 0.1) / 0.18) ** 2 + ((yy + 0.2) / 0.22) ** 2 + ((xx.abs() - 0.4) / 0.15) ** 2))

    out = torch.empty((n_subjects, D, H, W), dtype=torch.uint8, device=device)
    coarse = (max(2, D // 8), max(2, H // 8), max(2, W // 8))
    lab_t = torch.from_numpy(labels).to(device)
    site_i = torch.from_numpy(site.astype(np.int64)).to(device)
    g_t = torch.from_numpy(site_gain).to(device)
    b_t = torch.from_numpy(site_bias).to(device)
    for s in range(0, n_subjects, chunk):
        e = min(n_subjects, s + chunk)
        n = e - s
        tex = _smooth_field(gen, n, coarse, shape, device)
        fine = _smooth_field(gen, n, (coarse[0] * 2, coarse[1] * 2, coarse[2] * 2), shape, device)
        v = brain * (0.55 + 0.18 * tex + 0.10 * fine)
        v = v + label_signal * lab_t[s:e].view(n, 1, 1, 1) * roi * brain
        v = v * g_t[site_i[s:e]].view(n, 1, 1, 1) + b_t[site_i[s:e]].view(n, 1, 1, 1) * brain
        v = v.clamp_(min=0)
        mx = v.flatten(1).amax(1).clamp(min=1e-6).view(n, 1, 1, 1)
        out[s:e] = (v / mx * 255.0).round_().to(torch.uint8)
    return VolumeStore(out, torch.from_numpy(labels).to(device), torch.from_numpy(site).to(device))


def reference_cohort_sizes(n_clients, n_train_total=9216, test_ratio=0.2):
    """Per-client train/test sizes for the headline config: the ABCD train pool (≈9.2k of 11,573
    subjects after the per-site 80/20 split) divided into ``n_clients`` equal
    quotas (the ``dir`` partitioner's sigma=0 lognormal quota)."""
    per = n_train_total // n_clients
    n_test = int(math.ceil(per * test_ratio / (1 - test_ratio)))
    return per, n_test
