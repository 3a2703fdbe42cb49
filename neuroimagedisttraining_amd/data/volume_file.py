"""NIDTVOL1 volume files: a flat, memory-mappable cohort format plus an overlapped host->HBM ingest pipeline.

The reference reads ABCD volumes from an HDF5 file that it re-opens for every batch and copies as float32
(``sailentgrads/my_model_trainer.py:185-199``).  Here a cohort is converted once into a flat file

    [128-B header "NIDTVOL1"][pad to 4 KiB][uint8 volumes N x D x H x W][float32 labels N][float32 sites N]

read by the native ``_nidt_io.VolumeReader`` (``csrc/runtime/volume_io.cpp``: mmap + a C++ worker pool that
gathers subjects into pinned host buffers, GIL released).  :func:`stream_to_device` moves a subject list into
HBM in chunks with three stages in flight — native gather of chunk k+1 into one pinned buffer, a non-blocking
H2D copy of chunk k on a dedicated copy stream, and (for the HIP engine) the polyphase + patch-moment kernels
of chunk k on the compute stream after an event wait — so ingest runs at the slower of disk/PCIe/kernel rate
instead of their sum.  uint8 on disk and over PCIe (2.1 MB per ABCD subject) is 4x less traffic than the
reference's float32.

CLI: ``python -m neuroimagedisttraining_amd.data.volume_file convert <in.npz|in.h5> <out.nidtvol>``
(``.npz`` keys / HDF5 datasets ``X`` [N,D,H,W] uint8, ``y``, ``site``; HDF5 needs h5py).
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np
import torch
from .volumes import quantize_cohort_volumes

MAGIC = b"NIDTVOL1"
HEADER = 128
ALIGN = 4096


def _header(n, shape, data_off, labels_off, sites_off):
    d, h, w = shape
    hdr = MAGIC + struct.pack("<II4Q3Q", 1, 0, n, d, h, w, data_off, labels_off, sites_off)
    return hdr + b"\0" * (HEADER - len(hdr))


def write_volume_file(path, volumes, labels, sites=None, chunk=64):
    """Write ``volumes`` (uint8 ``[N, D, H, W]`` numpy array / tensor / any sliceable) with ``labels`` and
    ``sites`` (float32 ``[N]``) as a NIDTVOL1 file, streaming ``chunk`` subjects at a time."""
    n = int(volumes.shape[0])
    shape = tuple(int(s) for s in volumes.shape[1:])
    assert len(shape) == 3, "volumes must be [N, D, H, W]"
    vox = shape[0] * shape[1] * shape[2]
    data_off = ALIGN
    labels_off = data_off + n * vox
    sites_off = labels_off + 4 * n
    lab = np.asarray(labels.cpu() if torch.is_tensor(labels) else labels, dtype=np.float32).reshape(n)
    sit = np.zeros(n, np.float32) if sites is None else \
        np.asarray(sites.cpu() if torch.is_tensor(sites) else sites, dtype=np.float32).reshape(n)
    with open(path, "wb") as f:
        f.write(_header(n, shape, data_off, labels_off, sites_off))
        f.write(b"\0" * (data_off - HEADER))
        for s in range(0, n, chunk):
            v = volumes[s:s + chunk]
            v = v.cpu().numpy() if torch.is_tensor(v) else np.asarray(v)
            if v.dtype != np.uint8:  # the reference's float k/255 maps quantise exactly; anything else raises
                v = quantize_cohort_volumes(v)
            f.write(np.ascontiguousarray(v).tobytes())
        f.write(lab.tobytes())
        f.write(sit.tobytes())
    return path


class VolumeFile:
    """Native reader of a NIDTVOL1 file (``threads`` C++ gather workers)."""

    def __init__(self, path, threads=0):
        from .. import runtime
        self.r = runtime.io().VolumeReader(os.fspath(path), int(threads))
        self.path = os.fspath(path)

    def __len__(self):
        return int(self.r.n)

    @property
    def shape(self):
        return tuple(int(s) for s in self.r.shape)

    @property
    def labels(self):
        return self.r.labels()

    @property
    def sites(self):
        return self.r.sites()

    def gather(self, indices, out=None):
        """Subjects ``indices`` -> uint8 tensor ``[len, D, H, W]`` (into ``out`` if given, e.g. pinned)."""
        ix = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(-1))
        if out is None:
            out = torch.empty((ix.size,) + self.shape, dtype=torch.uint8)
        assert out.dtype == torch.uint8 and out.is_contiguous() and out.device.type == "cpu"
        assert out.numel() >= ix.size * int(self.r.voxels), "destination too small"
        self.r.gather(ix, out.data_ptr())
        return out[:ix.size]

    def submit(self, indices, out):
        ix = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(-1))
        assert out.dtype == torch.uint8 and out.is_contiguous() and out.device.type == "cpu"
        assert out.numel() >= ix.size * int(self.r.voxels), "destination too small"
        return self.r.submit(ix, out.data_ptr())

    def wait(self, ticket):
        self.r.wait(ticket)

    def prefetch(self, indices):
        self.r.prefetch(np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(-1)))

    def to_store(self, indices=None, device="cpu", chunk=64):
        """:class:`VolumeStore` of ``indices`` (default: all) resident on ``device``."""
        from .volumes import VolumeStore
        ix = np.arange(len(self)) if indices is None else np.asarray(indices, dtype=np.int64)
        vol = stream_to_device(self, ix, device, chunk=chunk)
        lab = torch.from_numpy(self.labels[ix]).to(device)
        sit = torch.from_numpy(self.sites[ix]).to(device)
        return VolumeStore(vol, lab, sit)


def stream_to_device(vf: VolumeFile, indices, device, chunk=64, hip_store=False):
    """Move subjects ``indices`` of ``vf`` to ``device`` with gather / H2D / (HIP) transform overlapped.

    Returns a uint8 ``[N, D, H, W]`` tensor, or with ``hip_store=True`` (ABCD-shape volumes on a GPU) the HIP
    engine's ``(x8 polyphase store, patch moments)`` pair — the raw volumes then never live in HBM at once."""
    device = torch.device(device)
    ix = np.asarray(indices, dtype=np.int64).reshape(-1)
    N = ix.size
    shp = vf.shape
    if device.type != "cuda":
        return vf.gather(ix)
    pin = [torch.empty((chunk,) + shp, dtype=torch.uint8).pin_memory() for _ in range(2)]
    dev = [torch.empty((chunk,) + shp, dtype=torch.uint8, device=device) for _ in range(2)]
    copy_stream = torch.cuda.Stream(device=device)
    compute = torch.cuda.current_stream(device)
    copied = [torch.cuda.Event() for _ in range(2)]
    consumed = [torch.cuda.Event() for _ in range(2)]
    if hip_store:
        from .. import ops
        m = ops.ext()
        x8 = torch.empty((N, 61, 73, 61, 8), dtype=torch.uint8, device=device)
        mom = torch.empty((N, 125 + 125 * 125), dtype=torch.float64, device=device)
    else:
        out = torch.empty((N,) + shp, dtype=torch.uint8, device=device)
    starts = list(range(0, N, chunk))
    tickets = {}

    def _submit(k):
        s = starts[k]
        tickets[k] = vf.submit(ix[s:s + chunk], pin[k % 2])

    if starts:
        _submit(0)
    for k, s in enumerate(starts):
        e = min(N, s + chunk)
        b = k % 2
        vf.wait(tickets.pop(k))                      # chunk k is in pinned buffer b
        with torch.cuda.stream(copy_stream):
            copy_stream.wait_event(consumed[b])      # device buffer b no longer read by chunk k-2's kernels
            dev[b][:e - s].copy_(pin[b][:e - s], non_blocking=True)
            copied[b].record(copy_stream)
        if k + 1 < len(starts):
            # pinned buffer (k+1)%2 was last read by chunk k-1's H2D copy: wait for it before refilling
            copied[(k + 1) % 2].synchronize()
            _submit(k + 1)
        compute.wait_event(copied[b])
        if hip_store:
            st = compute.cuda_stream
            m.polyphase(dev[b].data_ptr(), x8[s].data_ptr(), e - s, st)
            m.conv1_sample_moments(x8[s].data_ptr(), e - s, mom[s].data_ptr(), st)
        else:
            out[s:e].copy_(dev[b][:e - s])
        consumed[b].record(compute)
    torch.cuda.current_stream(device).synchronize()
    return (x8, mom) if hip_store else out


def convert(src, dst):
    if src.endswith(".npz"):
        d = np.load(src, allow_pickle=False)
        X, y = d["X"], d["y"]
        site = d["site"] if "site" in d else None
    else:
        import h5py  # optional
        with h5py.File(src, "r") as f:
            X, y = f["X"], f["y"][()]
            site = f["site"][()] if "site" in f else None
            return write_volume_file(dst, X, y, site)
    return write_volume_file(dst, X, y, site)


if __name__ == "__main__":
    if len(sys.argv) != 4 or sys.argv[1] != "convert":
        print("usage: python -m neuroimagedisttraining_amd.data.volume_file convert <in.npz|in.h5> <out.nidtvol>")
        sys.exit(2)
    print(convert(sys.argv[2], sys.argv[3]))
