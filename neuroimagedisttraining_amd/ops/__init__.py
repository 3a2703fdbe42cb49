"""Python bindings of the hand-written CDNA4 (gfx950) HIP kernels in ``csrc/kernels``.

The extension ``_nidt_hip`` is built in-tree by ``python tools/build_ext.py`` (or
``__graft_entry__.build()``) with ``hipcc --offload-arch=gfx950`` and lives next to this file, so it
travels with the repository snapshot.  It is a plain pybind11 module: every entry point takes raw
device pointers, sizes and the HIP stream of the current torch stream.  The wrappers in
:mod:`.kernels` validate shapes / dtypes / contiguity on the host *before* any launch (a mis-shaped
launch could fault the GPU).

Policy: on a machine with a GPU the HIP path is mandatory — :func:`require` raises if the extension is
missing, so nothing silently falls back to eager PyTorch.  CPU-only hosts use the PyTorch reference
implementations in :mod:`.reference` (the same code the numerics tests compare against).
"""
from __future__ import annotations

import importlib
import os
import sys

_EXT = None
_ERR = None


def _load():
    global _EXT, _ERR
    if _EXT is not None or _ERR is not None:
        return _EXT
    here = os.path.dirname(os.path.abspath(__file__))
    if here not in sys.path:
        sys.path.insert(0, here)
    alt = os.environ.get("NIDT_EXT_DIR")  # A/B runs: load another build of _nidt_hip from this directory
    if alt:
        sys.path.insert(0, os.path.abspath(alt))
    try:
        _EXT = importlib.import_module("_nidt_hip")
    except Exception as e:  # noqa: BLE001
        _ERR = e
        _EXT = None
    return _EXT


def available() -> bool:
    return _load() is not None


def ext():
    m = _load()
    if m is None:
        raise RuntimeError("HIP extension _nidt_hip not importable (%r); build it with "
                           "`python tools/build_ext.py`" % (_ERR,))
    return m


def require(device) -> bool:
    """True if the HIP path must be used for tensors on ``device``; raises if the extension is missing."""
    import torch
    dev = torch.device(device)
    if dev.type != "cuda":
        return False
    ext()
    return True


def stream() -> int:
    """Raw ``hipStream_t`` of the current stream on the current device (honours ``torch.cuda.stream(...)``
    contexts and graph capture).  ``torch.cuda.current_stream()`` builds a Python stream object per call
    (~8 us); the small-model engines launch ~10^5 kernels per round, so every launch site uses this instead."""
    import torch
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def ext_path():
    m = _load()
    return getattr(m, "__file__", None) if m is not None else None
