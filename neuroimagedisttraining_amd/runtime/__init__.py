"""Host-side native runtime modules (C++17, built in-tree by ``tools/build_ext.py`` from ``csrc/runtime``).

* ``_nidt_io`` — memory-mapped NIDTVOL1 volume-store reader with a worker-pool gather into pinned buffers
  (``csrc/runtime/volume_io.cpp``; Python side: :mod:`neuroimagedisttraining_amd.data.volume_file`).

Unlike the GPU extension these have no device dependency, so they build, import and are tested on CPU.
:func:`io` raises if the module was not built (no silent Python fallback).
"""
from __future__ import annotations

import importlib
import os
import sys

_MODS = {}


def _load(name):
    if name not in _MODS:
        here = os.path.dirname(os.path.abspath(__file__))
        if here not in sys.path:
            sys.path.insert(0, here)
        try:
            _MODS[name] = importlib.import_module(name)
        except ImportError as e:
            _MODS[name] = e
    m = _MODS[name]
    if isinstance(m, Exception):
        raise RuntimeError("native runtime module %s not built (%r); run `python tools/build_ext.py`" % (name, m))
    return m


def io():
    """The ``_nidt_io`` module (VolumeReader)."""
    return _load("_nidt_io")
