"""Build the in-tree HIP extension ``neuroimagedisttraining_amd/ops/_nidt_hip*.so`` for gfx950.

hipcc cross-compiles without a GPU.  Objects are rebuilt only when their source (or common.h) is newer;
compilation runs in parallel (one hipcc per .hip).  Usage: ``python tools/build_ext.py [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "csrc", "kernels")
BUILD = os.path.join(ROOT, "build", "hip")
OUT_DIR = os.path.join(ROOT, "neuroimagedisttraining_amd", "ops")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def ext_name():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(OUT_DIR, "_nidt_hip" + suffix)


def _includes():
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-I" + KDIR]


def _compile(src, obj, extra):
    cmd = [HIPCC] + FLAGS + extra + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr[-4000:]))
    return obj


def build(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    inc = _includes()
    common_m = max(os.path.getmtime(os.path.join(KDIR, f)) for f in os.listdir(KDIR) if f.endswith(".h"))
    srcs = sorted(os.path.join(KDIR, f) for f in os.listdir(KDIR) if f.endswith(".hip"))
    srcs.append(os.path.join(ROOT, "csrc", "bindings.cpp"))
    jobs = []
    objs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        stale = force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), common_m)
        if stale:
            extra = inc if s.endswith(".cpp") else ["-I" + KDIR]
            if s.endswith(".cpp"):
                extra = extra + ["-x", "hip"]
            jobs.append((s, o, extra))
    nproc = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    if jobs:
        with cf.ThreadPoolExecutor(nproc) as ex:
            futs = [ex.submit(_compile, *j) for j in jobs]
            for f in futs:
                f.result()
                if verbose:
                    print("[build_ext] compiled", os.path.basename(f.result()), flush=True)
    out = ext_name()
    if force or jobs or not os.path.exists(out):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", out] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
        if verbose:
            print("[build_ext] linked", out, flush=True)
    build_runtime(force, verbose)
    return out


def runtime_name(name):
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(ROOT, "neuroimagedisttraining_amd", "runtime", name + suffix)


def build_runtime(force=False, verbose=True):
    """Host-only native runtime modules (csrc/runtime/*.cpp -> neuroimagedisttraining_amd/runtime/<name>.so),
    built with the system C++ compiler: no GPU toolchain or device needed to build, import or test them."""
    rdir = os.path.join(ROOT, "csrc", "runtime")
    cxx = os.environ.get("CXX", "g++")
    outs = []
    for f in sorted(os.listdir(rdir)):
        if not f.endswith(".cpp"):
            continue
        src = os.path.join(rdir, f)
        out = runtime_name("_nidt_" + f[:-4].split("_")[-1])
        outs.append(out)
        deps = [src] + [os.path.join(rdir, h) for h in os.listdir(rdir) if h.endswith(".h")]
        if not force and os.path.exists(out) and os.path.getmtime(out) >= max(map(os.path.getmtime, deps)):
            continue
        cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-Wall", "-Wno-unused-result"] + \
            _includes()[:2] + [src, "-o", out]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("runtime build failed:\n%s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
        if verbose:
            print("[build_ext] built", out, flush=True)
    return outs


if __name__ == "__main__":
    build(force="--force" in sys.argv)
