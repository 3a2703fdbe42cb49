"""Upper-bound probe (NOT a valid training run): tools/bench_cifar.py with some extension entry points replaced by
no-ops, to measure what removing that work from the step could gain before building the fusion.
Usage: NIDT_SKIP=gn_param_grads,res_grad python tools/debug/cifar_skip_ab.py [bench_cifar args]."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402,F401  (torch's HIP runtime first, as the package does)
from neuroimagedisttraining_amd import ops  # noqa: E402

m = ops.ext()
for name in filter(None, os.environ.get("NIDT_SKIP", "").split(",")):
    setattr(m, name, lambda *a, **k: None)
    print("probe: %s is a no-op" % name)
if os.environ.get("NIDT_PROBE_NOTRANS") == "1":  # the dgrad-image transposes skipped (stale images: timing only)
    _pc = m.pack_convs

    def _pack_convs(tab, n, nplain, nplain1, ntrans, *rest):
        if nplain or nplain1:
            _pc(tab, n, nplain, nplain1, 0, *rest)
    m.pack_convs = _pack_convs
    print("probe: pack_convs without the transposes")
sys.argv = ["bench_cifar.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_cifar.py"),
               run_name="__main__")
