"""Host-side time of the lockstep step phases of tools/bench_cifar.py (eager steps): wraps FLRunner._step and the
engine's train_step / local_opt with perf_counter stamps and prints mean / median us per phase, plus the gap between
consecutive steps.  Usage: python tools/debug/step_host_times.py [bench_cifar args]."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from neuroimagedisttraining_amd.engine import resnet2d_hip as R  # noqa: E402
from neuroimagedisttraining_amd.engine import runner as RU  # noqa: E402

rec = {"ts": [], "opt": [], "step": [], "between": [], "fwd": [], "bwd": []}
_last = [None]
o_step, o_ts, o_opt = RU.FLRunner._step, R.ResNetHipEngine.train_step, R.ResNetHipEngine.local_opt
o_feat, o_head = R.GroupedResNet18GN.features, R.GroupedResNet18GN._head_train


def step(self, *a, **k):
    t0 = time.perf_counter()
    if _last[0] is not None:
        rec["between"].append(t0 - _last[0])
    o_step(self, *a, **k)
    _last[0] = time.perf_counter()
    rec["step"].append(_last[0] - t0)


def ts(self, *a, **k):
    t0 = time.perf_counter()
    r = o_ts(self, *a, **k)
    rec["ts"].append(time.perf_counter() - t0)
    return r


def opt(self, *a, **k):
    t0 = time.perf_counter()
    r = o_opt(self, *a, **k)
    rec["opt"].append(time.perf_counter() - t0)
    return r


def feat(self, *a, **k):
    t0 = time.perf_counter()
    r = o_feat(self, *a, **k)
    if k.get("train") or (len(a) > 3 and a[3]):
        rec["fwd"].append(time.perf_counter() - t0)
    return r


RU.FLRunner._step, R.ResNetHipEngine.train_step, R.ResNetHipEngine.local_opt = step, ts, opt
R.GroupedResNet18GN.features = feat
sys.argv = ["bench_cifar.py"] + sys.argv[1:]
import runpy  # noqa: E402
try:
    runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_cifar.py"),
                   run_name="__main__")
finally:
    for k, v in rec.items():
        if v:
            a = np.array(v[len(v) // 2:]) * 1e6  # second half: steady
            print("host %-8s n=%5d mean %8.1f us  median %8.1f  p90 %8.1f" % (k, len(v), a.mean(), np.median(a),
                                                                            np.percentile(a, 90)))
