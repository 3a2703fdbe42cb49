"""GPU time of the phases of one FL round (tools/bench_cifar.py): every wrapped call is bracketed by
torch.cuda.synchronize(), so each phase's wall time is its device time (plus one drain each; the round gets slower
by those drains — a breakdown, not a rounds/s number).  Prints per-phase totals per round for the steady rounds.
Usage: python tools/debug/round_phases.py [bench_cifar args]."""
import collections
import os
import runpy
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from neuroimagedisttraining_amd.engine import masks as MK  # noqa: E402
from neuroimagedisttraining_amd.engine import runner as RU  # noqa: E402
from neuroimagedisttraining_amd.engine import personalized as PE  # noqa: E402

tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
depth = [0]


def wrap(owner, name, label=None, key_arg=None):
    orig = getattr(owner, name)

    def f(*a, **k):
        if depth[0]:
            return orig(*a, **k)
        lab = label or name
        if key_arg is not None:
            v = k.get("which", a[key_arg] if len(a) > key_arg else "test")
            lab = "%s[%s]" % (lab, v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        depth[0] += 1
        try:
            return orig(*a, **k)
        finally:
            depth[0] -= 1
            torch.cuda.synchronize()
            tot[lab] += time.perf_counter() - t0
            cnt[lab] += 1
    setattr(owner, name, f)


wrap(RU.FLRunner, "train_rows")
wrap(RU.FLRunner, "eval_grouped", key_arg=5)
wrap(MK.MaskSpace, "percentile_prune")
wrap(MK.MaskSpace, "hamming")
wrap(RU.FLRunner, "state_nonzeros")
wrap(PE.SubAvgRunner, "_real_prune_rows")
wrap(RU.FLRunner, "end_of_training")
# DisPFL's round (personalized.py DisPFLRunner.run_round)
wrap(PE.PersonalizedRunner, "eval_local")
wrap(PE.PersonalizedRunner, "snapshot")
wrap(RU.FLRunner, "local_grad")
wrap(MK.MaskSpace, "select")
wrap(MK.MaskSpace, "popcount")
wrap(PE.DisPFLRunner, "_aggregate_neighbours")
rounds = []


def timed_round(orig_round):
    def run_round(self, *a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        before = dict(tot)
        r = orig_round(self, *a, **k)
        torch.cuda.synchronize()
        rounds.append((time.perf_counter() - t0, {kk: tot[kk] - before.get(kk, 0.0) for kk in tot}))
        return r
    return run_round


for cls in (PE.SubAvgRunner, PE.DisPFLRunner):
    cls.run_round = timed_round(cls.run_round)
sys.argv = ["bench_cifar.py"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_cifar.py"),
                   run_name="__main__")
finally:
    for i, (w, ph) in enumerate(rounds):
        rest = w - sum(ph.values())
        print("round %d: %.1f ms | %s | other %.1f ms" % (i, 1e3 * w, ", ".join(
            "%s %.1f" % (kk, 1e3 * v) for kk, v in sorted(ph.items(), key=lambda kv: -kv[1]) if v > 0), 1e3 * rest))
