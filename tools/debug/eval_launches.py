"""Per-launch device time of the grouped evaluation of tools/bench_cifar.py (eval_logits bracketed by
torch.cuda.synchronize): launch shape (G clients x ch samples), ms, us per sample, for the last round's test
evaluation.  Usage: python tools/debug/eval_launches.py [bench_cifar args]."""
import os
import runpy
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from neuroimagedisttraining_amd.engine import resnet2d_hip as R  # noqa: E402
from neuroimagedisttraining_amd.engine import runner as RU  # noqa: E402

log = []
cur = [None]
o_eval, o_grouped = R.ResNetHipEngine.eval_logits, RU.FLRunner.eval_grouped


def eval_logits(self, theta, bufs, idx, G, B):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = o_eval(self, theta, bufs, idx, G, B)
    torch.cuda.synchronize()
    if cur[0] is not None:
        cur[0].append((G, B, time.perf_counter() - t0))
    return r


def grouped(self, theta, bufs, rows, clients, which="test", device_out=False):
    cur[0] = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = o_grouped(self, theta, bufs, rows, clients, which, device_out)
    torch.cuda.synchronize()
    log.append((which, time.perf_counter() - t0, cur[0]))
    cur[0] = None
    return r


R.ResNetHipEngine.eval_logits, RU.FLRunner.eval_grouped = eval_logits, grouped
sys.argv = ["bench_cifar.py"] + sys.argv[1:]
try:
    runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_cifar.py"),
                   run_name="__main__")
finally:
    for which, tot, ls in log[-2:]:
        n = sum(g * b for g, b, _ in ls)
        print("eval_grouped[%s] %.1f ms, %d launches, %d sample slots, launches sum %.1f ms" % (
            which, 1e3 * tot, len(ls), n, 1e3 * sum(t for *_, t in ls)))
        for g, b, t in ls:
            print("   G=%3d ch=%4d  %7.2f ms  %6.2f us/sample" % (g, b, 1e3 * t, 1e6 * t / (g * b)))
