"""Debug: DisPFL on the ResNet engine, hipGraph vs eager, per-round NaN / difference check and capture failures."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig
from neuroimagedisttraining_amd.engine.personalized import make_runner
from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
from neuroimagedisttraining_amd.models import customized_resnet18
from neuroimagedisttraining_amd.parallel import runtime as rt
import neuroimagedisttraining_amd.engine.runner as R
info = rt.init_distributed(prefer_gpu=True)
C, ntr, nte = 4, 20, 8
x8, y = synthetic_cifar(C * (ntr + nte), seed=5)
splits = [ClientSplit(train=np.arange(c * (ntr + nte), c * (ntr + nte) + ntr - 3 * c),
                      test=np.arange(c * (ntr + nte) + ntr, (c + 1) * (ntr + nte))) for c in range(C)]
alg = sys.argv[1] if len(sys.argv) > 1 else "dispfl"
runs = []
for graphs in (False, True):
    torch.manual_seed(0)
    m = customized_resnet18(class_num=10)
    eng = ResNetHipEngine(m, x8, y, "cuda")
    cfg = FLConfig(comm_round=2, epochs=2, batch_size=8, dense_ratio=0.3, seed=1, frac=0.5, lr=0.05,
                   frequency_of_the_test=1, final_round=False, hip_graphs=graphs)
    r = make_runner(alg, eng, splits, cfg, info, m)
    orig = r._graph_step
    log = []
    def gs(sub, r0, idx, G, B, spec, cids, seed, _o=orig, _r=r, _log=log):
        key = (sub.theta.data_ptr(), r0, G, B, tuple(int(c) for c in cids), spec.key())
        before = _r._graphs.get(key, "new")
        _o(sub, r0, idx, G, B, spec, cids, seed)
        torch.cuda.synchronize()
        after = _r._graphs.get(key)
        _log.append((r0, G, B, tuple(cids), "new" if before == "new" else ("cap" if before is None else "replay"),
                     "fail" if after is False else "ok", bool(torch.isnan(sub.theta).any())))
    r._graph_step = gs
    snaps = []
    for k in range(2):
        r.run_round(k)
        torch.cuda.synchronize()
        snaps.append(r.theta.clone())
    runs.append((snaps, log))
    if graphs:
        for e in log:
            print(e)
for k in range(2):
    a, b = runs[0][0][k], runs[1][0][k]
    print("round", k, "nan eager", bool(torch.isnan(a).any()), "nan graph", bool(torch.isnan(b).any()),
          "maxdiff", float((a - b).abs().nan_to_num(9).max()))
