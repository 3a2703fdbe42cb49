"""The two evaluation forms of the runner give the same per-client metrics: personal rows read in place + the global
model from min(C, 64) reused copies (default) vs one grouped pass over a 2C-row copy (``NIDT_EVAL_STAGE=1``), with
more clients than reused copies so the row mapping j mod K is exercised."""
import copy

import numpy as np
import torch

from test_cpu_records import _Tiny3D


def test_eval_forms_agree(monkeypatch):
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    N = 70  # > 64 reused global copies
    x = torch.rand(N * 3, 13, 13, 13)
    y = torch.randint(0, 10, (N * 3,)).float()
    splits = [ClientSplit(np.arange(3 * c, 3 * c + 2), np.arange(3 * c + 2, 3 * c + 3)) for c in range(N)]
    model = _Tiny3D()
    cfg = FLConfig(comm_round=1, epochs=1, batch_size=2, seed=1, frequency_of_the_test=0, test_batch=8)
    r = make_runner("fedavg", TorchEngine(copy.deepcopy(model), x, y, "cpu", loss="ce"), splits, cfg,
                    rt.DistInfo(0, 1, 0, torch.device("cpu"), "none"), copy.deepcopy(model))
    r.run_round(0)
    with torch.no_grad():  # personal rows different from the global model and from each other
        r.theta[:, :r.P] += 0.01 * torch.randn_like(r.theta[:, :r.P])
    monkeypatch.delenv("NIDT_EVAL_STAGE", raising=False)
    g0, p0 = r._eval_global_and_personal()
    monkeypatch.setenv("NIDT_EVAL_STAGE", "1")
    g1, p1 = r._eval_global_and_personal()
    assert np.allclose(g0, g1, rtol=1e-6, atol=1e-6) and np.allclose(p0, p1, rtol=1e-6, atol=1e-6)
    assert not np.allclose(g0[:, 1], p0[:, 1])  # the two model sets really differ


def _runner():
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    N = 5
    x = torch.rand(N * 4, 13, 13, 13)
    y = torch.randint(0, 10, (N * 4,)).float()
    splits = [ClientSplit(np.arange(4 * c, 4 * c + 3), np.arange(4 * c + 3, 4 * c + 4)) for c in range(N)]
    model = _Tiny3D()
    cfg = FLConfig(comm_round=3, epochs=1, batch_size=2, seed=1, frequency_of_the_test=1, test_batch=8,
                   final_round=False)
    return make_runner("fedavg", TorchEngine(copy.deepcopy(model), x, y, "cpu", loss="ce"), splits, cfg,
                       rt.DistInfo(0, 1, 0, torch.device("cpu"), "none"), copy.deepcopy(model))


def test_deferred_metrics_equal_immediate(monkeypatch):
    """Timed GPU runs read a round's evaluation one round later (device result, pinned copy, event); the deferred
    bookkeeping (forced on the CPU here) yields the same ordered stat_info lists and run_round results as reading
    each round at once, and an unread round is folded in by any read of the lists."""
    import math
    outs = {}
    for mode in ("0", "force"):
        monkeypatch.setenv("NIDT_DEFER_METRICS", mode)
        r = _runner()
        res = [r.run_round(k) for k in range(3)]
        assert (len(r._pending_metrics) == 1) == (mode == "force")  # the last round is still in flight
        outs[mode] = ([dict(x) for x in res], {k: list(r.stat_info[k]) for k in
                                               ("global_test_acc", "global_test_loss", "person_test_acc",
                                                "person_test_loss")})
        assert not r._pending_metrics
    a, b = outs["0"], outs["force"]
    for k, v in a[1].items():
        assert len(v) == 3 and all(math.isclose(x, y, rel_tol=1e-12) for x, y in zip(v, b[1][k])), k
    for x, y in zip(a[0], b[0]):
        assert x.keys() == y.keys() and all(math.isclose(x[k], y[k], rel_tol=1e-12) for k in x)
