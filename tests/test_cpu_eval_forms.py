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
