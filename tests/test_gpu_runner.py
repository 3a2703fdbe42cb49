"""GPU tests of runner-level device paths: the sparse-update (top-k) FedAvg aggregation (segmented radix select,
coalesced combine) against a torch.topk oracle, and the background-written checkpoint of device rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _runner(**kw):
    import torch.nn as nn
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, TorchEngine
    from neuroimagedisttraining_amd.parallel import runtime as rt

    class Tiny(nn.Module):
        def __init__(self):
            super().__init__()
            self.features = nn.Sequential(nn.Conv3d(1, 4, 3, 2), nn.BatchNorm3d(4), nn.ReLU(), nn.Conv3d(4, 8, 3))
            self.classifier = nn.Linear(8, 1)

        def forward(self, x):
            return self.classifier(self.features(x).amax((2, 3, 4)))

    torch.manual_seed(0)
    n = 5 * 10
    vols = torch.randint(0, 256, (n, 11, 11, 11), dtype=torch.uint8, device=DEV)
    labels = torch.randint(0, 2, (n,), device=DEV).float()
    splits = [ClientSplit(np.arange(c * 10, c * 10 + 7), np.arange(c * 10 + 7, c * 10 + 10)) for c in range(5)]
    model = Tiny()
    eng = TorchEngine(model, vols, labels, DEV)
    info = rt.DistInfo(0, 1, 0, torch.device(DEV), "none")
    return FLRunner(eng, splits, FLConfig(comm_round=1, epochs=1, batch_size=4, seed=3, **kw), info, model)


def test_topk_update_aggregation_matches_torch_topk():
    r = _runner(update_topk=0.05)
    g = torch.Generator(device=DEV).manual_seed(1)
    r.theta[:, :r.P] = r.w_global + torch.randn(r.C, r.P, device=DEV, generator=g)
    sampled = [0, 2, 3, 4]
    w0 = r.w_global.clone()
    k = int(np.ceil(0.05 * r.P))
    n_tot = float(sum(r.sizes[c] for c in sampled))
    want = w0.clone()
    for c in sampled:  # the reference order of the old per-client loop
        d = r.theta[r.row_of[c], :r.P] - w0
        top = torch.topk(d.abs(), k).indices
        want.index_add_(0, top, d[top] * float(r.sizes[c] / n_tot))
    r.aggregate_topk(sampled)
    assert torch.allclose(r.w_global, want, atol=1e-6, rtol=0), float((r.w_global - want).abs().max())
    # exactly k coordinates per client moved (distinct random values: no ties)
    assert int((r.w_global != w0).sum()) <= k * len(sampled)


def test_async_checkpoint_of_device_rows_round_trips(tmp_path):
    from neuroimagedisttraining_amd.utils import checkpoint as ck
    a = _runner()
    a.theta[:, :a.P] = torch.randn(a.C, a.P, device=DEV)
    a.w_global.normal_()
    saver = ck.Checkpointer(str(tmp_path), a.info, every=1, keep_last=1, async_write=True)
    saver.save(a, 1)
    keep = a.theta.clone()
    a.theta.zero_()  # the pinned snapshot was taken on the stream before this write
    saver.save(a, 2)
    saver.close()
    b = _runner()
    assert ck.load_runner(b, str(tmp_path)) == 2
    assert torch.equal(b.theta, a.theta) and not torch.equal(b.theta, keep)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["latest", "round_2"]


def test_hip_runner_training_log_with_graphs_equals_eager():
    """AlexNet3D on the HIP engine: the per-client epoch losses the runner logs are accumulated on device inside the
    captured hipGraph steps; they equal the eager (un-captured) run's, and sum_comm_params equals the formula."""
    import logging
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes, to_hip_store
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, HipEngine
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.parallel import runtime as rt
    C, ntr, nte = 3, 6, 2
    vol, labels, sp = build_fl_volumes(list(range(C)), C, ntr, nte, torch.device(DEV), seed=3)
    x8, mom = to_hip_store(vol)
    del vol
    splits = [sp[c] for c in range(C)]
    out = {}
    for graphs in (True, False):
        lines = []

        class H(logging.Handler):
            def emit(self, rec):
                lines.append(rec.getMessage())
        lg = logging.getLogger("nidt.gpu.log.%d" % graphs)
        lg.handlers[:] = [H()]
        lg.propagate = False
        lg.setLevel(logging.INFO)
        torch.manual_seed(0)
        model = AlexNet3D_Dropout(num_classes=1)
        eng = HipEngine(model, x8, mom, labels, torch.device(DEV))
        info = rt.DistInfo(0, 1, 0, torch.device(DEV), "none")
        cfg = FLConfig(comm_round=3, epochs=2, batch_size=4, seed=3, hip_graphs=graphs, frequency_of_the_test=0)
        r = FLRunner(eng, splits, cfg, info, model, logger=lg)
        r.generate_global_mask_snip()
        comm = 0
        for k in range(3):  # round 0 captures nothing new, round 1 captures, round 2 replays
            down = int(torch.count_nonzero(r.w_global) + torch.count_nonzero(r.b_global))
            r.run_round(k)
            comm += C * down + sum(int(torch.count_nonzero(r.theta[j, :r.P]) + torch.count_nonzero(r.bufs[j, :r.Q]))
                                   for j in range(r.C))
        assert r.stat_info["sum_comm_params"] == comm
        out[graphs] = [float(ln.split("Loss: ")[1]) for ln in lines if ln.startswith("Client Index")]
    assert len(out[True]) == 3 * C * 2
    assert all(np.isfinite(out[True])) and min(out[True]) > 0
    assert np.allclose(out[True], out[False], rtol=1e-5, atol=1e-6), (out[True], out[False])
