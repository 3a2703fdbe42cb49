"""Training-log / statistics parity of the client-batched runners with the reference APIs (verdict r3 item 4).

* the runner emits the reference's per-client lines (``Training Client CM(r): c``, ``Client Index = c\\tEpoch: e\\t
  Loss: l`` per epoch, ``communication parameters for search n``; ``sailentgrads/my_model_trainer.py:234``,
  ``sailentgrads/client.py:101``) in the same shapes and counts as the eager SailentGradsAPI;
* the logged epoch loss is the mean of that epoch's per-batch losses (device accumulation, no per-step sync);
* ``sum_comm_params`` = sum over rounds and sampled clients of nnz(w_global) + nnz(local model) over every state
  entry (``count_communication_params``), and ``sum_training_flops`` matches the eager API exactly;
* ``record_information`` round-trips stat_info through JSON + npz (no pickle) into a created directory;
* ``avg_inference_flops`` of the runner (per-layer coefficients x non-zeros) equals the reference's forward-hook
  counter on the same masked weights (SubAvg) and on w_global (Ditto).
"""
import copy
import logging
import re

import numpy as np
import torch
import torch.nn as nn

from test_cpu_fl import Tiny3DNoDrop, _args  # noqa: F401  (shared fixtures)


class _Capture(logging.Handler):
    def __init__(self):
        super().__init__()
        self.lines = []

    def emit(self, record):
        self.lines.append(record.getMessage())


def _logger(name):
    lg = logging.getLogger(name)
    lg.handlers[:] = []
    lg.propagate = False
    lg.setLevel(logging.INFO)
    h = _Capture()
    lg.addHandler(h)
    return lg, h


def _cohort(clients=2, n_tr=12, n_te=4, seed=11):
    g = torch.Generator().manual_seed(seed)
    N = clients * (n_tr + n_te)
    vols = torch.randint(0, 256, (N, 13, 13, 13), dtype=torch.uint8, generator=g)
    labels = (torch.rand(N, generator=g) < 0.4).float()
    per = n_tr + n_te
    train = {c: np.arange(c * per, c * per + n_tr) for c in range(clients)}
    test = {c: np.arange(c * per + n_tr, (c + 1) * per) for c in range(clients)}
    return vols, labels, train, test


KINDS = {"train": re.compile(r"^@@@@@@@@@@@@@@@@ Training Client CM\((-?\d+)\): (\d+)$"),
         "loss": re.compile(r"^Client Index = (\d+)\tEpoch: (\d+)\tLoss: (-?[0-9.]+)$"),
         "comm": re.compile(r"^communication parameters for search (\d+)$")}


def _kinds(lines):
    out = {k: [] for k in KINDS}
    for ln in lines:
        for k, rx in KINDS.items():
            m = rx.match(ln)
            if m:
                out[k].append(m.groups())
    return out


def test_runner_training_log_and_comm_accounting_match_reference_semantics():
    from neuroimagedisttraining_amd.algorithms.salientgrads import SailentGradsAPI
    from neuroimagedisttraining_amd.algorithms.trainers import VolumeTrainer
    from neuroimagedisttraining_amd.data.abcd import _assemble
    from neuroimagedisttraining_amd.data.volumes import VolumeStore
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, TorchEngine
    from neuroimagedisttraining_amd.parallel import runtime as rt
    clients, B, rounds, epochs = 2, 4, 2, 2
    vols, labels, train, test = _cohort(clients)
    torch.manual_seed(3)
    model = Tiny3DNoDrop()

    # eager reference-semantics API
    lg_e, cap_e = _logger("nidt.test.eager")
    store = VolumeStore(vols, labels, torch.zeros(len(labels)))
    ds = _assemble(store, train, test, B, seed=5)
    args = _args(client_num_in_total=clients, client_num_per_round=clients, batch_size=B, comm_round=rounds,
                 epochs=epochs, seed=5)
    api = SailentGradsAPI(ds, torch.device("cpu"), args, VolumeTrainer(copy.deepcopy(model), args, lg_e), lg_e)
    api.train()
    ke = _kinds(cap_e.lines)

    # client-batched runner (CPU twin engine), with per-step losses recorded for the check
    lg_r, cap_r = _logger("nidt.test.runner")
    splits = [ClientSplit(train[c], test[c]) for c in range(clients)]
    eng = TorchEngine(copy.deepcopy(model), vols, labels, "cpu")
    steps = []
    orig = eng.train_step

    def spy(theta, bufs, grads, idx, G, B_, *a, **kw):
        out = orig(theta, bufs, grads, idx, G, B_, *a, **kw)
        steps.append((kw.get("cids"), out.detach().clone()))
        return out
    eng.train_step = spy
    info = rt.DistInfo(0, 1, 0, torch.device("cpu"), "none")
    cfg = FLConfig(comm_round=rounds, epochs=epochs, batch_size=B, dense_ratio=0.5, seed=5)
    r = FLRunner(eng, splits, cfg, info, copy.deepcopy(model), logger=lg_r)
    r.generate_global_mask_snip()
    steps.clear()
    expect_comm = 0
    for k in range(rounds):
        down = int(torch.count_nonzero(r.w_global) + torch.count_nonzero(r.b_global))
        r.run_round(k)
        nz = [int(torch.count_nonzero(r.theta[j, :r.P]) + torch.count_nonzero(r.bufs[j, :r.Q])) for j in range(r.C)]
        expect_comm += clients * down + sum(nz)
    r.finish()
    kr = _kinds(cap_r.lines)

    # the same line kinds and counts as the eager API: per round and client one header, `epochs` loss lines, one comm
    for kind, n in (("train", rounds * clients), ("loss", rounds * clients * epochs), ("comm", rounds * clients)):
        assert len(kr[kind]) == n, (kind, len(kr[kind]), cap_r.lines[:12])
        assert len(ke[kind]) == n, (kind, len(ke[kind]))
    assert sorted({int(c) for c, _, _ in kr["loss"]}) == sorted({int(c) for c, _, _ in ke["loss"]})
    # statistics: exact flop count (epochs x samples) like the eager API; comm = downlink + uplink non-zeros
    assert r.stat_info["sum_training_flops"] == api.stat_info["sum_training_flops"]
    assert r.stat_info["sum_comm_params"] == expect_comm
    # the logged epoch loss = mean of that epoch's per-batch losses (per client: ceil(12 / 4) = 3 steps per epoch)
    per_client = {c: [] for c in range(clients)}
    for cids, out in steps:
        for j, c in enumerate(cids):
            per_client[int(c)].append(float(out[j]))
    nb = -(-len(train[0]) // B)
    logged = {}
    for c, e, l in kr["loss"]:
        logged.setdefault(int(c), []).append(float(l))
    for c in range(clients):
        want = [float(np.mean(per_client[c][i * nb:(i + 1) * nb])) for i in range(rounds * epochs)]
        assert np.allclose(logged[c], want, atol=2e-6), (c, logged[c], want)
    # eager comm counts are of the same order (its SNIP mask differs only by ties, its batches by shuffling)
    assert abs(api.stat_info["sum_comm_params"] - r.stat_info["sum_comm_params"]) < 0.05 * expect_comm


def test_record_information_json_npz_round_trip(tmp_path):
    from neuroimagedisttraining_amd.utils.records import load_information, record_information
    st = {"sum_comm_params": 123, "global_test_acc": [0.5, 0.75], "avg_inference_flops": 1.5e9,
          "mask_dis_matrix": [[0.0, 2.0], [2.0, 0.0]], "final_masks": torch.ones(3, 5000, dtype=torch.bool),
          "label_num": {"0": 4, "1": 6}, "np": np.arange(6)}
    path = record_information(st, str(tmp_path / "results"), "cifar10", "SubAVG-test")
    assert path.endswith("results/cifar10/SubAVG-test.json")
    back = load_information(path)
    assert back["sum_comm_params"] == 123 and back["global_test_acc"] == [0.5, 0.75]
    assert back["mask_dis_matrix"] == [[0.0, 2.0], [2.0, 0.0]] and back["np"] == list(range(6))
    assert isinstance(back["final_masks"], np.ndarray) and back["final_masks"].shape == (3, 5000)
    assert back["final_masks"].all()


class _Tiny3D(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv3d(1, 6, 3, 2)
        self.conv2 = nn.Conv3d(6, 8, 3, bias=False)
        self.fc = nn.Linear(8, 10)

    def forward(self, x):
        x = torch.relu(self.conv2(torch.relu(self.conv1(x))))
        return self.fc(x.amax((2, 3, 4)))


def test_avg_inference_flops_runner_equals_reference_counter():
    from neuroimagedisttraining_amd.engine import masks as MK
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    from neuroimagedisttraining_amd.utils.flops import count_inference_flops
    torch.manual_seed(0)
    model = _Tiny3D()
    N = 3
    x = torch.rand(N * 4, 13, 13, 13)
    y = torch.randint(0, 10, (N * 4,)).float()
    splits = [ClientSplit(np.arange(4 * c, 4 * c + 3), np.arange(4 * c + 3, 4 * c + 4)) for c in range(N)]
    info = rt.DistInfo(0, 1, 0, torch.device("cpu"), "none")
    cfg = FLConfig(comm_round=1, epochs=1, batch_size=2, seed=1)
    eng = TorchEngine(copy.deepcopy(model), x, y, "cpu", loss="ce")
    r = make_runner("subavg", eng, splits, cfg, info, copy.deepcopy(model))
    # personal masks: random sparsity per client
    g = torch.Generator().manual_seed(4)
    masks = (torch.rand(N, r.P, generator=g) < torch.tensor([0.9, 0.5, 0.2]).view(N, 1)).float()
    r.mbits = MK.pack_bits(masks)
    got = r.record_avg_inference_flops(r.mbits)
    ref = []
    for c in range(N):
        m = copy.deepcopy(model)
        with torch.no_grad():
            flat = r.w_global * masks[c]
            for i, n in enumerate(eng.players.names):
                o, k = eng.players.offsets[i], eng.players.numel(i)
                dict(m.named_parameters())[n].copy_(flat[o:o + k].view(eng.players.shapes[i]))
        ref.append(count_inference_flops(m, input_shape=(1, 13, 13, 13)))
    assert abs(got - float(np.mean(ref))) <= 1e-6 * got, (got, np.mean(ref))
    # Ditto: every client runs w_global
    d = make_runner("ditto", TorchEngine(copy.deepcopy(model), x, y, "cpu", loss="ce"), splits, cfg, info,
                    copy.deepcopy(model))
    want = count_inference_flops(copy.deepcopy(model), input_shape=(1, 13, 13, 13))
    assert abs(d.record_avg_inference_flops() - want) < 1e-3
