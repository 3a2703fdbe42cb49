"""CPU unit tests: partitioners, robust aggregation, messages/backends, topologies, secure aggregation, FLOPs."""
import json

import time

import numpy as np
import pytest
import torch

from neuroimagedisttraining_amd.core import partition as P
from neuroimagedisttraining_amd.core import robustness as RB
from neuroimagedisttraining_amd.comm import (InProcCommManager, Message, ServerManager, ClientManager,
                                             SymmetricTopologyManager, AsymmetricTopologyManager, mixing_matrix)
from neuroimagedisttraining_amd.algorithms import turboaggregate as TA
from neuroimagedisttraining_amd.algorithms import sparse as SP


def _labels(n=2000, c=10, seed=0):
    return np.random.RandomState(seed).randint(0, c, n)


@pytest.mark.parametrize("method", ["dir", "n_cls", "my_part", "hetero"])
def test_partitioners_cover_and_quota(method):
    y = _labels()
    rs = np.random.RandomState(1)
    m = P.partition_labels(method, y, 10, 0.3 if method != "n_cls" else 2, n_cls=10, rng=rs)
    assert len(m) == 10
    tot = sum(len(v) for v in m.values())
    if method in ("dir", "n_cls", "my_part"):
        assert all(len(v) == 200 for v in m.values())  # equal quotas (lognormal sigma=0)
    if method in ("dir", "hetero"):
        allix = np.concatenate([m[i] for i in range(10)])
        assert len(np.unique(allix)) == len(allix), "no sample reuse"
    assert tot >= 1900


def test_dir_partition_is_non_iid():
    y = _labels(5000)
    m = P.partition_dir(y, 20, 0.1, n_cls=10, rng=np.random.RandomState(3))
    ent = []
    for ix in m.values():
        h = np.bincount(y[ix], minlength=10) / len(ix)
        ent.append(-(h[h > 0] * np.log(h[h > 0])).sum())
    assert np.mean(ent) < 0.8 * np.log(10)


def test_per_client_test_sets_follow_reference_sizes():
    """cifar10/data_loader.py:226-236: tmp_tst_num = ceil(|test| / client_number); class c gets
    ceil(count_c / total * tmp_tst_num) samples, drawn from the test images of class c."""
    y = _labels(5000)
    yte = _labels(10000)[::-1].copy()
    m = P.partition_dir(y, 100, 0.3, n_cls=10, rng=np.random.RandomState(3))
    te = P.per_client_test_indices(y, yte, m, n_cls=10, rng=np.random.RandomState(4))
    for c, ix in m.items():
        h = np.bincount(y[ix], minlength=10)
        want = sum(int(np.ceil(h[k] / h.sum() * 100)) for k in range(10))
        assert len(te[c]) == want and 100 <= want <= 110
        assert np.array_equal(np.bincount(yte[te[c]], minlength=10) > 0, h > 0)
        assert len(set(te[c].tolist())) == len(te[c])


def test_homo_and_site_partition():
    m = P.partition_homo(103, 4, rng=np.random.RandomState(0))
    assert sorted(np.concatenate(list(m.values())).tolist()) == list(range(103))
    site = np.array([0] * 50 + [1] * 30 + [2] * 20)
    tr, te, _ = P.partition_by_site(site, max_clients=3)
    assert len(tr[0]) == 40 and len(te[0]) == 10 and len(tr[2]) == 16


def test_robust_aggregators():
    torch.manual_seed(0)
    good = [{"w": torch.randn(5) * 0.01 + 1.0} for _ in range(6)]
    bad = [{"w": torch.full((5,), 100.0)}]
    wl = [(1, s) for s in good + bad]
    med = RB.robust_aggregate("median", wl)
    assert torch.allclose(med["w"], torch.ones(5), atol=0.05)
    kr = RB.robust_aggregate("krum", wl, f=1)
    assert float(kr["w"].max()) < 2
    tm = RB.robust_aggregate("trimmed_mean", wl, trim_ratio=0.2)
    assert float(tm["w"].max()) < 2
    avg = RB.robust_aggregate("fedavg", wl) if hasattr(RB, "robust_aggregate") else None
    if avg is not None:
        assert float(avg["w"].mean()) > 10


def test_message_json_roundtrip_and_inproc_dispatch():
    m = Message(3, 0, 1)
    m.add_params(Message.MSG_ARG_KEY_MODEL_PARAMS, {"a.weight": torch.arange(6.).view(2, 3), "n": 4})
    s = m.to_json()
    m2 = Message()
    m2.init_from_json_string(s)
    assert m2.get_type() == 3 and m2.get_receiver_id() == 1
    assert torch.equal(m2.get(Message.MSG_ARG_KEY_MODEL_PARAMS)["a.weight"], torch.arange(6.).view(2, 3))

    got = []

    class S(ServerManager):
        def register_message_receive_handlers(self):
            self.register_message_receive_handler(7, lambda msg: got.append(msg.get("x")))

    srv = S(None, rank=0, size=2, backend="INPROC", world="t1")
    srv.register_message_receive_handlers()
    cli = ClientManager(None, rank=1, size=2, backend="INPROC", world="t1")
    msg = Message(7, 1, 0)
    msg.add_params("x", 42)
    cli.send_message(msg)
    assert srv.com_manager.poll_once(timeout=1.0)
    assert got == [42]


def test_grpc_backend_roundtrip():
    pytest.importorskip("grpc")
    from neuroimagedisttraining_amd.comm import GRPCCommManager
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    base = s.getsockname()[1]
    s.close()
    a = GRPCCommManager("127.0.0.1", None, client_id=0, base_port=base)
    b = GRPCCommManager("127.0.0.1", None, client_id=1, base_port=base)
    try:
        m = Message(5, 1, 0)
        m.add_params("w", torch.ones(3))
        b.send_message(m)
        r = a.q.get(timeout=10)
        assert r.get_type() == 5 and torch.equal(r.get("w"), torch.ones(3))
    finally:
        a.stop_receive_message()
        b.stop_receive_message()


def test_mqtt_backend_roundtrip_with_builtin_broker():
    """Reference topic scheme (server 0 <-> clients 1..N) over the built-in MQTT 3.1.1 client and broker."""
    from neuroimagedisttraining_amd.comm import MqttCommManager
    from neuroimagedisttraining_amd.comm.mqtt import MqttBroker, topic_matches
    assert topic_matches("fedml/+/x", "fedml/3/x") and topic_matches("a/#", "a/b/c") and not topic_matches("a", "a/b")
    broker = MqttBroker()
    srv = MqttCommManager("127.0.0.1", broker.port, client_id=0, client_num=2)
    c1 = MqttCommManager("127.0.0.1", broker.port, client_id=1, client_num=2)
    c2 = MqttCommManager("127.0.0.1", broker.port, client_id=2, client_num=2)
    try:
        for c in (c1, c2):
            m = Message(3, c.client_id, 0)
            m.add_params("w", torch.full((4,), float(c.client_id)))
            c.send_message(m)
        got = sorted((srv.q.get(timeout=10) for _ in range(2)), key=lambda r: r.get_sender_id())
        assert [r.get_sender_id() for r in got] == [1, 2]
        assert torch.equal(got[1].get("w"), torch.full((4,), 2.0))
        m = Message(4, 0, 2)
        m.add_params("round", 7)
        srv.send_message(m)
        r = c2.q.get(timeout=10)
        assert r.get_type() == 4 and r.get("round") == 7 and c1.q.empty()
        seen = []

        class Obs:
            def receive_message(self, t, p):
                seen.append((t, p.get("round")))
        c2.add_observer(Obs())
        srv.send_message(m)
        assert c2.poll_once(timeout=10.0) and seen == [(4, 7)]
    finally:
        for c in (srv, c1, c2):
            c.stop_receive_message()
        broker.close()


def test_topologies_row_stochastic():
    t = SymmetricTopologyManager(8, 4)
    W = t.generate_topology()
    assert np.allclose(W.sum(1), 1) and np.allclose(W, W.T)
    assert t.get_in_neighbor_idx_list(0) == [1, 2, 6, 7]
    a = AsymmetricTopologyManager(8, 2, 2, seed=0)
    W2 = a.generate_topology()
    assert np.allclose(W2.sum(1), 1)
    for kind in ("ring", "full", "random"):
        M = mixing_matrix(kind, 6, round_idx=3, neighbors=2)
        assert np.allclose(M.sum(1), 1)


def test_mpc_bgw_lcc_additive():
    p = TA.P_DEFAULT
    rs = np.random.RandomState(0)
    X = rs.randint(0, 1000, size=(2, 5))
    sh = TA.BGW_encoding(X, 5, 2, p, rs)
    rec = TA.BGW_decoding(sh[[0, 2, 4]], [0, 2, 4], p)
    assert np.array_equal(rec, X % p)
    X2 = rs.randint(0, 1000, size=(4, 3))
    enc = TA.LCC_encoding(X2, N=6, K=2, T=1, p=p, rng=rs)
    dec = TA.LCC_decoding(enc, 1, 6, 2, 1, list(range(6)), p)
    assert np.array_equal(np.concatenate(list(dec), 0), X2 % p)
    # shares equal the reference's: worker j holds the Lagrange interpolant through the blocks at the centred
    # points beta = {-1, 0, 1} evaluated at the centred alpha_j = j - 3 (mpc_function.py:121-125)
    beta, alpha = [-1, 0, 1], [j - 3 for j in range(6)]
    rs2 = np.random.RandomState(5)
    enc = TA.LCC_encoding(X2, N=6, K=2, T=1, p=p, rng=rs2)
    rnd = np.random.RandomState(5).randint(p, size=(2, 3))
    blocks = [X2[:2] % p, X2[2:] % p, rnd]
    for j, a in enumerate(alpha):
        want = np.zeros((2, 3), dtype=np.int64)
        for k, b in enumerate(beta):
            num = den = 1
            for o in beta:
                if o != b:
                    num = num * ((a - o) % p) % p
                    den = den * ((b - o) % p) % p
            coef = num * pow(den, p - 2, p) % p
            want = (want + coef * blocks[k]) % p
        assert np.array_equal(enc[j], want), j
    # odd K: the reference-compatible decoder's targets differ from the encoder's points (it warns); the matching
    # decoder recovers the blocks for any K, T
    X3 = rs.randint(0, 1000, size=(3, 4))
    enc = TA.LCC_encoding(X3, N=7, K=3, T=1, p=p, rng=rs)
    with pytest.warns(UserWarning):
        TA.LCC_decoding(enc, 1, 7, 3, 1, list(range(7)), p)
    dec = TA.LCC_decode_blocks(enc[[6, 1, 4, 0]], 1, 7, 3, 1, [6, 1, 4, 0], p)  # any K + T workers
    assert np.array_equal(np.concatenate(list(dec), 0), X3 % p)
    ss = TA.Gen_Additive_SS(7, 4, p, rs)
    assert np.all(ss.sum(0) % p == 0)
    assert TA.modular_inv(3, p) * 3 % p == 1


def test_secure_aggregation_equals_fedavg_with_dropout():
    rs = np.random.RandomState(1)
    n = 5
    vecs = [rs.randn(100) for _ in range(n)]
    wts = rs.dirichlet(np.ones(n))
    tr = TA.TurboAggregateTrainer(n, seed=3)
    ups = {i: tr.client_upload(i, vecs[i], wts[i]) for i in range(n)}
    agg = tr.server_aggregate(ups)
    ref = sum(w * v for w, v in zip(wts, vecs))
    assert np.allclose(agg, ref, atol=1e-3)
    ups.pop(2)
    agg2 = tr.server_aggregate(ups, dropped=[2])
    ref2 = sum(wts[i] * vecs[i] for i in range(n) if i != 2)
    assert np.allclose(agg2, ref2, atol=1e-3)
    # reference-style clients with the isdrop flag (TA_client.py:20-26)
    from fedml_api.standalone.turboaggregate.TA_client import TA_Client
    clients = [TA_Client(None, None, 10, None, "cpu", i) for i in range(n)]
    clients[4].set_dropout(True)
    agg3 = TA.secure_round(tr, clients, vecs, wts)
    assert np.allclose(agg3, sum(wts[i] * vecs[i] for i in range(4)), atol=1e-3)


def test_sparse_mask_ops():
    torch.manual_seed(0)
    params = {"a": torch.randn(64, 32), "b": torch.randn(10, 64)}
    sp = SP.erk_sparsities(params, 0.5)
    masks = SP.init_masks(params, sp)
    dens = sum(float(m.sum()) for m in masks.values()) / sum(m.numel() for m in masks.values())
    assert abs(dens - 0.5) < 0.02
    new, nrm = SP.fire_mask(masks, params, 0, 0.5, 10)
    assert all(float(new[k].sum()) == float(masks[k].sum()) - nrm[k] for k in masks)
    grown = SP.regrow_mask(new, nrm, {k: torch.randn_like(v) for k, v in params.items()})
    assert all(float(grown[k].sum()) == float(masks[k].sum()) for k in masks)
    d, tot = SP.hamming_distance(masks, grown)
    assert 0 < d < tot
    w = {"a.weight": torch.randn(100)}
    m = {"a.weight": torch.ones(100)}
    m2 = SP.fake_prune(0.3, w, m)
    assert abs(float(m2["a.weight"].sum()) - 70) <= 1
    srv = {"a.weight": torch.zeros(100)}
    agg = SP.masked_average(srv, [(m, {"a.weight": torch.ones(100)}), (m2, {"a.weight": 3 * torch.ones(100)})])
    assert torch.all((agg["a.weight"] == 2) | (agg["a.weight"] == 1) | (agg["a.weight"] == 4))


def test_flops_counts_conv3d():
    from neuroimagedisttraining_amd.models import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.utils.flops import count_inference_flops
    m = AlexNet3D_Dropout(num_classes=1, in_shape=(69, 69, 69))
    f = count_inference_flops(m, input_shape=(1, 69, 69, 69), full=True)
    assert f > 1e8


@pytest.mark.parametrize("algo,expected", [
    ("sailentgrads", "SailentGrads-ABCD-dir0.3-mdl3DCNNcustomizedlowbatch-csv0-ERK_init-same_init-DST-cm200-total_clnt4"
                     "-neighbor4-dr0.5-active1.0-seed1024-lr0.01-batchsize16-iteration1-stratifiedFalse"),
    ("fedavg", "fedavg-dir0.3-mdl3DCNN-batchsize16-cm200-total_clnt4-neighbor3-seed0-lr0.001"),
    ("dispfl", "DisPFL-ABCD-dir0.3-mdl3DCNN-csrandom-ERK_init-same_init-DST-cm10-total_clnt21-neighbor2-dr0.5"
               "-batchsize16-active1.0-lr0.001-seed1024"),
    ("subavg", "SubAVGdir0.3-mdlresnet18-batchsize128-cm1000-total_clnt100-neighbor10-seed0-dr0.5"),
    ("ditto", "ditto-dir0.3-mdlresnet18-ge2-le3-batchsize128-lambda0.5-cm1000-total_clnt100-neighbor10-seed0"),
    ("dpsgd", "dpsgd-cifar10-dir0.3-mdlresnet18-csring-batchsize128-cm50-total_clnt100-neighbor10-seed0-typeepoch"),
    ("fedfomo", "fedfomo-dir0.3-mdlresnet18-cm1000-total_clnt100-batchsize128-neighbor10-seed0"),
    ("local", "local-dir0.3-cm10-total_clnt100-neighbor100-seed1024"),
])
def test_cli_identity_strings_match_reference(algo, expected):
    """The identity string is the log file name (LOG/<dataset>/<identity>.log): byte-compatible with the
    reference entry points' defaults (main_<algo>.py)."""
    import argparse
    from neuroimagedisttraining_amd import cli
    args = cli.add_args(argparse.ArgumentParser(), algo).parse_args([])
    assert cli.identity(args, algo) == expected


def test_alexnet3d_state_dict_keys_match_reference():
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    keys = list(AlexNet3D_Dropout(num_classes=1).state_dict().keys())
    exp = []
    for c, b in zip((0, 4, 8, 11, 14), (1, 5, 9, 12, 15)):
        exp += ["features.%d.weight" % c, "features.%d.bias" % c]
        exp += ["features.%d.%s" % (b, k) for k in ("weight", "bias", "running_mean", "running_var",
                                                     "num_batches_tracked")]
    exp += ["classifier.1.weight", "classifier.1.bias", "classifier.4.weight", "classifier.4.bias"]
    assert keys == exp
    n = sum(p.numel() for p in AlexNet3D_Dropout(num_classes=1).parameters())
    assert n == 2570241  # SURVEY.md §6 workload constants


def test_meta_resnet_generates_weights_for_any_gene():
    import random
    from neuroimagedisttraining_amd.models.meta_resnet import MetaResNet20
    torch.manual_seed(0)
    m = MetaResNet20(num_classes=10, blocks=2)
    x = torch.randn(3, 3, 32, 32)
    rng = random.Random(1)
    for gene in (m.max_gene(), m.random_gene(rng), [0] * m.gene_length()):
        out = m(x, gene)
        assert out.shape == (3, 10)
    out.sum().backward()
    assert m.stem.gen.fc2.weight.grad is not None and float(m.stem.gen.fc2.weight.grad.abs().sum()) > 0


def test_model_zoo_forward_shapes():
    """Every reference model family builds and runs forward + backward at its dataset's input shape."""
    import importlib
    A3 = importlib.import_module("neuroimagedisttraining_amd.models.alexnet3d")
    NR = importlib.import_module("neuroimagedisttraining_amd.models.norm_resnets")
    R3 = importlib.import_module("neuroimagedisttraining_amd.models.resnet3d")
    Z = importlib.import_module("neuroimagedisttraining_amd.models.zoo2d")
    torch.manual_seed(0)
    x32 = torch.randn(2, 3, 32, 32)
    cases = [
        (Z.customized_resnet18(class_num=10), x32, (2, 10)),
        (Z.vgg11(10), x32, (2, 10)),
        (Z.vgg16(10), x32, (2, 10)),
        (Z.LeNet5_cifar(), x32, (2, 10)),
        (Z.cnn_cifar10(), x32, (2, 10)),
        (Z.cnn_cifar100(), x32, (2, 100)),
        (Z.cnn_cifar10_meta(), x32, (2, 10)),
        (Z.CNN_DropOut(), torch.randn(2, 1, 28, 28), (2, 10)),
        (Z.CNN_OriginalFedAvg(), torch.randn(2, 1, 28, 28), (2, 10)),
        (Z.LeNet5(), torch.randn(2, 1, 28, 28), (2, 10)),
        (NR.resnet18_gn(num_classes=10), torch.randn(2, 3, 64, 64), (2, 10)),
        (NR.resnet29_ip(num_classes=10), x32, (2, 10)),
        (R3.resnet3d_18(num_classes=1, width=8), torch.randn(2, 1, 32, 32, 32), (2, 1)),
        (A3.AlexNet3D_Dropout(num_classes=1, in_shape=(80, 96, 80)), torch.randn(2, 1, 80, 96, 80), (2, 1)),
    ]
    for model, x, shape in cases:
        out = model(x)
        out = out[0] if isinstance(out, (list, tuple)) else out
        assert tuple(out.shape) == shape, (type(model).__name__, tuple(out.shape))
        out.float().sum().backward()
    # SyncBN without a process group behaves as BatchNorm
    bn = NR.SynchronizedBatchNorm3d(4)
    y = bn(torch.randn(3, 4, 5, 5, 5))
    assert y.shape == (3, 4, 5, 5, 5) and abs(float(y.mean())) < 1e-5


def test_heartbeat_failure_detector_reports_silent_rank():
    """Store-based heartbeats: a rank that stops publishing is reported dead after the timeout; live ranks are not."""
    import socket
    import torch.distributed as dist
    from neuroimagedisttraining_amd.comm.failure import HeartbeatMonitor, PeerFailure
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    master = dist.TCPStore("127.0.0.1", port, 3, True, wait_for_workers=False)
    stores = [master] + [dist.TCPStore("127.0.0.1", port, 3, False) for _ in range(2)]
    mons = [HeartbeatMonitor(stores[r], r, 3, interval_s=0.05, timeout_s=0.6) for r in range(3)]
    try:
        assert mons[0].wait_all_alive(5.0)
        assert mons[0].dead_ranks() == [] and mons[1].dead_ranks() == []
        time.sleep(0.3)
        assert mons[0].dead_ranks() == []
        mons[2].stop()                      # rank 2 "dies"
        t_end = time.time() + 5
        while time.time() < t_end and not (mons[0].dead_ranks() == [2] and mons[1].dead_ranks() == [2]):
            time.sleep(0.1)  # each observer times a silent peer from its own last observed change
        assert mons[0].dead_ranks() == [2] and mons[1].dead_ranks() == [2]
        with pytest.raises(PeerFailure) as ei:
            mons[1].check_or_raise()
        assert ei.value.dead == [2]
    finally:
        for m in mons:
            m.stop()


def test_flops_match_reference_multiply_adds_by_hand():
    """The reference counter with its default ``multiply_adds=True`` (``main_flops_counter.py:58-80``): a conv is
    ``(2 * nnz(W) + Cout) * H_out * W_out`` with a bias, a linear layer ``2 * nnz(W) + nnz(b)`` at batch 1; computed
    here by hand for a small CIFAR-shape net with some zeroed weights and bias entries."""
    import torch.nn as nn
    from neuroimagedisttraining_amd.utils.flops import count_inference_flops
    from neuroimagedisttraining_amd.utils.records import flop_coefficients

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 4, 3, padding=1)             # 32x32 out
            self.conv2 = nn.Conv2d(4, 2, 3, stride=2, bias=False)  # 15x15 out
            self.fc = nn.Linear(2 * 15 * 15, 10)

        def forward(self, x):
            return self.fc(torch.flatten(self.conv2(self.conv(x)), 1))

    torch.manual_seed(0)
    m = Net()
    with torch.no_grad():
        m.conv.weight[0].zero_()     # 27 zeros
        m.fc.weight[:, :7].zero_()   # 70 zeros
        m.fc.bias[:3].zero_()        # 3 zero biases
    nnz_c1 = 4 * 27 - 27
    nnz_c2 = 2 * 36
    nnz_fc = 10 * 450 - 70
    want = (2 * nnz_c1 + 4) * 32 * 32 + (2 * nnz_c2) * 15 * 15 + (2 * nnz_fc + 7)
    assert count_inference_flops(m, input_shape=(3, 32, 32)) == want
    full = (2 * 108 + 4) * 32 * 32 + (2 * 72) * 15 * 15 + (2 * 4500 + 10)
    assert count_inference_flops(m, input_shape=(3, 32, 32), full=True) == full
    coef = flop_coefficients(m, input_shape=(3, 32, 32))
    sd = dict(m.named_parameters())
    got = sum(a * int(torch.count_nonzero(sd[n])) + b for n, (a, b) in coef.items())
    assert got == want


def test_alexnet_step_mode_follows_launch_size(monkeypatch):
    """[EAGER-BRANCH]: row sets of <= 32 clients (the per-GPU loads of the 2/4/8-GPU bench) train in eager steps with
    the weight-gradient branch, larger ones in captured steps; FLConfig.hip_graphs still overrides in the runner."""
    from neuroimagedisttraining_amd.engine import alexnet_hip as AX
    from neuroimagedisttraining_amd.engine.executor import HipEngine
    assert [HipEngine.graphs_default_for(k) for k in (1, 8, 16, 32, 33, 64)] == [False] * 4 + [True] * 2
    monkeypatch.setattr(AX, "_WS_ENV", None)
    monkeypatch.setattr(AX.torch.cuda, "is_current_stream_capturing", lambda: False)
    assert AX._wgrad_branch(8) and not AX._wgrad_branch(64)
    monkeypatch.setattr(AX.torch.cuda, "is_current_stream_capturing", lambda: True)
    assert not AX._wgrad_branch(8)  # a captured step never forks the branch
    monkeypatch.setattr(AX, "_WS_ENV", "0")
    assert not AX._wgrad_branch(8)
    monkeypatch.setattr(AX, "_WS_ENV", "1")
    assert AX._wgrad_branch(64)
    monkeypatch.setattr(AX, "_WG2_EARLY_ENV", None)
    assert AX._wg2_early(8) and not AX._wg2_early(16)
    monkeypatch.setattr(AX, "_WG2_EARLY_ENV", "0")
    assert not AX._wg2_early(8)
