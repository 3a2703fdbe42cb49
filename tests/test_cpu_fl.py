"""CPU end-to-end tests of the FL stack: reference-semantics algorithm APIs on small synthetic data, the
client-batched executor (TorchEngine) incl. SNIP masks and aggregation, and a 2-rank gloo run that must
reproduce the 1-rank result exactly (client sharding must not change the math)."""
import os
import types

import numpy as np
import pytest
import torch
import torch.nn as nn

from neuroimagedisttraining_amd.algorithms.trainers import ClassificationTrainer, VolumeTrainer
from neuroimagedisttraining_amd.data.images import load_partition_data, load_partition_data_synthetic_tabular
from neuroimagedisttraining_amd.models import LeNet5_cifar, LogisticRegression


def _args(**kw):
    a = dict(client_num_in_total=3, client_num_per_round=3, comm_round=2, epochs=1, batch_size=32, lr=0.05,
             lr_decay=0.998, wd=5e-4, momentum=0.0, client_optimizer="sgd", frequency_of_the_test=1, ci=0,
             dense_ratio=0.5, anneal_factor=0.5, active=1.0, cs="random", static=False, dis_gradient_check=False,
             uniform=False, different_initial=False, diff_spa=False, erk_power_scale=1.0, save_masks=False,
             each_prune_ratio=0.2, dist_thresh=1e-4, acc_thresh=0.0, lamda=0.5, local_epochs=1,
             itersnip_iteration=1, snip_mask=True, dataset="cifar10", record_mask_diff=True)
    a.update(kw)
    return types.SimpleNamespace(**a)


def test_fedavg_logistic_regression_two_clients_learns():
    from neuroimagedisttraining_amd.algorithms.fedavg import FedAvgAPI
    torch.manual_seed(0)
    ds = load_partition_data_synthetic_tabular(client_number=2, batch_size=32, n_per_client=400, dim=20, n_cls=5)
    args = _args(client_num_in_total=2, client_num_per_round=2, comm_round=15, lr=0.1, final_finetune=False)
    tr = ClassificationTrainer(LogisticRegression(20, 5), args)
    api = FedAvgAPI(ds, torch.device("cpu"), args, tr)
    api.train()
    assert api.engine_used == "eager"  # a CPU device keeps the eager loop (the HIP dispatch needs a GPU)
    acc = api.stat_info["global_test_acc"]
    assert acc[-1] > 0.5 and acc[-1] >= acc[0]


@pytest.fixture(scope="module")
def img_ds():
    return load_partition_data("cifar10", None, "dir", 0.5, 3, 32, n_train=300, n_test=150, seed=1)


@pytest.mark.parametrize("algo", ["dispfl", "subavg", "ditto", "dpsgd", "fedfomo", "local", "salientgrads", "fedavg"])
def test_algorithms_run(algo, img_ds):
    from neuroimagedisttraining_amd.algorithms import personalized as PZ
    from neuroimagedisttraining_amd.algorithms.fedavg import FedAvgAPI
    from neuroimagedisttraining_amd.algorithms.salientgrads import SailentGradsAPI
    torch.manual_seed(0)
    np.random.seed(0)
    args = _args(client_num_per_round=2 if algo in ("dispfl", "fedfomo") else 3)
    tr = ClassificationTrainer(LeNet5_cifar(10), args)
    cls = {"dispfl": PZ.DisPFLAPI, "subavg": PZ.SubAvgAPI, "ditto": PZ.DittoAPI, "dpsgd": PZ.DPSGDAPI,
           "fedfomo": PZ.FedFomoAPI, "local": PZ.LocalAPI, "salientgrads": SailentGradsAPI, "fedavg": FedAvgAPI}[algo]
    ds = img_ds
    if algo == "fedfomo":
        ds = load_partition_data("cifar10", None, "dir", 0.5, 3, 32, n_train=300, n_test=150, seed=1, with_val=True)
    api = cls(ds, torch.device("cpu"), args, tr)
    out = api.train()
    assert out is not None
    if algo == "dispfl":
        m = api.masks[0]
        dens = sum(float(v.sum()) for v in m.values()) / sum(v.numel() for v in m.values())
        assert abs(dens - 0.5) < 0.05
    if algo == "salientgrads":
        mask = api.mask
        w = api.w_global
        for k, v in mask.items():
            if v.dim() > 1:
                assert float((w[k] * (1 - v)).abs().max()) == 0.0  # masked weights stay zero


# ------------------------------------------------------------------------------------------------ executor
class Tiny3D(nn.Module):
    def __init__(self):
        super().__init__()
        self.features = nn.Sequential(nn.Conv3d(1, 4, 3, 2), nn.BatchNorm3d(4), nn.ReLU(), nn.MaxPool3d(2, 2),
                                      nn.Conv3d(4, 8, 3), nn.BatchNorm3d(8), nn.ReLU())
        self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(8, 1))

    def forward(self, x):
        return self.classifier(self.features(x).amax((2, 3, 4)))


def _runner(rank=0, world=1, clients=4, rounds=2, **cfg_kw):
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, TorchEngine
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(5)
    n_tr, n_te = 10, 4
    N = clients * (n_tr + n_te)
    vols = torch.randint(0, 256, (N, 15, 15, 15), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 2, (N,), generator=g).float()
    splits = [ClientSplit(np.arange(c * 14, c * 14 + n_tr), np.arange(c * 14 + n_tr, c * 14 + 14))
              for c in range(clients)]
    model = Tiny3D()
    eng = TorchEngine(model, vols, labels, "cpu")
    info = rt.DistInfo(rank, world, rank, torch.device("cpu"), "gloo" if world > 1 else "none")
    cfg = FLConfig(comm_round=rounds, epochs=2, batch_size=4, lr=0.05, dense_ratio=0.5, seed=7, **cfg_kw)
    return FLRunner(eng, splits, cfg, info, model)


def test_executor_snip_rounds_and_aggregation():
    r = _runner()
    mask = r.generate_global_mask_snip()
    sel = mask[r.maskable]
    assert abs(float(sel.mean()) - 0.5) < 0.02
    assert float(mask[~r.maskable].min()) == 1.0
    res = r.run_round(0)
    # global = sample-weighted mean of the clients' rows (equal sizes -> plain mean), params and buffers
    assert torch.allclose(r.w_global, r.theta.mean(0), atol=1e-6)
    assert torch.allclose(r.b_global, r.bufs.mean(0), atol=1e-5)
    # SalientGrads: masked weights are exactly zero on every client after local training
    assert float((r.theta[:, r.maskable] * (1 - mask[r.maskable])).abs().max()) == 0.0
    assert 0.0 <= res["global_test_acc"] <= 1.0


def _dist_worker(rank, world, port, out, cfg_kw=None):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = _runner(rank, world, **(cfg_kw or {}))
    r.generate_global_mask_snip()
    for k in range(2):
        r.run_round(k)
    if rank == 0:
        torch.save({"w": r.w_global, "acc": r.stat_info["global_test_acc"]}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg_kw", [{}, {"aggregator": "median"}, {"update_topk": 0.1}, {"heartbeat_s": 0.5}])
def test_two_rank_gloo_matches_single_process(tmp_path, cfg_kw):
    """2 ranks (clients sharded, mask-compacted all-reduce / all-gathered robust aggregation) == 1 process."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "w.pt")
    mp.start_processes(_dist_worker, args=(2, port, out, cfg_kw), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    r = _runner(**cfg_kw)
    r.generate_global_mask_snip()
    for k in range(2):
        r.run_round(k)
    assert torch.allclose(got["w"], r.w_global, atol=1e-5), float((got["w"] - r.w_global).abs().max())
    assert np.allclose(got["acc"], r.stat_info["global_test_acc"])


def _rows_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.save(_trained_rows(rank, world), "%s.%d" % (out, rank))
    dist.destroy_process_group()


def _trained_rows(rank=0, world=1):
    """Each local client's row after round 0's local training (before the first aggregation)."""
    r = _runner(rank, world)
    r.generate_global_mask_snip()
    r._round_start(0)
    sampled = r.sample_clients(0)
    r.local_train(0, sampled)
    rows, loc = r._local_rows(range(r.N))
    return {int(c): r.theta[i].clone() for i, c in zip(rows, loc)}


def test_sharded_rows_bit_identical_to_single_process(tmp_path):
    """A client's local training does not depend on which rank trains it: after the SNIP mask and round 0's local
    training, every client row of 2 gloo ranks is bit-identical to the same client's row in one process.  (Later
    rounds start from an all-reduced global model, whose summation order differs across layouts: the two-rank test
    above checks that at fp32 rounding.)"""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "rows")
    mp.start_processes(_rows_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    got = {}
    for k in range(2):
        got.update(torch.load("%s.%d" % (out, k), weights_only=True))
    ref = _trained_rows()
    assert set(got) == set(ref) and len(ref) > 2
    bad = [c for c in ref if not torch.equal(got[c], ref[c])]
    assert not bad, bad


def test_executor_robust_aggregation_rejects_outlier():
    from neuroimagedisttraining_amd.core import robustness as R
    for kind in ("krum", "multikrum", "median", "trimmed_mean"):
        r = _runner(clients=5, aggregator=kind, byzantine_f=1, trim_ratio=0.2)
        r.mask = torch.ones(r.P)
        sampled = list(range(5))
        r.theta[:, :r.P] = torch.randn(5, r.P) * 0.01
        r.theta[3, :r.P] += 100.0  # Byzantine client
        r.aggregate(sampled)
        assert float(r.w_global.abs().max()) < 1.0, kind
        M = torch.cat([r.theta[:, :r.P], r.bufs[:, :r.Q]], 1)
        if kind == "median":
            assert torch.allclose(r.w_global, R.coordinate_median(M)[:r.P])


def test_executor_checkpoint_resume_is_exact(tmp_path):
    from neuroimagedisttraining_amd.utils import checkpoint as ck
    a = _runner(rounds=3)
    a.generate_global_mask_snip()
    for k in range(3):
        a.run_round(k)
    b = _runner(rounds=3)
    b.generate_global_mask_snip()
    b.run_round(0)
    ck.save_runner(b, str(tmp_path), 1)
    c = _runner(rounds=3)
    start = ck.load_runner(c, str(tmp_path))
    assert start == 1
    for k in range(start, 3):
        c.run_round(k)
    assert torch.equal(a.w_global, c.w_global)
    assert torch.equal(a.theta, c.theta)
    assert c.stat_info["global_test_acc"][-1] == a.stat_info["global_test_acc"][-1]


def test_topk_update_aggregation_full_k_equals_fedavg():
    """update_topk = 1.0 sends every coordinate: identical to dense FedAvg of the params."""
    a = _runner(update_topk=1.0)
    b = _runner()
    for r in (a, b):
        r.generate_global_mask_snip()
        r.run_round(0)
    assert torch.allclose(a.w_global, b.w_global, atol=1e-6)
    assert torch.allclose(a.b_global, b.b_global, atol=1e-6)


@pytest.mark.parametrize("algo", ["fedavg", "fedprox", "ditto", "dpsgd", "fedfomo", "local", "subavg", "dispfl"])
def test_cli_entry_points_run_end_to_end(algo, tmp_path):
    """Every reference entry point (main_<algo>.py flags) runs a tiny federation end to end on the CPU path and
    writes its log under LOG/<dataset>/<identity>.log; frac 0.1 of 3 clients still samples one client."""
    from neuroimagedisttraining_amd import cli
    argv = ["--model", "lenet5", "--dataset", "cifar10", "--client_num_in_total", "3", "--comm_round", "1",
            "--epochs", "1", "--batch_size", "32", "--synthetic_size", "240", "--engine", "torch",
            "--log_dir", str(tmp_path)]
    out = cli.main(algo, argv)
    assert out is not None
    logs = list((tmp_path / "cifar10").glob("*.log"))
    assert len(logs) == 1 and logs[0].stat().st_size > 0


class Tiny3DNoDrop(nn.Module):
    """Tiny 3D CNN without dropout (SNIP scores of the two paths are then deterministic functions of the batch)."""

    def __init__(self):
        super().__init__()
        self.features = nn.Sequential(nn.Conv3d(1, 4, 3, 2), nn.BatchNorm3d(4), nn.ReLU(), nn.Conv3d(4, 8, 3))
        self.classifier = nn.Linear(8, 1)

    def forward(self, x):
        return self.classifier(self.features(x).amax((2, 3, 4)))


def test_stratified_itersnip_eager_and_runner_select_the_same_mask():
    """--stratified_sampling --itersnip_iteration 3: the reference-semantics SailentGradsAPI and the client-batched
    FLRunner draw the same label-stratified batches (snip.stratified_batch, RNG keyed by (seed, client, iter)) and
    select the same global SNIP mask; a stratified batch holds each class in proportion (largest remainders)."""
    from neuroimagedisttraining_amd.algorithms import snip as S
    from neuroimagedisttraining_amd.algorithms.salientgrads import SailentGradsAPI
    from neuroimagedisttraining_amd.data.abcd import _assemble
    from neuroimagedisttraining_amd.data.volumes import VolumeStore
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, TorchEngine
    from neuroimagedisttraining_amd.parallel import runtime as rt
    g = torch.Generator().manual_seed(11)
    clients, n_tr, n_te, B = 3, 20, 5, 8
    N = clients * (n_tr + n_te)
    vols = torch.randint(0, 256, (N, 13, 13, 13), dtype=torch.uint8, generator=g)
    labels = (torch.rand(N, generator=g) < 0.3).float()
    train = {c: np.arange(c * 25, c * 25 + n_tr) for c in range(clients)}
    test = {c: np.arange(c * 25 + n_tr, c * 25 + 25) for c in range(clients)}
    # the stratified draw itself: class counts proportional to the client's label histogram
    y0 = labels[train[0]].numpy()
    b = S.stratified_batch(train[0], y0, B, S.stratified_rng(5, 0, 0))
    assert len(set(b.tolist())) == B and set(b.tolist()) <= set(train[0].tolist())
    want = B * np.bincount(y0.astype(int), minlength=2) / len(y0)
    got = np.bincount(labels[b].numpy().astype(int), minlength=2)
    assert np.all(np.abs(got - want) < 1.0)

    torch.manual_seed(3)
    model = Tiny3DNoDrop()
    store = VolumeStore(vols, labels, torch.zeros(N))
    ds = _assemble(store, train, test, B, seed=5)
    args = _args(client_num_in_total=clients, client_num_per_round=clients, batch_size=B, itersnip_iteration=3,
                 stratified_sampling=True, seed=5)
    import copy
    api = SailentGradsAPI(ds, torch.device("cpu"), args, VolumeTrainer(copy.deepcopy(model), args))
    eager = api.generate_global_mask_snip()

    splits = [ClientSplit(train[c], test[c]) for c in range(clients)]
    eng = TorchEngine(copy.deepcopy(model), vols, labels, "cpu")
    info = rt.DistInfo(0, 1, 0, torch.device("cpu"), "none")
    cfg = FLConfig(comm_round=1, epochs=1, batch_size=B, dense_ratio=0.5, seed=5, itersnip_iteration=3,
                   stratified_sampling=True)
    r = FLRunner(eng, splits, cfg, info, copy.deepcopy(model))
    flat = r.generate_global_mask_snip()
    pl = eng.players
    n_diff = n_tot = 0
    for i, name in enumerate(pl.names):
        m = flat[pl.offsets[i]:pl.offsets[i] + pl.numel(i)].view(pl.shapes[i])
        n_diff += int((m != eager[name]).sum())
        n_tot += m.numel()
    # identical batches and scores; only fp32 summation order differs (a borderline tie may flip)
    print("mask mismatches", n_diff, "of", n_tot)
    assert n_diff <= max(1, n_tot // 1000), (n_diff, n_tot)
