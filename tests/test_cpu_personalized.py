"""CPU tests of the client-batched personalized runners and the mask layer.

* mask ops (torch twins of the HIP kernels) against the reference-style per-layer dict ops of
  ``algorithms/sparse.py`` (fire / regrow with torch.sort, numpy.percentile fake_prune, masked average);
* every runner (DisPFL, SubAvg, Ditto, D-PSGD, FedFomo, Local, SalientGrads, FedAvg) with ragged client sizes and
  partial last batches: 2 gloo ranks (and 3 for the neighbour-exchange algorithms) == 1 process.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.nn as nn


class Tiny3D(nn.Module):
    def __init__(self):
        super().__init__()
        self.features = nn.Sequential(nn.Conv3d(1, 4, 3, 2), nn.BatchNorm3d(4), nn.ReLU(), nn.MaxPool3d(2, 2),
                                      nn.Conv3d(4, 8, 3), nn.BatchNorm3d(8), nn.ReLU())
        self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(8, 1))

    def forward(self, x):
        return self.classifier(self.features(x).amax((2, 3, 4)))


# ------------------------------------------------------------------------------------------------ mask layer
def _space():
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.engine import masks as MK
    m = Tiny3D()
    pl = ParamLayout.from_tensors(list(m.named_parameters()))
    return m, pl, MK.MaskSpace(pl)


def test_fire_regrow_match_reference_dict_ops():
    from neuroimagedisttraining_amd.algorithms import sparse as SP
    from neuroimagedisttraining_amd.engine import masks as MK
    model, pl, ms = _space()
    torch.manual_seed(0)
    P = pl.total
    w = torch.randn(1, P)
    w[0, ::5] = torch.round(w[0, ::5])  # ties
    g = torch.randn(1, P)
    m = (torch.rand(1, P) < 0.5).float()
    named = lambda flat: {n: flat[0, o:o + pl.numel(i)].view(pl.shapes[i])  # noqa: E731
                          for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
    new, num_remove = SP.fire_mask(named(m), named(w), 3, 0.5, 10)
    new = SP.regrow_mask(new, num_remove, named(g))
    bits = MK.pack_bits(m)
    nnz = ms.popcount(bits)
    k = torch.ceil(torch.tensor(SP.cosine_annealing(0.5, 3, 10), dtype=torch.float32) * nnz.float()).long()
    assert [int(x) for x in k[0]] == [num_remove[n] for n in pl.names]
    ms.select(MK.FIRE, w, bits, k)
    ms.select(MK.REGROW_ABS, g, bits, k)
    got = MK.unpack_bits(bits, P)[0]
    exp = torch.cat([new[n].reshape(-1) for n in pl.names])
    assert torch.equal(got, exp)


def test_percentile_prune_matches_numpy_fake_prune():
    from neuroimagedisttraining_amd.algorithms import sparse as SP
    from neuroimagedisttraining_amd.engine import masks as MK
    model, pl, ms = _space()
    torch.manual_seed(1)
    P = pl.total
    w = torch.randn(2, P)
    w[1, ::3] = 0
    m = (torch.rand(2, P) < 0.7).float()
    names = [n for n in pl.names if "weight" in n and "bn" not in n]
    out = MK.unpack_bits(ms.percentile_prune(w, MK.pack_bits(m), 0.2, names), P)
    for r in range(2):
        sd = {n: w[r, o:o + pl.numel(i)].view(pl.shapes[i]) for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
        mk = {n: m[r, o:o + pl.numel(i)].view(pl.shapes[i]) for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
        ref = SP.fake_prune(0.2, sd, mk)
        assert torch.equal(out[r], torch.cat([ref[n].reshape(-1).float() for n in pl.names]))


def test_masked_average_matches_subavg_aggregate():
    from neuroimagedisttraining_amd.algorithms import sparse as SP
    from neuroimagedisttraining_amd.engine import masks as MK
    model, pl, ms = _space()
    torch.manual_seed(2)
    P = pl.total
    rows = torch.randn(3, P)
    m = (torch.rand(3, P) < 0.5).float()
    rows = rows * m
    s, c = torch.zeros(P), torch.zeros(P)
    MK.masked_rows_sum(rows, P, MK.pack_bits(m), s, c)
    srv = torch.randn(P)
    ours = torch.where(c > 0, s / c, srv)
    named = lambda v: {n: v[o:o + pl.numel(i)].view(pl.shapes[i]).clone()  # noqa: E731
                       for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
    ref = SP.masked_average(named(srv), [(named(m[i]), named(rows[i])) for i in range(3)])
    assert torch.allclose(ours, torch.cat([ref[n].reshape(-1) for n in pl.names]), atol=1e-6)


def test_masked_mean_rows_matches_dispfl_neighbour_formula():
    """DisPFL's masked neighbour average (dispfl_api.py:138-142, the paper's aggregation): per coordinate the mean of
    the neighbours whose mask keeps it, times the client's own mask, 0 where no neighbour keeps it."""
    from neuroimagedisttraining_amd.engine import masks as MK
    torch.manual_seed(3)
    n, K = 200, 4
    src = [torch.randn(n + 8) for _ in range(K)]
    m = (torch.rand(K, n) < 0.4)
    own = torch.rand(n) < 0.6
    bits = MK.pack_bits(m.float())
    obits = MK.pack_bits(own.float().view(1, -1))[0]
    outs = [torch.full((n + 8,), 7.0), torch.full((n + 8,), 7.0)]
    plan = [(outs[0], obits, [(src[k], bits[k]) for k in range(K)]),
            (outs[1], obits, [(src[k], bits[k]) for k in (1, 3)])]
    MK.masked_mean_rows(plan, n)
    for o, ks in zip(outs, ([0, 1, 2, 3], [1, 3])):
        num = sum(src[k][:n] * m[k] for k in ks)
        cnt = sum(m[k].float() for k in ks)
        want = torch.where(cnt > 0, num / cnt.clamp_min(1), torch.zeros(n)) * own
        assert torch.allclose(o[:n], want, atol=1e-6)
        assert torch.all(o[n:] == 7.0)  # nothing past n written


# ------------------------------------------------------------------------------------------------ runners
SIZES = [10, 7, 14, 10, 6, 11]


def _runner(algo, rank=0, world=1, rounds=2, sizes=None, **kw):
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(5)
    splits, off = [], 0
    for s in (sizes or SIZES):
        tr = np.arange(off, off + s)
        splits.append(ClientSplit(tr, np.arange(off + s, off + s + 4), tr[:3]))
        off += s + 4
    vols = torch.randint(0, 256, (off, 15, 15, 15), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 2, (off,), generator=g).float()
    model = Tiny3D()
    eng = TorchEngine(model, vols, labels, "cpu")
    info = rt.DistInfo(rank, world, rank, torch.device("cpu"), "gloo" if world > 1 else "none")
    cfg = dict(comm_round=rounds, epochs=2, batch_size=4, lr=0.05, dense_ratio=0.5, seed=7, acc_thresh=0.0,
               each_prune_ratio=0.2, local_epochs=1, dist_thresh=0.0)
    cfg.update(kw)
    return make_runner(algo, eng, splits, FLConfig(**cfg), info, model)


def _collect(r):
    """Per-client model rows (global client order) + headline metrics."""
    rows = {c: r.theta[r.row_of[c], :r.P].clone() for c in r.local}
    bits = {c: r.mbits[r.row_of[c]].clone() for c in r.local} if getattr(r, "mbits", None) is not None else {}
    pers = {c: r.pers.theta[r.row_of[c], :r.P].clone() for c in r.local} if hasattr(r, "pers") else {}
    return {"rows": rows, "bits": bits, "pers": pers, "w": r.w_global.clone(),
            "comm": int(r.stat_info.get("sum_comm_params", 0)),
            "stats": {k: v for k, v in r.stat_info.items() if isinstance(v, list) and v and
                      isinstance(v[0], float) and "time" not in k}}


def _drive(r, rounds):
    if r.alg == "salientgrads":
        r.generate_global_mask_snip()
    for k in range(rounds):
        r.run_round(k)
    r.finish()


def _worker(rank, world, port, out, algo, kw, ckpt=None):
    """ckpt = (directory, mode): "save" runs round 0 and checkpoints; "resume" loads and runs round 1."""
    import torch.distributed as dist
    from neuroimagedisttraining_amd.utils import checkpoint as ck
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = _runner(algo, rank, world, **kw)
    if ckpt is None:
        _drive(r, 2)
    elif ckpt[1] == "save":
        if r.alg == "salientgrads":
            r.generate_global_mask_snip()
        r.run_round(0)
        ck.save_runner(r, ckpt[0], 1)
    elif ckpt[1] == "save_async":  # background-written saves after rounds 0 and 1, keep only the newest
        if r.alg == "salientgrads":
            r.generate_global_mask_snip()
        saver = ck.Checkpointer(ckpt[0], r.info, every=1, keep_last=1, async_write=True)
        for k in range(2):
            r.run_round(k)
            saver.maybe_save(r, k + 1)
        saver.close()
    else:
        loaded = []
        real_load = torch.load

        def spy(path, *a, **k):
            loaded.append(os.path.basename(str(path)))
            return real_load(path, *a, **k)
        torch.load = spy
        try:
            start = ck.load_runner(r, ckpt[0])
        finally:
            torch.load = real_load
        for k in range(start, 2):
            r.run_round(k)
        r.finish()
        torch.save({"loaded": loaded, "local": list(r.local)}, out + ".loaded.%d" % rank)
    torch.save(_collect(r), out + ".%d" % rank)
    dist.destroy_process_group()


def _spawn(world, out, algo, kw, ckpt=None):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _port(), out, algo, kw, ckpt), nprocs=world, join=True,
                       start_method="spawn")
    got = {"rows": {}, "bits": {}, "pers": {}}
    for rk in range(world):
        d = torch.load(out + ".%d" % rk, weights_only=True)
        for key in ("rows", "bits", "pers"):
            got[key].update(d[key])
        if rk == 0:
            got["w"], got["stats"], got["comm"] = d["w"], d["stats"], d["comm"]
    return got


def _same(got, ref, n, algo, atol=1e-5):
    for c in range(n):
        assert torch.allclose(got["rows"][c], ref["rows"][c], atol=atol), (algo, c)
        if ref["bits"]:
            assert torch.equal(got["bits"][c], ref["bits"][c]), (algo, c)
        if ref["pers"]:
            assert torch.allclose(got["pers"][c], ref["pers"][c], atol=atol), (algo, c)
    assert torch.allclose(got["w"], ref["w"], atol=atol)
    if algo == "dispfl":  # finish() folds the device-side communication counter (summed over ranks)
        assert ref["comm"] > 0 and got.get("comm", ref["comm"]) == ref["comm"], (got.get("comm"), ref["comm"])
    for k, v in ref["stats"].items():
        assert np.allclose(got["stats"][k], v, atol=1e-6), (algo, k)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CASES = [("dispfl", 2, {}), ("dispfl", 3, {"frac": 0.5, "active": 0.8, "dis_gradient_check": True}),
         ("dispfl", 2, {"frac": 0.5, "dispfl_aggregate": True}),
         ("subavg", 2, {"frac": 0.5}), ("ditto", 2, {"frac": 0.5}), ("dpsgd", 3, {"frac": 0.5, "cs": "ring"}),
         ("dpsgd", 2, {"frac": 0.5, "cs": "random"}), ("fedfomo", 3, {"frac": 0.5}), ("local", 2, {"frac": 0.5}),
         ("salientgrads", 2, {}), ("fedavg", 3, {"frac": 0.5})]


@pytest.mark.parametrize("algo,world,kw", CASES)
def test_runner_multirank_matches_single_process(algo, world, kw, tmp_path):
    """Clients sharded over gloo ranks (neighbour rows exchanged point-to-point, partial sums all-reduced) give the
    same per-client models, masks and metrics as one process."""
    got = _spawn(world, str(tmp_path / "r"), algo, kw)
    r = _runner(algo, **kw)
    _drive(r, 2)
    _same(got, _collect(r), len(SIZES), algo)


def test_hundred_clients_four_ranks_frac_quarter_matches_single_process(tmp_path):
    """100 clients, frac 0.25 (25 sampled per round, unevenly spread over the 4 ranks' shards) == 1 process."""
    kw = {"sizes": [6 + (c % 5) * 2 for c in range(100)], "frac": 0.25, "epochs": 1}
    got = _spawn(4, str(tmp_path / "r"), "fedavg", kw)
    r = _runner("fedavg", **kw)
    _drive(r, 2)
    _same(got, _collect(r), 100, "fedavg")


@pytest.mark.parametrize("algo", ["salientgrads", "dispfl", "fedfomo"])
def test_checkpoint_from_four_ranks_resumes_on_two_exactly(algo, tmp_path):
    """Round 0 on 4 ranks -> checkpoint -> resume round 1 on 2 ranks == 2 uninterrupted rounds in one process
    (client rows keyed by id, RNG streams and affinities restored, round tagged shards + latest pointer)."""
    d = str(tmp_path / "ck")
    _spawn(4, str(tmp_path / "a"), algo, {}, ckpt=(d, "save"))
    got = _spawn(2, str(tmp_path / "b"), algo, {}, ckpt=(d, "resume"))
    r = _runner(algo)
    _drive(r, 2)
    _same(got, _collect(r), len(SIZES), algo)


def test_async_indexed_checkpoint_four_ranks_resumes_on_two(tmp_path):
    """Background-written saves (pinned snapshot, writer thread, lagged barrier + ``latest`` commit) with
    keep_last=1 on 4 ranks; stale shards of a larger crashed run in the round directory; resume on 2 ranks:
    each rank opens only the shards its clients live in (client index), and the state equals 2 rounds in one
    process."""
    d = tmp_path / "ck"
    _spawn(4, str(tmp_path / "a"), "dispfl", {}, ckpt=(str(d), "save_async"))
    assert sorted(p.name for p in d.iterdir()) == ["latest", "round_2"]  # round_1 pruned
    assert (d / "latest").read_text() == "2"
    # a crashed 8-rank run left shards 4..7 of its own round 2 behind: never read (index names shards 0..3)
    for k in range(4, 8):
        torch.save({"junk": torch.zeros(1)}, d / "round_2" / ("clients_rank%d.pt" % k))
    got = _spawn(2, str(tmp_path / "b"), "dispfl", {}, ckpt=(str(d), "resume"))
    g = torch.load(d / "round_2" / "global.pt", weights_only=True)
    index = g["index"].tolist()
    for rk in range(2):
        rec = torch.load(str(tmp_path / "b") + ".loaded.%d" % rk, weights_only=True)
        shards = sorted(n for n in rec["loaded"] if n.startswith("clients_rank"))
        assert shards == sorted({"clients_rank%d.pt" % index[c] for c in rec["local"]}), (rk, shards)
    r = _runner("dispfl")
    _drive(r, 2)
    _same(got, _collect(r), len(SIZES), "dispfl")


def test_dispfl_masks_keep_density_and_masked_weights_zero():
    from neuroimagedisttraining_amd.engine import masks as MK
    r = _runner("dispfl", rounds=3)
    d0 = r.mspace.popcount(r.mbits).sum(1)
    _drive(r, 3)
    assert torch.equal(r.mspace.popcount(r.mbits).sum(1), d0)  # fire k == regrow k per layer
    m = MK.unpack_bits(r.mbits, r.P)
    # weights outside the mask they were trained with are zero; after fire/regrow only newly regrown ones may be 0
    moved = r.mspace.hamming(r.shared_bits, r.mbits).sum()
    assert int(moved) > 0
    assert float((r.theta[:, :r.P] * (1 - MK.unpack_bits(r.shared_bits, r.P))).abs().max()) == 0.0
    assert m.shape == (r.C, r.P)


def test_subavg_prunes_and_aggregates_over_mask_counts():
    from neuroimagedisttraining_amd.engine import masks as MK
    r = _runner("subavg", rounds=3, dense_ratio=0.1, acc_thresh=-1.0)
    _drive(r, 3)
    dens = MK.unpack_bits(r.mbits, r.P).mean(1)
    assert float(dens.min()) < 1.0  # something was pruned (percentile 0.2 per weight layer)
    assert np.isfinite(r.w_global.numpy()).all()


REBALANCE_CASES = [("fedavg", 4, {"sizes": [6 + (c % 5) * 2 for c in range(100)], "frac": 0.25, "epochs": 1}),
                   ("salientgrads", 3, {"frac": 0.5}), ("subavg", 2, {"frac": 0.5}), ("ditto", 2, {"frac": 0.5}),
                   ("local", 3, {"frac": 0.5})]


@pytest.mark.parametrize("algo,world,kw", REBALANCE_CASES)
def test_rebalanced_multirank_matches_single_process(algo, world, kw, tmp_path):
    """Sampling-aware rebalancing (sampled clients' rows / masks / personal models migrate point-to-point to the
    least loaded ranks each round) changes where clients train, not what they compute."""
    kw = dict(kw, rebalance=True)
    got = _spawn(world, str(tmp_path / "r"), algo, kw)
    r = _runner(algo, **kw)
    _drive(r, 2)
    # fp32 partial sums are all-reduced from different per-rank groupings: w_global agrees to ~1e-7, rows to ~2e-5
    _same(got, _collect(r), len(kw.get("sizes", SIZES)), algo, atol=5e-5)


def _worker_sharded(rank, world, port, out, algo, kw):
    """A rank that holds ONLY its shard's samples (placeholder splits for the other clients), as bench.py and the
    CLI load them: rebalancing must move sample rows with the migrating clients."""
    import torch.distributed as dist
    from neuroimagedisttraining_amd.engine.executor import ClientSplit
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = _runner(algo, rank, world, **kw)
    full = r.e.store
    mine = [c for c in range(r.N) if r.owner[c] == rank]
    rows = np.concatenate([r._sample_rows(c) for c in mine])
    r.e.store = full[torch.as_tensor(rows)].clone()
    r.e.labels = r.e.labels[torch.as_tensor(rows)].clone()
    splits, off = [], 0
    for c, sp in enumerate(r.splits):
        ntr, nte, nva = len(sp.train), len(sp.test), 0 if sp.val is None else len(sp.val)
        if c in mine:
            splits.append(ClientSplit(np.arange(off, off + ntr), np.arange(off + ntr, off + ntr + nte),
                                      None if sp.val is None else np.arange(off + ntr + nte, off + ntr + nte + nva)))
            off += ntr + nte + nva
        else:
            splits.append(ClientSplit(np.zeros(ntr, np.int64), np.zeros(nte, np.int64),
                                      None if sp.val is None else np.zeros(nva, np.int64)))
    r.splits = splits
    held = [len(r.e.store)]
    _drive(r, 2)
    held.append(len(r.e.store))
    d = _collect(r)
    d["held"] = held
    torch.save(d, out + ".%d" % rank)
    dist.destroy_process_group()


@pytest.mark.parametrize("algo,world,kw", [
    ("fedavg", 4, {"sizes": [6 + (c % 5) * 2 for c in range(40)], "frac": 0.25, "epochs": 1}),
    ("fedfomo", 4, {"sizes": [6 + (c % 5) * 2 for c in range(16)], "frac": 0.5})])
def test_rebalancing_moves_samples_with_clients_on_sharded_stores(algo, world, kw, tmp_path):
    """4 gloo ranks, each holding only its own clients' samples: sampling-aware rebalancing migrates the sampled
    clients' sample rows (volumes + labels, train/test/val) with their state; every rank's store stays the size of
    its current clients (no replicated cohort) and the models equal the 1-process run."""
    import torch.multiprocessing as mp
    kw = dict(kw, rebalance=True)
    out = str(tmp_path / "r")
    mp.start_processes(_worker_sharded, args=(world, _port(), out, algo, kw), nprocs=world, join=True,
                       start_method="spawn")
    got = {"rows": {}, "bits": {}, "pers": {}}
    total = 0
    for rk in range(world):
        d = torch.load(out + ".%d" % rk, weights_only=True)
        for key in ("rows", "bits", "pers"):
            got[key].update(d[key])
        if rk == 0:
            got["w"], got["stats"], got["comm"] = d["w"], d["stats"], d["comm"]
        total += d["held"][1]
    n_all = sum(s + 4 + 3 for s in kw["sizes"])  # train + test + val rows of every client (_runner: val = 3)
    assert total == n_all  # the stores partition the cohort after migration
    r = _runner(algo, **kw)
    _drive(r, 2)
    _same(got, _collect(r), len(kw["sizes"]), algo, atol=5e-5)


def test_balanced_owner_evens_the_sampled_load():
    from neuroimagedisttraining_amd.engine.runner import FLRunner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    r = FLRunner.__new__(FLRunner)
    r.N = 12
    r.sizes = np.array([30, 5, 5, 5, 20, 20, 4, 4, 9, 9, 9, 9], dtype=np.int64)
    r.owner = np.array([0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2], dtype=np.int64)
    r.info = rt.DistInfo(0, 3, 0, torch.device("cpu"), "gloo")
    sampled = [0, 1, 2, 3, 4, 5, 8]
    own = r.balanced_owner(sampled)
    load = np.zeros(3, dtype=np.int64)
    before = np.zeros(3, dtype=np.int64)
    for c in sampled:
        load[own[c]] += r.sizes[c]
        before[r.owner[c]] += r.sizes[c]
    assert load.max() < before.max() and load.sum() == before.sum()
    assert load.max() - load.min() <= max(r.sizes[c] for c in sampled)
    assert all(own[c] == r.owner[c] for c in range(r.N) if c not in sampled)  # only sampled clients move
    assert np.array_equal(own, r.balanced_owner(sampled))                       # deterministic


def test_padded_bucket_eval_equals_exact_grouping(monkeypatch):
    """Ragged test splits evaluated in padded buckets (rows past a client's size repeat its first sample and are masked
    out; chunks of test_batch across the group) give the same per-client (correct, loss_sum, total) as the exact-size
    grouping, also for model rows shared by several clients."""
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(9)
    test_sizes = [3, 9, 17, 5, 30, 70, 9, 1]
    splits, off = [], 0
    for t in test_sizes:
        tr = np.arange(off, off + 6)
        splits.append(ClientSplit(tr, np.arange(off + 6, off + 6 + t), tr[:3]))
        off += 6 + t
    vols = torch.randint(0, 256, (off, 15, 15, 15), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 2, (off,), generator=g).float()
    model = Tiny3D()
    eng = TorchEngine(model, vols, labels, "cpu")
    info = rt.DistInfo(0, 1, 0, torch.device("cpu"), "none")
    r = make_runner("fedavg", eng, splits, FLConfig(comm_round=1, epochs=1, batch_size=4, lr=0.05, seed=7,
                                                    test_batch=16, group=3), info, model)
    with torch.no_grad():
        r.theta[:, :r.P].add_(torch.randn(r.theta.shape[0], r.P) * 0.05)
    C = len(test_sizes)
    for rows in (list(range(C)), [0] * C, [C - 1 - j for j in range(C)]):
        monkeypatch.setenv("NIDT_EVAL_PAD", "1")
        a = r.eval_grouped(r.theta, r.bufs, rows, list(range(C)))
        monkeypatch.setenv("NIDT_EVAL_PAD", "0")
        b = r.eval_grouped(r.theta, r.bufs, rows, list(range(C)))
        assert np.array_equal(a[:, 2], np.array(test_sizes, dtype=np.float64))
        assert np.allclose(a, b, rtol=1e-5, atol=1e-5), (a, b)
    assert [r._pad_size(n) for n in (1, 8, 9, 64, 65, 100, 1000)] == [8, 8, 16, 64, 77, 108, 1024]


def test_subavg_deferred_metrics_match_immediate(monkeypatch):
    """SubAvg's evaluation read one round late (NIDT_DEFER_METRICS=force on the CPU) gives the same rounds' results,
    stat_info lists and model rows as the immediate read."""
    out = {}
    for mode in ("0", "force"):
        monkeypatch.setenv("NIDT_DEFER_METRICS", mode)
        r = _runner("subavg")
        res = [r.run_round(k) for k in range(2)]
        out[mode] = ([dict(x) if x is not None else None for x in res], _collect(r))
    (ra, ca), (rb, cb) = out["0"], out["force"]
    assert ra == rb
    assert ca["stats"] == cb["stats"] and ca["stats"].get("test_acc")
    for c in ca["rows"]:
        assert torch.equal(ca["rows"][c], cb["rows"][c])
