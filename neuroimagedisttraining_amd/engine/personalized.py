"""Personalized and decentralized FL algorithms on the client-batched executor (HIP kernels on MI355X).

Every algorithm of the reference harness besides SalientGrads / FedAvg runs here with the same building blocks as
:class:`~.runner.FLRunner`: client rows resident on the GPU, lockstep local steps (hipGraphs), the fused optimizer
(per-client bit masks in weight or gradient mode, Ditto's pull), per-(client, layer) mask kernels, and RCCL for
everything that crosses ranks (all-reduce of partial sums, point-to-point neighbour rows, metric gathers).

* :class:`DisPFLRunner`  — ``DisPFL/dispfl_api.py:46-184``, ``DisPFL/client.py:32-99``: ERK / uniform per-client
  masks over all parameters, masked local training, eval-mode ``screen_gradients``, cosine-annealed fire (smallest
  |w| among active) + regrow (largest |g| among inactive, or random) per layer on device (K15), mask Hamming
  bookkeeping (K18), client dropout ``--active``.  Neighbour aggregation is commented out in the reference (Q10),
  so every client continues its own model; ``dispfl_aggregate`` enables the masked neighbour average.
* :class:`SubAvgRunner`  — ``subavg/subavg_api.py:43-139``, ``subavg/client.py:36-63``: gradient-masked training,
  ``fake_prune`` percentiles at the first and last epoch (K16), prune when the mask moved and the pruned model is
  accurate enough on the local training data, server average of each coordinate over the clients keeping it.
* :class:`DittoRunner`   — ``ditto/ditto_api.py:40-105``: FedAvg global model + personal models pulled towards the
  round's global model after every step (fused in the optimizer, K20).
* :class:`DPSGDRunner`   — ``dpsgd/dpsgd_api.py:41-178``: neighbour averaging (ring / random / full) as one row-mixing
  launch, neighbours on other ranks fetched point-to-point, global mean for evaluation, fine-tune every 100 rounds.
* :class:`FedFomoRunner` — ``fedfomo/fedfomo_api.py:53-217``: first-order model optimisation — validation losses of
  the candidate models (grouped evaluation launches), parameter distances (one kernel over all pairs), affinity-driven
  neighbour choice and the weighted neighbour update (row mixing).
* :class:`LocalRunner`   — ``local/local_api.py:51-84``: local-only training.

Host-side random decisions (client dropout, neighbour choice) are drawn from dedicated generators on every rank in
the reference's order, so all ranks agree without communication.
"""
from __future__ import annotations

import math
import random
import os
import time
from dataclasses import replace

import numpy as np
import torch

from ..algorithms import sparse as SP
from ..parallel import runtime as rt
from . import masks as MK
from .executor import padded_rows
from .runner import MASK_GRAD, MASK_WEIGHT, FLRunner, RowSet, StepSpec


def _sparsities(params, dense_ratio, cfg):
    dist = "uniform" if cfg.uniform else "ERK"
    return SP.erk_sparsities(params, dense_ratio, erk_power_scale=cfg.erk_power_scale, distribution=dist)


class PersonalizedRunner(FLRunner):
    """Shared machinery: personal rows, per-client mask bit rows, neighbour row exchange, local evaluations."""

    def __init__(self, engine, splits, cfg, info, template_model, logger=None, algorithm="local"):
        super().__init__(engine, splits, cfg, info, template_model, logger, algorithm)
        self.mspace = MK.MaskSpace(engine.players)  # masks cover every parameter (the reference's named_parameters)
        self.mbits = None
        self.np_rng = np.random.RandomState(cfg.seed)
        self.py_rng = random.Random(cfg.seed)
        for k in ("old_mask_test_acc", "new_mask_test_acc", "test_acc", "test_loss", "mask_dis_matrix"):
            self.stat_info.setdefault(k, [])
        self.rowset = RowSet(self.theta, self.bufs)

    # ---------------------------------------------------------------------------------------------- helpers
    def _row_state(self):
        out = super()._row_state()
        for name in ("mbits", "shared_bits"):
            t = getattr(self, name, None)
            if t is not None:
                out.append((name, t))
        return out

    def all_rows(self):
        return list(range(self.C)), list(self.local)

    def snapshot(self, rs=None):
        """Copy of a row set with 16-B aligned rows (``clone`` of the padded views would pack rows at stride P)."""
        rs = rs or self.rowset
        n = rs.theta.shape[0]
        out = RowSet(padded_rows(n, self.P, self.device), padded_rows(n, self.Q, self.device))
        out.theta.copy_(rs.theta)
        out.bufs.copy_(rs.bufs)
        return out

    def cat_rows(self, *sets):
        """Concatenate row sets into one padded row set."""
        n = sum(s.theta.shape[0] for s in sets)
        out = RowSet(padded_rows(max(1, n), self.P, self.device), padded_rows(max(1, n), self.Q, self.device))
        o = 0
        for s in sets:
            k = s.theta.shape[0]
            out.theta[o:o + k].copy_(s.theta)
            out.bufs[o:o + k].copy_(s.bufs)
            o += k
        return out

    def fetch(self, needs, src):
        """{client: (theta_row [P], bufs_row [Q])} for every client in ``needs[self.rank]``: local clients are views
        of ``src``, remote ones arrive point-to-point from their owners (same ``needs`` on every rank)."""
        P, Q = self.P, self.Q
        Pp = (P + 63) // 64 * 64  # the buffer section of a received row starts 16-B aligned (vector kernels)

        def row(c):
            v = torch.zeros(Pp + Q, dtype=torch.float32, device=self.device)
            v[:P] = src.theta[self.row_of[c], :P]
            v[Pp:] = src.bufs[self.row_of[c], :Q]
            return v
        recv = rt.exchange_rows(self.info, self.owner, needs, row, Pp + Q, self.device)
        out = {}
        for c in needs[self.info.rank]:
            if c in self.row_of:
                out[c] = (src.theta[self.row_of[c]], src.bufs[self.row_of[c]])
            else:
                v = recv[c]
                out[c] = (v[:P], v[Pp:])
        return out

    def pool(self, entries):
        """Stack (theta_row, bufs_row) pairs into a fresh row set (16-B aligned rows for the kernels)."""
        th = padded_rows(max(1, len(entries)), self.P, self.device)
        bu = padded_rows(max(1, len(entries)), self.Q, self.device)
        for i, (t, b) in enumerate(entries):
            th[i].copy_(t[:self.P])
            bu[i].copy_(b[:self.Q])
        return RowSet(th, bu)

    def eval_local(self, rs, rows, clients, which="test"):
        """[N, 3] (correct, loss_sum, total) of model rows[j] on clients[j] (this rank's part), gathered."""
        res = self.eval_grouped(rs.theta, rs.bufs, rows, clients, which) if rows else np.zeros((0, 3))
        return self.gather_metrics(clients, res)

    def log_test(self, r, key=None, tag="test"):
        acc, loss = self.mean_acc_loss(r)
        if key:
            self.stat_info[key].append(acc)
        if self.log is not None and self.info.is_main:
            self.log.info({"%s_acc" % tag: acc, "%s_loss" % tag: loss})
        return acc, loss

    def local_masks_from(self, per_client_float):
        """list of N flat float masks [P] (host or device) -> this rank's bit rows [C, W]."""
        m = torch.stack([per_client_float[c].to(self.device) for c in self.local]) if self.C else \
            torch.zeros((1, self.P), device=self.device)
        return MK.pack_bits(m)

    def flat_mask(self, named_masks):
        """{name: tensor} mask dict -> flat [P] float (ones for names without a mask)."""
        lay = self.e.players
        out = torch.ones(self.P, dtype=torch.float32)
        for i, n in enumerate(lay.names):
            if n in named_masks:
                out[lay.offsets[i]:lay.offsets[i] + lay.numel(i)] = named_masks[n].reshape(-1).float().cpu()
        return out

    def end_of_training(self, round_idx, clients):
        self.flush_round_log(round_idx, clients, comm_lines=False)
        if self.log is not None or self.device.type != "cuda":
            self.sync_stats()

    def finish(self):
        self.sync_stats()
        return None

    def train(self):
        for r in range(self.cfg.comm_round):
            self.run_round(r)
        self.finish()
        return self.stat_info


# ================================================================================================== Local
class LocalRunner(PersonalizedRunner):
    """Local-only baseline: sampled clients continue their own model (``local/local_api.py:51-84``)."""

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        self._round_start(round_idx)
        sampled = self.sample_clients(round_idx)
        self.rebalance(sampled)
        rows, loc = self._local_rows(sampled)
        self.train_rows(self.rowset, rows, loc, round_idx, self.cfg.epochs)
        t1 = time.perf_counter()
        self.timers["train"] += t1 - t0
        self.stat_info["sum_training_flops"] += int(self.cfg.epochs * sum(self.sizes[c] for c in sampled))
        self.end_of_training(round_idx, sampled)
        r = self.eval_local(self.rowset, rows, loc)  # client.train tests right after training (local/client.py)
        acc, _ = self.log_test(r, "person_test_acc")
        self.timers["eval"] += time.perf_counter() - t1
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return {"person_test_acc": acc}


# ================================================================================================== Ditto
class DittoRunner(PersonalizedRunner):
    """FedAvg global model + personal models with the proximal pull ``w -= lr*lamda*(w - w_global)`` after every
    step for ``local_epochs`` (``ditto/ditto_api.py:40-78``, ``ditto/my_model_trainer.py:38-68``)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.pers = RowSet(padded_rows(max(1, self.C), self.P, self.device),
                           padded_rows(max(1, self.C), self.Q, self.device))
        self.pers.theta.copy_(self.w_global.expand_as(self.pers.theta))
        self.pers.bufs.copy_(self.b_global.expand_as(self.pers.bufs))
        self._pull_ref = torch.zeros_like(self.w_global)

    def _row_state(self):
        return super()._row_state() + [("pers.theta", self.pers.theta), ("pers.bufs", self.pers.bufs)]

    def finish(self):
        self.record_avg_inference_flops()  # ditto_api.py:78: w_global for every client
        return super().finish()

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        self._round_start(round_idx)
        sampled = self.sample_clients(round_idx)
        self.rebalance(sampled)
        self._pull_ref.copy_(self.w_global)  # the round's global model (deepcopy(w_global) in the reference)
        self.local_train(round_idx, sampled)  # global-model training from w_global
        rows, loc = self._local_rows(sampled)
        spec = StepSpec(lamda=self.cfg.lamda, pref=self._pull_ref)
        self.train_rows(self.pers, rows, loc, round_idx, self.cfg.local_epochs or self.cfg.epochs, spec, tag=1)
        t1 = time.perf_counter()
        self.aggregate(sampled)
        t2 = time.perf_counter()
        self.end_of_training(round_idx, sampled)
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        res = None
        if self._eval_due(round_idx):
            r = self.eval_local(self.pers, *self.all_rows())
            acc, loss = self.log_test(r, "person_test_acc")
            res = {"person_test_acc": acc, "person_test_loss": loss}
        self.timers["eval"] += time.perf_counter() - t2
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return res


# ================================================================================================== D-PSGD
class DPSGDRunner(PersonalizedRunner):
    """Decentralized SGD: every client averages its neighbours' last models, then trains (``dpsgd_api.py:41-103``)."""

    def neighbours(self, round_idx, c):
        N, K, cs = self.N, max(1, int(self.N * self.cfg.frac)), self.cfg.cs
        if N == K:
            return list(range(N))
        if cs == "random":
            np.random.seed(round_idx + c)
            idx = np.random.choice(range(N), min(K, N), replace=False)
            while c in idx:
                idx = np.random.choice(range(N), min(K, N), replace=False)
            nei = list(idx)
        elif cs == "ring":
            nei = [(c - 1 + N) % N, (c + 1) % N]
        elif cs == "full":
            nei = [j for j in range(N) if j != c]
        else:
            raise ValueError("unknown cs %r" % cs)
        return sorted(int(j) for j in list(nei) + [c])

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        self._round_start(round_idx)
        nei = {c: self.neighbours(round_idx, c) for c in range(self.N)}
        needs = [sorted({j for c in self.shards[r] for j in nei[c]}) for r in range(self.info.world)]
        last = self.snapshot()
        src = self.fetch(needs, last)
        plan = []
        for c in self.local:  # w_local = mean of the neighbourhood's last models (params and buffers)
            i = self.row_of[c]
            w = 1.0 / len(nei[c])
            plan.append((self.theta[i], [(src[j][0], w) for j in nei[c]]))
        MK.mix_rows(plan, self.P)
        MK.mix_rows([(self.bufs[self.row_of[c]], [(src[j][1], 1.0 / len(nei[c])) for j in nei[c]])
                     for c in self.local], self.Q)
        del src, last
        rows, loc = self.all_rows()
        self.train_rows(self.rowset, rows, loc, round_idx, self.cfg.epochs)
        t1 = time.perf_counter()
        # global model = uniform mean of all personal models (evaluation only)
        buf, Pp = self.weighted_partial(self.theta, self.bufs, rows, [1.0 / self.N] * len(rows))
        rt.all_reduce_buckets(buf, self.info)
        self.w_global.copy_(buf[:self.P])
        self.b_global.copy_(buf[Pp:])
        t2 = time.perf_counter()
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        self.stat_info["sum_training_flops"] += int(self.cfg.epochs * self.sizes.sum())
        self.end_of_training(round_idx, range(self.N))
        res = self.evaluate(round_idx)
        if round_idx % 100 == 99:  # fine-tune evaluation (dpsgd_api.py:89-101); state is unchanged
            self.finetune_round()
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return res


# ================================================================================================== FedFomo
class FedFomoRunner(PersonalizedRunner):
    """FedFomo (``fedfomo/fedfomo_api.py:53-217``): after local training, client c weighs each candidate j by
    ``(L_val(theta_c^old) - L_val(theta_j)) / ||theta_j - theta_c^old||`` and moves to
    ``theta_c^old + sum_j w_j^+ (theta_j - theta_c^old) / sum w^+`` (its own new model stands in for j = c)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        N = self.N
        self.weights_locals = np.full((N, N), 1.0 / N)
        self.p_choose = np.ones((N, N))

    def choose(self, c):
        N, K = self.N, max(1, int(self.N * self.cfg.frac))
        if N == K:
            return list(range(N))
        p = self.p_choose[c]
        p[c] = 0
        if self.py_rng.random() >= 0.5:
            idx = np.argsort(p)[-K:]
        else:
            idx = self.np_rng.choice(range(N), K, replace=False)
            while c in idx:
                idx = self.np_rng.choice(range(N), K, replace=False)
        return sorted(int(j) for j in list(idx) + [c])

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        self._round_start(round_idx)
        last = self.snapshot()
        rows, loc = self.all_rows()
        self.train_rows(self.rowset, rows, loc, round_idx, self.cfg.epochs)
        self.stat_info["sum_training_flops"] += int(self.cfg.epochs * self.sizes.sum())
        self.end_of_training(round_idx, range(self.N))
        t1 = time.perf_counter()
        after_train = self.eval_local(self.rowset, rows, loc)
        nei = {c: self.choose(c) for c in range(self.N)}  # same generator sequence on every rank
        needs = [sorted({j for c in self.shards[r] for j in nei[c]}) for r in range(self.info.world)]
        src = self.fetch(needs, last)
        # candidate pool: [old own models (C) | new own models (C) | remote candidates]
        remote = [j for j in needs[self.info.rank] if j not in self.row_of]
        parts = [last.rows(0, self.C), self.rowset.rows(0, self.C)]
        if remote:
            parts.append(self.pool([src[j] for j in remote]).rows(0, len(remote)))
        pool = self.cat_rows(*parts)
        prow = {("old", c): self.row_of[c] for c in self.local}
        prow.update({("new", c): self.C + self.row_of[c] for c in self.local})
        for k, j in enumerate(remote):
            prow[("old", j)] = 2 * self.C + k
        # validation losses: (model row, client whose val split) pairs, grouped launches
        pairs = []
        for c in self.local:
            pairs.append((prow[("old", c)], c))
            for j in nei[c]:
                pairs.append((prow[("new", c)] if j == c else prow[("old", j)], c))
        which = "val" if getattr(self.splits[0], "val", None) is not None else "test"  # same rule on every rank
        met = self.eval_grouped(pool.theta, pool.bufs, [p for p, _ in pairs], [c for _, c in pairs], which)
        # parameter distances ||theta_j - theta_c^old|| over the whole state (params and buffers)
        dpairs = []
        for c in self.local:
            base = prow[("old", c)]
            for j in nei[c]:
                dpairs.append((prow[("new", c)] if j == c else prow[("old", j)], base))
        d2 = MK.pair_sqdist([(pool.theta[a], pool.theta[b]) for a, b in dpairs], self.P) + \
            MK.pair_sqdist([(pool.bufs[a], pool.bufs[b]) for a, b in dpairs], self.Q)
        d2 = d2.cpu().numpy()
        wl = np.zeros((self.N, self.N))
        k = kd = 0
        plan_t, plan_b = [], []
        for c in self.local:
            loss_cur = met[k, 1]
            k += 1
            w_row = self.weights_locals[c].copy()
            for j in nei[c]:
                lj = met[k, 1]
                k += 1
                dist = math.sqrt(max(float(d2[kd]), 0.0))
                kd += 1
                w_row[j] = 0.0 if dist == 0 else (loss_cur - lj) / dist
            wl[c] = w_row
        # every rank needs every client's new weight row (next round's neighbour choice): one all-reduce
        wl_all = torch.from_numpy(wl).to(self.device)
        rt.all_reduce_buckets(wl_all, self.info)
        wl_all = wl_all.cpu().numpy()
        self.weights_locals = wl_all
        self.p_choose = self.p_choose + wl_all
        new_t = {c: self.theta[self.row_of[c]] for c in self.local}
        new_b = {c: self.bufs[self.row_of[c]] for c in self.local}
        out = RowSet(padded_rows(max(1, self.C), self.P, self.device), padded_rows(max(1, self.C), self.Q, self.device))
        for c in self.local:
            i = self.row_of[c]
            wpos = np.maximum(self.weights_locals[c][nei[c]], 0)
            tot = float(np.sum(wpos))
            if tot == 0.0:  # no useful neighbour: keep the round-start model (fedfomo_api.py:204-205)
                plan_t.append((out.theta[i], [(last.theta[i], 1.0)]))
                plan_b.append((out.bufs[i], [(last.bufs[i], 1.0)]))
                continue
            a = wpos / tot
            terms_t = [(last.theta[i], 1.0 - float(a.sum()))]
            terms_b = [(last.bufs[i], 1.0 - float(a.sum()))]
            for j, aj in zip(nei[c], a):
                if aj == 0:
                    continue
                terms_t.append((new_t[c] if j == c else src[j][0], float(aj)))
                terms_b.append((new_b[c] if j == c else src[j][1], float(aj)))
            plan_t.append((out.theta[i], terms_t))
            plan_b.append((out.bufs[i], terms_b))
        MK.mix_rows(plan_t, self.P)
        MK.mix_rows(plan_b, self.Q)
        self.theta[:self.C].copy_(out.theta[:self.C])
        self.bufs[:self.C].copy_(out.bufs[:self.C])
        t2 = time.perf_counter()
        after_agg = self.eval_local(self.rowset, rows, loc)
        self.log_test(after_train, "old_mask_test_acc")
        acc, loss = self.log_test(after_agg, "person_test_acc")
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        self.timers["eval"] += time.perf_counter() - t2
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return {"person_test_acc": acc, "person_test_loss": loss}


# ================================================================================================== DisPFL
class DisPFLRunner(PersonalizedRunner):
    """Decentralized sparse personalized FL with dynamic masks (``DisPFL/dispfl_api.py:46-184``)."""

    def __init__(self, engine, splits, cfg, info, template_model, logger=None, algorithm="dispfl", mask_gen=None):
        super().__init__(engine, splits, cfg, info, template_model, logger, algorithm)
        params = {n: p.detach().cpu() for n, p in template_model.named_parameters()}
        N = self.N
        self.w_spa = [cfg.dense_ratio] * N
        gen = mask_gen if mask_gen is not None else torch.Generator().manual_seed(cfg.seed + 17)
        if not cfg.different_initial:
            base = SP.init_masks(params, _sparsities(params, cfg.dense_ratio, cfg), generator=gen)
            masks = [base] * N
        elif not cfg.diff_spa:
            masks = [SP.init_masks(params, _sparsities(params, cfg.dense_ratio, cfg), generator=gen) for _ in range(N)]
        else:
            p_divide = [0.2, 0.4, 0.6, 0.8, 1.0]
            masks = []
            for i in range(N):
                self.w_spa[i] = p_divide[i % 5]
                masks.append(SP.init_masks(params, _sparsities(params, p_divide[i % 5], cfg), generator=gen))
        flat = {c: self.flat_mask(masks[c]) for c in self.local}
        self.mbits = self.local_masks_from(flat)
        self.shared_bits = self.mbits.clone()  # mask_pers_shared: the mask each client last trained with
        # w_per = w_global * mask (every parameter is masked)
        if self.C:
            MK.masked_rows(self.theta[:self.C], self.mbits[:self.C], P=self.P)
        self.dist_locals = np.zeros((N, N))

    def benefit_choose(self, c, active):
        N, K = self.N, max(1, int(self.N * self.cfg.frac))
        if N == K:
            return list(range(N))
        # the reference forces cs = "random" (dispfl_api.py:201), drawing from the global numpy stream
        idx = self.np_rng.choice(range(N), min(K, N), replace=False)
        while c in idx:
            idx = self.np_rng.choice(range(N), min(K, N), replace=False)
        return [int(j) for j in idx]

    def run_round(self, round_idx, sync_timers=False):
        cfg = self.cfg
        t0 = time.perf_counter()
        self._round_start(round_idx)
        N = self.N
        active = self.np_rng.choice([0, 1], size=N, p=[1.0 - cfg.active, cfg.active])
        rows, loc = self.all_rows()
        # mask movement since the last round (hamming(shared_last[c], local[c])), K18 on device
        if self.C:
            moved = self.mspace.hamming(self.shared_bits[:self.C], self.mbits[:self.C]).sum(1).cpu().numpy()
            for j, c in enumerate(self.local):
                self.dist_locals[c][c] = moved[j]
        nei = {}
        for c in range(N):
            nb = [] if active[c] == 0 else self.benefit_choose(c, active)
            if N != max(1, int(N * cfg.frac)):
                nb = list(nb) + [c]
            nei[c] = sorted(int(j) for j in nb)
        last = self.snapshot() if cfg.dispfl_aggregate else None
        if cfg.dispfl_aggregate:
            self._aggregate_neighbours(nei, active, last)
        self.shared_bits.copy_(self.mbits)
        before = self.eval_local(self.rowset, rows, loc)  # test of w_local before training
        w_old = self.snapshot()
        spec = StepSpec(mask_mode=MASK_WEIGHT, bits=self.mbits[:self.C])
        self.train_rows(self.rowset, rows, loc, round_idx, cfg.epochs, spec)
        t1 = time.perf_counter()
        after = self.eval_local(self.rowset, rows, loc)
        if not cfg.static and self.C:
            drop = cfg.anneal_factor / 2 * (1 + np.cos((round_idx * np.pi) / cfg.comm_round))
            nnz = self.mspace.popcount(self.mbits[:self.C])
            k = torch.ceil(torch.tensor(drop, dtype=torch.float32) * nnz.float()).to(torch.int64)
            k = torch.minimum(k, nnz)
            self.mspace.select(MK.FIRE, self.theta, self.mbits, k.to(self.device))
            if not cfg.dis_gradient_check:
                self.local_grad(self.rowset, rows, loc, round_idx, bn_train=False)
                self.mspace.select(MK.REGROW_ABS, self.grads, self.mbits, k.to(self.device))
            else:
                self.mspace.select(MK.REGROW_RAND, None, self.mbits, k.to(self.device), cids=loc,
                                   seed=(cfg.seed << 20) + round_idx)
        upd = self.state_nonzeros(self.theta - w_old.theta, self.bufs - w_old.bufs, rows)
        self.add_comm(self.state_nonzeros(w_old.theta, w_old.bufs, rows) + upd, loc)
        self.end_of_training(round_idx, range(N))
        self.timers["train"] += t1 - t0
        t2 = time.perf_counter()
        acc, _ = self.log_test(after, "old_mask_test_acc")
        self.log_test(before, "new_mask_test_acc")
        self.stat_info["person_test_acc"].append(acc)
        self.timers["eval"] += time.perf_counter() - t2
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return {"person_test_acc": acc}

    def _aggregate_neighbours(self, nei, active, last):
        """The DisPFL paper's masked neighbour average (commented out in the reference, ``dispfl_api.py:138-142``):
        per coordinate, the mean over the neighbours whose shared mask keeps it, times the client's own mask; the
        buffers a plain neighbour mean.  One launch each for every local client (``masks.masked_mean_rows`` /
        ``mix_rows``), neighbour rows of other ranks fetched point-to-point."""
        needs = [sorted({j for c in self.shards[r] if active[c] for j in nei[c]}) for r in range(self.info.world)]
        src = self.fetch(needs, last)
        all_bits = self._all_bits(self.shared_bits)
        plan, bplan = [], []
        for c in self.local:
            if not active[c] or not nei[c]:
                continue
            i = self.row_of[c]
            plan.append((self.theta[i], self.mbits[i], [(src[j][0], all_bits[j]) for j in nei[c]]))
            bplan.append((self.bufs[i], [(src[j][1], 1.0 / len(nei[c])) for j in nei[c]]))
        MK.masked_mean_rows(plan, self.P)
        MK.mix_rows(bplan, self.Q)

    def _all_bits(self, bits):
        """[N, W] int32 mask bit rows of every client: ONE all-gather of each rank's own rows (their per-rank counts
        are known everywhere from the shard map, so no size exchange), placed by client id."""
        out = torch.zeros((self.N, self.W), dtype=torch.int32, device=self.device)
        mine = bits[:self.C].contiguous().view(-1) if self.C else torch.zeros(0, dtype=torch.int32, device=self.device)
        if self.info.enabled:
            sizes = [len(sh) * self.W for sh in self.shards]
            flat = rt.all_gather_sized(mine, sizes, self.info).view(-1, self.W)
            # each rank's rows are in its row order (size-sorted, ties by id: the rule of FLRunner.__init__/migrate)
            order = [c for sh in self.shards for c in sorted(sh, key=lambda c: (-int(self.sizes[c]), c))]
            out[self._to_dev(order)] = flat
        elif self.C:
            out[self._to_dev(self.local)] = mine.view(self.C, self.W)
        return out

    def finish(self):
        all_bits = self._all_bits(self.mbits)
        # [N, N] Hamming matrix on device, a chunk of rows per launch, one device->host copy at the end
        N, ch = self.N, max(1, min(self.N, (1 << 26) // max(1, self.N * self.W)))
        mat = torch.empty((N, N), dtype=torch.int64, device=self.device)
        for i0 in range(0, N, ch):
            i1 = min(N, i0 + ch)
            a = all_bits[i0:i1].unsqueeze(1).expand(i1 - i0, N, self.W).reshape(-1, self.W)
            b = all_bits.unsqueeze(0).expand(i1 - i0, N, self.W).reshape(-1, self.W)
            mat[i0:i1] = self.mspace.hamming(a.contiguous(), b.contiguous()).sum(1).view(i1 - i0, N).to(torch.int64)
        self.stat_info["mask_dis_matrix"] = mat.cpu().tolist()
        if self.cfg.save_masks:
            self.stat_info["final_masks"] = MK.unpack_bits(all_bits, self.P).bool().cpu()
        return super().finish()  # folds the device-side counters (sum_comm_params) into stat_info


# ================================================================================================== SubAvg
class SubAvgRunner(PersonalizedRunner):
    """Sub-FedAvg unstructured pruning (``subavg/subavg_api.py:43-139``, ``subavg/client.py:36-63``)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.mbits = MK.pack_bits(torch.ones((max(1, self.C), self.P), device=self.device))
        names = self.e.players.names
        self.prune_names = [n for n in names if "weight" in n and "bn" not in n]  # prune_func.py:23

    def finish(self):
        # subavg_api.py:91: w_global under every client's personal mask (the whole federation, every rank's rows)
        self.record_avg_inference_flops(self.mbits[:self.C] if self.C else self.mbits[:0])
        return super().finish()

    def _record_subavg(self, round_idx, r):
        sl = dict.__getitem__  # the raw lists (called from the metric flush too)
        acc, loss = self.mean_acc_loss(r)
        sl(self.stat_info, "test_acc").append(acc)
        sl(self.stat_info, "person_test_acc").append(acc)
        if self.log is not None and self.info.is_main:
            self.log.info({"test_acc": acc, "test_loss": loss})
        return {"test_acc": acc, "test_loss": loss}

    def _real_prune_rows(self, rs, rows, bits_rows):
        ix = self._to_dev(rows)
        t = rs.theta[ix]
        rs.theta[ix] = MK.masked_rows(t, bits_rows, P=self.P)

    def run_round(self, round_idx, sync_timers=False):
        cfg = self.cfg
        t0 = time.perf_counter()
        self._round_start(round_idx)
        sampled = self.sample_clients(round_idx)
        self.rebalance(sampled)
        rows, loc = self._local_rows(sampled)
        hooks = {}
        if rows:
            ix = self._to_dev(rows)
            old_bits = self.mbits[ix].clone()
            self.theta[ix] = self.w_global.unsqueeze(0).expand(len(rows), -1)
            self.bufs[ix] = self.b_global.unsqueeze(0).expand(len(rows), -1)
            self._real_prune_rows(self.rowset, rows, old_bits)  # w_per = real_prune(w_global, mask)
            nz_dev = self.state_nonzeros(self.theta, self.bufs, rows)  # print_pruning over the whole state
            self.add_comm(nz_dev)

            # [late prune] NIDT_SUBAVG_LATE_PRUNE=1 (default) keeps an fp32 copy of every trained row's parameters from
            # the end of epoch 0 until after training (rows x P x 4 B: ~450 MB for ResNet-18 at frac 0.1); it is
            # skipped (the epoch-0 prune runs in training, with its host read) when that copy would exceed a quarter
            # of the free device memory or NIDT_SUBAVG_LATE_PRUNE_GB (default 8)
            late = os.environ.get("NIDT_SUBAVG_LATE_PRUNE", "1") != "0"
            if late and self.device.type == "cuda":
                need = len(rows) * self.theta.stride(0) * 4
                cap = float(os.environ.get("NIDT_SUBAVG_LATE_PRUNE_GB", "8")) * 2 ** 30
                late = need <= min(cap, torch.cuda.mem_get_info(self.device)[0] / 4)

            def hook(ep, view, clients):  # fake_prune after the first and the last epoch (the training masks)
                if ep == 0 and cfg.epochs > 1 and not late:
                    hooks["m1"] = self.mspace.percentile_prune(view.theta, old_bits, cfg.each_prune_ratio,
                                                               self.prune_names)
                elif ep == 0 and cfg.epochs > 1:
                    # the first epoch's weights are kept and pruned after training: the percentile search reads
                    # its thresholds on the host, which in mid-training drained the device between epochs
                    hooks["t1"] = view.theta.clone()
                if ep == cfg.epochs - 1:
                    hooks["m2"] = self.mspace.percentile_prune(view.theta, old_bits, cfg.each_prune_ratio,
                                                               self.prune_names)
            spec = StepSpec(mask_mode=MASK_GRAD, bits=self.mbits)
            self.train_rows(self.rowset, rows, loc, round_idx, cfg.epochs, spec, epoch_hook=hook)
            m2 = hooks["m2"]
            m1 = hooks.get("m1")
            if m1 is None:
                m1 = (self.mspace.percentile_prune(hooks.pop("t1"), old_bits, cfg.each_prune_ratio, self.prune_names)
                      if cfg.epochs > 1 else m2)
            # one host read after training for both (a read before it drained the device at every round start)
            hd = torch.cat([nz_dev.double().view(-1, 1), self.mspace.hamming(m1, m2).double()], 1).cpu().numpy()
            dense, ham = hd[:, 0] / float(self.P + self.Q), hd[:, 1:]
            dist = (ham / self.mspace.seg_len[None, :]).mean(1)  # mean over every parameter (scipy hamming)
            cand = [j for j in range(len(rows)) if dist[j] > cfg.dist_thresh and dense[j] > cfg.dense_ratio]
            final_bits = old_bits.clone()
            if cand:
                pr = self.pool([(self.theta[rows[j]], self.bufs[rows[j]]) for j in cand])
                cb = torch.stack([m2[j] for j in cand])
                MK.masked_rows(pr.theta[:len(cand)], cb, P=self.P)
                met = self.eval_grouped(pr.theta, pr.bufs, list(range(len(cand))), [loc[j] for j in cand], "train")
                for q, j in enumerate(cand):
                    if met[q, 0] / max(1.0, met[q, 2]) > cfg.acc_thresh:
                        self.theta[rows[j], :self.P].copy_(pr.theta[q, :self.P])
                        final_bits[j] = m2[j]
            self.add_comm(self.state_nonzeros(self.theta, self.bufs, rows))
        t1 = time.perf_counter()
        self.end_of_training(round_idx, sampled)
        # masked average with the masks the clients trained with (subavg_api.py:123-139)
        s = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        cnt = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        sb = torch.zeros(self.Q, dtype=torch.float32, device=self.device)
        cb = torch.zeros(self.Q, dtype=torch.float32, device=self.device)
        if rows:
            sc = self._scratch_rows(len(rows))
            sc.theta[:len(rows)].copy_(self.theta[ix])
            sc.bufs[:len(rows)].copy_(self.bufs[ix])
            MK.masked_rows_sum(sc.theta[:len(rows)], self.P, old_bits, s, cnt)
            MK.masked_rows_sum(sc.bufs[:len(rows)], self.Q, None, sb, cb)
        red = torch.cat([s, cnt, sb, cb])
        rt.all_reduce_buckets(red, self.info)
        s, cnt, sb, cb = red.split([self.P, self.P, self.Q, self.Q])
        self.w_global.copy_(torch.where(cnt > 0, s / cnt, self.w_global))
        self.b_global.copy_(torch.where(cb > 0, sb / cb, self.b_global))
        t2 = time.perf_counter()
        res = None
        if self._eval_due(round_idx):  # every client tests real_prune(w_global, its current mask)
            er = self._eval_buffers(max(1, self.C))
            th, bu = er
            bu.copy_(self.b_global.expand_as(bu))
            if self.C:  # w_global * mask_c in one pass (masks.masked_rows)
                MK.masked_rows(th[:self.C], self.mbits[:self.C], src=self.w_global[:self.P])
                if th.shape[1] > self.P:
                    th[:self.C, self.P:].copy_(self.w_global[self.P:].expand(self.C, -1))
            th[self.C:].copy_(self.w_global.expand_as(th[self.C:]))
            if self._defer_metrics():  # read one round late (no end-of-round device drain; see FLRunner.evaluate)
                self._flush_metrics(ready_only=True)
                rows_e, clients_e = self.all_rows()
                loc = (self.eval_grouped(th, bu, rows_e, clients_e, "test", device_out=True) if rows_e
                       else torch.zeros((0, 3), dtype=torch.float64, device=self.device))
                res = self._defer_result(round_idx, self.gather_metrics(clients_e, loc, device_out=True),
                                         self._record_subavg)
            else:
                res = self._record_subavg(round_idx, self.eval_local(RowSet(th, bu), *self.all_rows()))
        if rows:
            self.mbits[ix] = final_bits
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        self.timers["eval"] += time.perf_counter() - t2
        self.stat_info["sum_training_flops"] += int(cfg.epochs * sum(self.sizes[c] for c in sampled))
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return res


RUNNERS = {"dispfl": DisPFLRunner, "subavg": SubAvgRunner, "ditto": DittoRunner, "dpsgd": DPSGDRunner,
           "fedfomo": FedFomoRunner, "local": LocalRunner}


def make_runner(algorithm, engine, splits, cfg, info, template_model, logger=None, **kw):
    """Runner of any algorithm of the harness on the client-batched executor."""
    if algorithm in RUNNERS:
        return RUNNERS[algorithm](engine, splits, cfg, info, template_model, logger, algorithm=algorithm, **kw)
    alg = {"sailentgrads": "salientgrads", "salientgrads": "salientgrads", "fedavg": "fedavg",
           "fedprox": "fedavg"}[algorithm]
    return FLRunner(engine, splits, cfg, info, template_model, logger, algorithm=alg)
