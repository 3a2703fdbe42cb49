"""Client-batched FL runner: many virtual clients per GPU, one process per GPU, RCCL collectives.

This replaces the reference's sequential client loop (``sailentgrads_api.py:86-147``, ``fedavg_api.py:40-88``):
instead of swapping one shared ``nn.Module``'s state_dict per client and copying weights host<->device, every rank
keeps its clients resident as rows of ``theta [C_local, P]`` (params) and ``bufs [C_local, Q]`` (BN running stats)
and trains all of them in lockstep — one launch sequence (or one replayed hipGraph) per local step.

Layout decisions that keep every launch dense:

* rows are ordered by training-set size (descending).  At local step ``s`` the clients whose batch has the same
  size (full batches, then each partial last-batch size) therefore form *contiguous* row ranges, so ragged
  federations (unequal sites, ``drop_last=False`` partial batches, ``ABCD/data_loader.py:195``) train without
  gather/scatter copies and keep hipGraph capture;
* a round that trains a subset of the local rows (``frac < 1``) gathers them once into a scratch row set, trains
  there and scatters back (one copy per round, not per step);
* everything a step needs besides its launch arguments lives on device (sample indices, learning rate, dropout
  counter), so steps replay as hipGraphs;
* the optimizer is one fused kernel for every algorithm (``StepSpec``): shared or per-client bit masks applied to
  weights (SalientGrads / DisPFL) or gradients (SubAvg), FedProx's proximal gradient and Ditto's personal pull.

Round semantics reproduced from the reference (SURVEY.md §2.2 "Shared algorithm behaviors"):
* sampling ``np.random.seed(round); choice(total, per_round, replace=False)`` (all if frac = 1);
* every sampled client starts from ``w_global``; SGD(lr * lr_decay**round, momentum, wd) rebuilt per round
  (momentum rows are zeroed at the start of each local training, Q4); ``clip_grad_norm_(10)``;
* one DataLoader(shuffle=True) pass per epoch over the client's train split (last batch may be partial);
* aggregation: sample-weighted average over ALL state entries incl. BN running stats and
  ``num_batches_tracked`` (Q3) — a local weighted row-sum followed by ONE all-reduce of P+Q floats;
* evaluation: global model and each client's last local ("personal") model on that client's test split;
  logged loss uses sigmoid-then-BCEWithLogits (Q1); metrics are unweighted means over clients (Q5).
The personalized / decentralized algorithms build on this class (``engine/personalized.py``).
"""
from __future__ import annotations

import gc
import math
import os
import time
from dataclasses import dataclass, replace

from collections.abc import Mapping

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..parallel import runtime as rt
from . import masks as MK
from .executor import (ClientSplit, FLConfig, gather_rows, maskable_flat_mask, padded_rows,  # noqa: F401
                       snip_maskable_names)

MASK_NONE, MASK_WEIGHT, MASK_GRAD = 0, 1, 2


@dataclass
class StepSpec:
    """What the fused optimizer does after each local step (see ``optim.hip`` ``local_opt``)."""
    mask_mode: int = MASK_NONE
    bits: torch.Tensor = None      # [R, W] bit rows aligned with the trained rows, or [1, W] when ``shared``
    shared: bool = False
    prox_mu: float = 0.0           # FedProx: g += mu (w - ref)
    ref: torch.Tensor = None       # [P] shared reference row
    lamda: float = 0.0             # Ditto: w -= lr lamda (w - pref) after the step
    pref: torch.Tensor = None      # [P] shared pull reference

    def rows(self, lo, hi):
        if self.bits is None or self.shared:
            return self
        return replace(self, bits=self.bits[lo:hi])

    def key(self):
        return (self.mask_mode, None if self.bits is None else (self.bits.data_ptr(), self.shared), self.prox_mu,
                None if self.ref is None else self.ref.data_ptr(), self.lamda,
                None if self.pref is None else self.pref.data_ptr())


@dataclass
class RowSet:
    theta: torch.Tensor            # [R, P] fp32 (16-B aligned row stride)
    bufs: torch.Tensor             # [R, Q]

    def rows(self, lo, hi):
        return RowSet(self.theta[lo:hi], self.bufs[lo:hi])


class StatInfo(dict):
    """``stat_info`` whose evaluation lists may trail the device by a round: reads first fold in the evaluations
    still in flight (:meth:`FLRunner._flush_metrics`), so every consumer sees the complete, ordered lists while a timed
    GPU loop never waits for a metric."""

    DEFERRED = ("global_test_acc", "global_test_loss", "person_test_acc", "person_test_loss", "test_acc")

    def __init__(self, flush, *a, **kw):
        super().__init__(*a, **kw)
        self._flush = flush

    def __getitem__(self, k):
        if k in self.DEFERRED:  # other keys (round_time, counters) never wait for the device
            self._flush()
        return super().__getitem__(k)

    def get(self, k, default=None):
        if k in self.DEFERRED:
            self._flush()
        return super().get(k, default)

    def items(self):
        self._flush()
        return super().items()

    def values(self):
        self._flush()
        return super().values()

    def __iter__(self):
        self._flush()
        return super().__iter__()

    def copy(self):
        self._flush()
        return dict(super().items())

    def __reduce__(self):
        self._flush()
        return (dict, (dict(super().items()),))


class LazyMetrics(Mapping):
    """A round's evaluation result that is read from the device only when looked at."""

    def __init__(self, runner, holder):
        self._runner, self._holder = runner, holder

    def _d(self):
        if "res" not in self._holder:
            self._runner._flush_metrics()
        return self._holder["res"]

    def __getitem__(self, k):
        return self._d()[k]

    def __iter__(self):
        return iter(self._d())

    def __len__(self):
        return len(self._d())

    def __repr__(self):
        return repr(self._d())


def _nullctx():
    import contextlib
    return contextlib.nullcontext()


def _contiguous(rows):
    return bool(rows) and rows == list(range(rows[0], rows[-1] + 1))


class FLRunner:
    """SalientGrads / FedAvg / FedProx over client-sharded, client-batched local training (and the base of the
    personalized runners)."""

    def __init__(self, engine, splits, cfg: FLConfig, info: rt.DistInfo, template_model, logger=None,
                 algorithm="salientgrads"):
        self.e, self.cfg, self.info, self.log = engine, cfg, info, logger
        self.alg = algorithm
        self.N = len(splits)
        self.splits = splits
        self.device = info.device
        self.sizes = np.array([len(s.train) for s in splits], dtype=np.int64)
        self.shards = rt.shard_clients(list(self.sizes), info.world)
        # rows ordered by train size (desc), ties by client id: equal-size step groups are contiguous row ranges
        self.local = sorted(self.shards[info.rank], key=lambda c: (-int(self.sizes[c]), c))
        self.row_of = {c: i for i, c in enumerate(self.local)}
        self.owner = np.zeros(self.N, dtype=np.int64)
        for r, sh in enumerate(self.shards):
            self.owner[list(sh)] = r
        self.C = len(self.local)
        P, Q = engine.players.total, engine.blayers.total
        self.P, self.Q = P, Q
        self.W = MK.mask_words(P)
        with torch.no_grad():
            flat_p = engine.players.flatten_state(dict(template_model.named_parameters()), self.device).detach()
            flat_b = engine.blayers.flatten_state(dict(template_model.named_buffers()), self.device).detach()
        self.w_global = flat_p.clone()
        self.b_global = flat_b.clone()
        nrow = max(1, self.C)
        self.theta = padded_rows(nrow, P, self.device)
        self.theta.copy_(flat_p.unsqueeze(0).expand(nrow, P))
        self.bufs = padded_rows(nrow, Q, self.device)
        self.bufs.copy_(flat_b.unsqueeze(0).expand(nrow, Q))
        self.grads = padded_rows(nrow, P, self.device)
        self.mom_buf = padded_rows(nrow, P, self.device) if cfg.momentum != 0 else None
        self.mask = None              # SalientGrads global mask, float [P]
        self.mask_bits = None         # the same as one shared bit row [1, W]
        self.maskable = maskable_flat_mask(engine.players, snip_maskable_names(template_model)).to(self.device)
        self.template = template_model   # layer structure for FLOP accounting (its weights are not used)
        self._pending_metrics = []     # deferred evaluations: (round, pinned host rows, event, result holder)
        self._pinned_free = []
        self.stat_info = StatInfo(self._flush_metrics, sum_comm_params=0, sum_training_flops=0, global_test_acc=[],
                                  person_test_acc=[], global_test_loss=[], person_test_loss=[], round_time=[])
        self.timers = {"train": 0.0, "aggregate": 0.0, "eval": 0.0, "snip": 0.0}
        self._graphs = {}             # step key -> captured local step (None until the shape repeats, False = eager)
        self.graph_stats = {}         # counts of first-seen (eager) / captured / replayed steps
        # captured steps kept (LRU); engines whose graphs own their activation memory (torch-allocated, e.g. the
        # ResNet engine) set a small limit, the AlexNet engine's graphs only reference its persistent buffers
        self.max_graphs = int(getattr(engine, "graph_cache_limit", 512))
        self.record_train_events = False  # bench: CUDA events around every local-training call (no host syncs)
        self.train_events = []
        self._lr_dev = self._seed_dev = None
        self._scratch = None
        self._eval_cache = None
        # reference training log (``Client Index = c\tEpoch: e\tLoss: l``, ``my_model_trainer.py:234-235``) and the
        # communication accounting (``count_communication_params``, ``sailentgrads/client.py:82,100``): per-step
        # losses are summed into a device row buffer inside the (captured) step and snapshotted per epoch, the
        # non-zero counts are device reductions — nothing syncs the host until a round's lines are logged
        self.track_loss = logger is not None
        self._loss_acc = None
        self._loss_log = {}           # client -> [device tensor of per-epoch mean losses, one per training call]
        self._comm_log = {}           # client -> device scalar (downlink + uplink non-zeros of this round)
        self._comm_dev = None         # device int64 sum of every counted client (this rank)

    # ---------------------------------------------------------------------------------------------- helpers
    def _rng(self, *key):
        return np.random.RandomState(abs(hash((self.cfg.seed,) + tuple(int(k) for k in key))) % (2 ** 31))

    def _groups(self, items):
        gmax = self.cfg.group or len(items)
        return [items[i:i + gmax] for i in range(0, len(items), gmax)]

    def _upload_i32(self, arr):
        """int32 host array -> device tensor through pinned memory, without blocking the host."""
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32))
        if self.device.type != "cuda":
            return t
        return t.pin_memory().to(self.device, non_blocking=True)

    def _to_dev(self, arr, dtype=torch.int64):
        """Small host list / array -> device tensor through pinned memory, without blocking the host.  (A plain
        ``torch.tensor(..., device=cuda)`` copies from pageable memory and synchronises the stream: the host then
        waits for all queued GPU work, e.g. the whole local training before the aggregation is enqueued.)"""
        t = torch.as_tensor(np.asarray(arr), dtype=dtype)
        if self.device.type != "cuda":
            return t
        return t.pin_memory().to(self.device, non_blocking=True)

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize()

    def _step_seed(self, round_idx, tag, ep, s):
        """Dropout stream position of one local step: a function of (round, training tag, epoch, step) only, so it
        does not depend on how clients are grouped or sharded (client ids key the per-client streams)."""
        return ((((round_idx + 2) * 64 + tag) * 64 + ep) * 8192 + s) & ((1 << 40) - 1)

    def _order(self, c, round_idx, tag, ep):
        """Sample order of one epoch of client c (DataLoader(shuffle=True))."""
        tr = self.splits[c].train
        return tr[self._rng(round_idx, c, tag, ep).permutation(len(tr))]

    def _stratified_batch(self, c, it, B):
        """A label-stratified mini-batch of client c (IterSNIP ``--stratified_sampling``): per class
        round(B * n_class / n) samples (largest remainders), drawn without replacement."""
        from ..algorithms.snip import stratified_batch, stratified_rng
        tr = self.splits[c].train
        y = self.e.labels.index_select(0, torch.as_tensor(tr, dtype=torch.long).to(self.e.labels.device))
        return stratified_batch(tr, y.cpu().numpy(), B, stratified_rng(self.cfg.seed, c, it))

    # ---------------------------------------------------------------------------------------------- planning
    def _plan(self, clients, chunks_of):
        """Lockstep launch plan over clients listed in row order.  ``chunks_of(j, c)`` -> list of per-step index
        arrays of client j.  Returns (plan, idx) where plan items are (r0, r1, step, offset, n, G, B) with rows
        relative to the listed clients and all sample indices uploaded in ONE pinned non-blocking copy."""
        chunks = [chunks_of(j, c) for j, c in enumerate(clients)]
        nsteps = max((len(ch) for ch in chunks), default=0)
        plan, flat, off = [], [], 0
        for s in range(nsteps):
            run = None
            items = []
            for j, ch in enumerate(chunks):
                if s < len(ch) and len(ch[s]):
                    items.append((j, ch[s]))
            # contiguous runs of equal batch size (rows are size sorted, so equal sizes are adjacent)
            runs = []
            for j, ch in items:
                if run and run[-1][0] == j - 1 and len(run[-1][1]) == len(ch):
                    run.append((j, ch))
                else:
                    run = [(j, ch)]
                    runs.append(run)
            for run in runs:
                for grp in self._groups(run):
                    n = sum(len(ch) for _, ch in grp)
                    plan.append((grp[0][0], grp[-1][0] + 1, s, off, n, len(grp), len(grp[0][1])))
                    flat.extend(ch for _, ch in grp)
                    off += n
        if not plan:
            return [], None
        return plan, self._upload_i32(np.concatenate(flat))

    def _epoch_chunks(self, round_idx, tag, ep, n_batches=None):
        B = self.cfg.batch_size

        def f(j, c):
            o = self._order(c, round_idx, tag, ep)
            ch = [o[i:i + B] for i in range(0, len(o), B)]
            return ch[:n_batches] if n_batches is not None else ch
        return f

    # ---------------------------------------------------------------------------------------------- training
    def _scratch_rows(self, k):
        if self._scratch is None or self._scratch.theta.shape[0] < k:
            n = max(k, self.C, 1)
            self._scratch = RowSet(padded_rows(n, self.P, self.device), padded_rows(n, self.Q, self.device))
            self._scratch_bits = torch.zeros((n, self.W), dtype=torch.int32, device=self.device)
            self._graphs = {}
        return self._scratch

    def _zero_mom(self, k):
        if self.mom_buf is not None:
            self.mom_buf[:k].zero_()

    def train_rows(self, rs, rows, clients, round_idx, epochs, spec=None, tag=0, epoch_hook=None, lr=None):
        """Local SGD (``epochs`` DataLoader passes) of ``clients`` living in rows ``rows`` of row set ``rs`` (rows
        listed in increasing order = the size-sorted row order).  ``epoch_hook(ep, view, clients)`` runs after every
        epoch on the rows being trained."""
        if not rows:
            return
        spec = spec or StepSpec()
        if self.record_train_events and self.device.type == "cuda":  # per-rank GPU time of local training (bench)
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            self._train_rows(rs, rows, clients, round_idx, epochs, spec, tag, epoch_hook, lr)
            ev[1].record()
            self.train_events.append(ev)
            return
        self._train_rows(rs, rows, clients, round_idx, epochs, spec, tag, epoch_hook, lr)

    def _train_rows(self, rs, rows, clients, round_idx, epochs, spec, tag, epoch_hook, lr):
        if _contiguous(rows):
            lo, hi = rows[0], rows[-1] + 1
            self._train_view(rs.rows(lo, hi), clients, round_idx, epochs, spec.rows(lo, hi), tag, epoch_hook, lr)
            return
        ix = self._to_dev(rows)
        k = len(rows)
        sc = self._scratch_rows(k)
        view = sc.rows(0, k)
        view.theta.copy_(rs.theta.index_select(0, ix))
        view.bufs.copy_(rs.bufs.index_select(0, ix))
        sspec = spec
        if spec.bits is not None and not spec.shared:
            self._scratch_bits[:k].copy_(spec.bits.index_select(0, ix))
            sspec = replace(spec, bits=self._scratch_bits[:k])
        self._train_view(view, clients, round_idx, epochs, sspec, tag, epoch_hook, lr)
        rs.theta[ix] = view.theta
        rs.bufs[ix] = view.bufs
        if spec.bits is not None and not spec.shared:
            spec.bits[ix] = self._scratch_bits[:k]  # epoch hooks may have changed the trained masks

    def _train_view(self, view, clients, round_idx, epochs, spec, tag, epoch_hook, lr):
        cfg = self.cfg
        lr = cfg.lr * (cfg.lr_decay ** round_idx) if lr is None else lr
        self._zero_mom(len(clients))
        hg = cfg.hip_graphs
        if hg is None:  # the engine's measured default, per trained row set where it depends on the launch size
            f = getattr(self.e, "graphs_default_for", None)
            hg = f(len(clients)) if f is not None else getattr(self.e, "graphs_default", True)
        use_graphs = (hg and getattr(self.e, "supports_graphs", False) and self.device.type == "cuda"
                      and os.environ.get("NIDT_HIP_GRAPHS", "1") != "0")  # NIDT_HIP_GRAPHS=0: eager steps (A/B)
        if self._lr_dev is None:
            self._lr_dev = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._seed_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._lr_dev.fill_(lr)
        side = self._side_streams() if use_graphs else None
        # client ids of the view's rows on the device: captured steps read a group's ids from a static buffer
        # refilled before each replay, so a graph serves any clients at the same rows (sampled rounds reuse the
        # previous rounds' captures instead of capturing every round)
        cdev = (self._upload_i32([int(c) for c in clients])
                if use_graphs and getattr(self.e, "accepts_cids_dev", False) else None)
        k = len(clients)
        sums = [] if self.track_loss else None
        if sums is not None:
            self._loss_rows(k)[:k].zero_()
        for ep in range(epochs):
            plan, idx = self._plan(clients, self._epoch_chunks(round_idx, tag, ep))
            main, cur, lanes_used = torch.cuda.current_stream() if side else None, -1, set()
            partial_steps = {it[2] for it in plan if it[6] < cfg.batch_size} if side else ()
            # [PACK-FUSE] engines whose optimizer can write the next step's weight images: eager steps always, captured
            # steps when the engine keeps the two variants (prepacked or not) as separate graphs
            pnext = (self._pack_next(plan) if not use_graphs or getattr(self.e, "fused_pack_graphs", False)
                     else None)
            fresh = set()  # row groups whose previous step (this epoch) wrote their images
            for pi, (r0, r1, s, off, n, G, B) in enumerate(plan):
                pn = bool(pnext and pnext[pi])
                pre = r0 in fresh
                fresh.discard(r0)
                if pn:
                    fresh.add(r0)
                if s != cur:  # fork point of this step: main has enqueued every earlier step
                    cur = s
                    fork = main.record_event() if s in partial_steps else None
                seed = self._step_seed(round_idx, tag, ep, s)
                cids = clients[r0:r1]
                sub = view.rows(r0, r1)
                if side and B < cfg.batch_size:
                    # a partial last batch: these clients are done with the epoch after this launch, so it runs
                    # on a side lane, overlapped with the following full-batch steps (see _lane)
                    st, sdev = self._lane(G, B)
                    st.wait_event(fork)
                    lanes_used.add(st)
                    with torch.cuda.stream(st):
                        sdev.fill_(seed)
                        self._graph_step(sub, r0, idx[off:off + n], G, B, spec.rows(r0, r1), cids, seed, fill=False,
                                         seed_dev=sdev, cids_dev=None if cdev is None else cdev[r0:r1])
                elif use_graphs:
                    self._graph_step(sub, r0, idx[off:off + n], G, B, spec.rows(r0, r1), cids, seed,
                                     cids_dev=None if cdev is None else cdev[r0:r1], prepacked=pre, pack_next=pn)
                else:
                    self._seed_dev.fill_(seed)
                    self._step(sub, r0, idx[off:off + n], G, B, spec.rows(r0, r1), cids, lr, pack_next=pn,
                               prepacked=pre)
            for st in lanes_used:
                main.wait_stream(st)
            self.concurrent_steps = getattr(self, "concurrent_steps", 0) + len(lanes_used)
            if sums is not None:
                sums.append(self._loss_acc[:k].clone())
                self._loss_acc[:k].zero_()
            if epoch_hook is not None:
                epoch_hook(ep, view, clients)
        if sums:
            B = cfg.batch_size
            nb = self._to_dev([max(1, -(-len(self.splits[c].train) // B)) for c in clients], torch.float32)
            means = torch.stack(sums, 1) / nb.view(-1, 1)   # mean batch loss per (client, epoch), as logged
            for j, c in enumerate(clients):
                self._loss_log.setdefault(int(c), []).append(means[j])

    def _side_streams(self):
        if self.cfg.step_streams <= 1:
            return None
        if getattr(self, "_streams", None) is None:
            self._streams = [torch.cuda.Stream(device=self.device) for _ in range(self.cfg.step_streams)]
            self._lane_seed = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in self._streams]
        return self._streams

    def _loss_rows(self, k):
        """Device accumulator of the per-client training-loss sums of the current epoch (row = position in the
        trained client list).  Captured steps add into it, so growing it drops the captured steps."""
        if self._loss_acc is None or self._loss_acc.shape[0] < k:
            self._loss_acc = torch.zeros(max(k, self.C, 1), dtype=torch.float32, device=self.device)
            self._graphs = {}
        return self._loss_acc

    # ---------------------------------------------------------------------------------------------- statistics
    def state_nonzeros(self, theta, bufs, rows):
        """``count_communication_params`` of whole states (every state_dict entry: params and buffers) per row, as
        a device int64 tensor."""
        if not rows:
            return torch.zeros(0, dtype=torch.int64, device=self.device)
        if _contiguous(rows):
            th, bu = theta[rows[0]:rows[-1] + 1, :self.P], bufs[rows[0]:rows[-1] + 1, :self.Q]
        else:
            ix = self._to_dev(rows)
            th, bu = gather_rows(theta, ix)[:, :self.P], gather_rows(bufs, ix)[:, :self.Q]
        return self._rows_nnz(th) + self._rows_nnz(bu)

    def _rows_nnz(self, mat):
        """Non-zeros per row of a [R, K] fp32 row view: the HIP row counter on aligned device rows, else torch."""
        R, K = mat.shape
        if (self.device.type == "cuda" and R and K and mat.stride(1) == 1 and (R == 1 or mat.stride(0) % 4 == 0)
                and mat.data_ptr() % 16 == 0 and mat.dtype == torch.float32):
            m = ops.ext()
            part = torch.empty((R, m.rows_nnz_blocks(K)), dtype=torch.int32, device=self.device)
            m.rows_nnz(mat.data_ptr(), R, K, mat.stride(0) if R > 1 else (K + 3) // 4 * 4, part.data_ptr(),
                       ops.stream())
            return part.sum(1, dtype=torch.int64)
        return torch.count_nonzero(mat, dim=1)

    def add_comm(self, per_client, clients=None):
        """Add communication counts (device int64 per client, or a host int) to ``sum_comm_params`` — kept on
        device and summed over ranks when the statistics are read (:meth:`sync_stats`)."""
        if self._comm_dev is None:
            self._comm_dev = torch.zeros((), dtype=torch.int64, device=self.device)
        if torch.is_tensor(per_client):
            self._comm_dev += per_client.sum().to(torch.int64)
            if clients is not None and self.log is not None:
                for j, c in enumerate(clients):
                    self._comm_log[int(c)] = per_client[j]
        else:
            self._comm_dev += int(per_client)

    def sync_stats(self):
        """Fold the device-side counters into ``stat_info`` (a collective on multi-rank runs: every rank calls it
        at the same points — the end of a logged round, ``finish``, checkpoints)."""
        if self._comm_dev is None:
            self._comm_dev = torch.zeros((), dtype=torch.int64, device=self.device)
        t = self._comm_dev.view(1).clone()
        rt.all_reduce_buckets(t, self.info)
        self.stat_info["sum_comm_params"] += int(t.item())
        self._comm_dev.zero_()
        return self.stat_info

    def record_avg_inference_flops(self, mask_bits=None):
        """``stat_info["avg_inference_flops"]``: mean over ALL clients of the sparse-aware inference FLOPs of
        ``w_global`` under each client's personal mask (``mask_bits`` [C, W] of this rank's clients; collective) or
        of ``w_global`` alone (``subavg_api.py:223-235``, ``ditto/ditto_api.py:78,153``)."""
        from ..utils.records import flop_coefficients, sparse_inference_flops
        coef = flop_coefficients(self.template, input_shape=getattr(self.e, "input_shape", None))
        lay = self.e.players
        if mask_bits is None:  # every client runs w_global
            avg = float(sparse_inference_flops(coef, lay, self.w_global.view(1, -1))[0])
        else:
            tot = torch.zeros(1, dtype=torch.float64, device=self.device)
            for j in range(self.C):  # one client row at a time: [P] temporaries only
                row = self.w_global.view(1, -1) * MK.unpack_bits(mask_bits[j:j + 1], self.P)
                tot += sparse_inference_flops(coef, lay, row)
            rt.all_reduce_buckets(tot, self.info)
            avg = float(tot.item()) / self.N
        self.stat_info["avg_inference_flops"] = avg
        return avg

    def flush_round_log(self, round_idx, clients, comm_lines=True):
        """Emit the reference's per-client training lines for this round (rank 0, reference order):
        ``@@@@@@@@@@@@@@@@ Training Client CM(r): c``, ``Client Index = c\tEpoch: e\tLoss: l`` per epoch and
        ``communication parameters for search n`` (``sailentgrads_api.py:127``, ``my_model_trainer.py:234``,
        ``client.py:101``).  No-op without a logger; one device->host copy (and one gather on multi-rank runs)."""
        if self.log is None:
            self._loss_log, self._comm_log = {}, {}
            return
        recs = []
        for c in sorted(self._loss_log):
            ls = torch.cat([v.view(-1) for v in self._loss_log[c]]).double()
            cm = self._comm_log.get(c)
            cm = cm.double().view(1) if cm is not None else torch.full((1,), -1.0, dtype=torch.float64,
                                                                      device=self.device)
            recs.append(torch.cat([torch.tensor([float(c), float(ls.numel())], dtype=torch.float64,
                                                device=self.device), ls, cm]))
        flat = torch.cat(recs) if recs else torch.zeros(0, dtype=torch.float64, device=self.device)
        flat = rt.all_gather_cat(flat, self.info).cpu().numpy()
        self._loss_log, self._comm_log = {}, {}
        if not self.info.is_main:
            return
        per, o = {}, 0
        while o < flat.size:
            c, n = int(flat[o]), int(flat[o + 1])
            per[c] = (flat[o + 2:o + 2 + n], flat[o + 2 + n])
            o += 3 + n
        for c in clients:
            if int(c) not in per:
                continue
            losses, cm = per[int(c)]
            self.log.info("@@@@@@@@@@@@@@@@ Training Client CM({}): {}".format(round_idx, int(c)))
            for e, l in enumerate(losses):
                self.log.info("Client Index = {}\tEpoch: {}\tLoss: {:.6f}".format(int(c), e, float(l)))
            if comm_lines and cm >= 0:
                self.log.info("communication parameters for search {}".format(int(cm)))

    def _lane(self, G, B):
        """Side stream (+ its own dropout-seed scalar) of a partial-batch launch shape.

        Ragged federations (unequal sizes, drop_last=False) add, at many lockstep steps, launches of the few
        clients whose partial last batch falls there: tiny, latency-bound grids.  Such a client trains no further
        in this epoch, so its launch only has to follow the full-batch launches that wrote its rows before (the
        current stream, forked with an event) and finish before the epoch ends (joined then): it overlaps the
        next full-batch steps instead of adding its latency to the step chain.  A shape always maps to the same
        lane, because launches of one (G, B) share the engine's scratch buffers for that shape; each lane has its
        own seed scalar, which its captured graphs read (the current stream rewrites the main one every step).
        Results equal the serial order: launches in flight together touch disjoint rows."""
        k = hash((int(G), int(B))) % len(self._streams)
        return self._streams[k], self._lane_seed[k]

    def _pack_next(self, plan):
        """Per plan entry: may its optimizer step write the next step's packed weight images (engines with
        ``fused_pack``)?  Only when the same rows train again next in this epoch at the same launch shape and no other
        row group shares that shape (groups of one shape share the image buffer), unless the engine keeps images per
        row group (``images_per_group``)."""
        if not getattr(self.e, "fused_pack", False):
            return None
        groups = {}
        for it in plan:
            groups.setdefault((it[5], it[6]), set()).add(it[0])
        out, last = [False] * len(plan), {}
        for i, it in enumerate(plan):
            j = last.get(it[0])
            if j is not None:
                out[j] = (plan[j][6] == it[6] and plan[j][1] == it[1]
                          and (len(groups[(it[5], it[6])]) == 1 or getattr(self.e, "images_per_group", False)))
            last[it[0]] = i
        return out

    def _step(self, sub, r0, idx, G, B, spec, cids, lr, seed_dev=None, lr_dev=None, cids_dev=None, pack_next=False,
              prepacked=False):
        cfg = self.cfg
        gr = self.grads[r0:r0 + G]
        mo = self.mom_buf[r0:r0 + G] if self.mom_buf is not None else None
        kw = {} if cids_dev is None else {"cids_dev": cids_dev}
        if prepacked and getattr(self.e, "fused_pack_graphs", False):  # (the 2-D engine tracks its images itself)
            kw["prepacked"] = True
        loss = self.e.train_step(sub.theta, sub.bufs, gr, idx, G, B, cfg.dropout_keep, cfg.seed << 40, cids=cids,
                                 seed_dev=self._seed_dev if seed_dev is None else seed_dev, **kw)
        if self.track_loss and self._loss_acc is not None and loss is not None:
            self._loss_acc[r0:r0 + G].add_(loss.view(-1).float())
        kw = {"pack_next": True} if pack_next else {}
        self.e.local_opt(sub.theta, gr, mo, spec, lr, cfg.wd, cfg.momentum, cfg.max_norm,
                         lr_dev=self._lr_dev if lr_dev is None else lr_dev, **kw)

    def _graph_step(self, sub, r0, idx, G, B, spec, cids, seed, fill=True, seed_dev=None, cids_dev=None,
                    prepacked=False, pack_next=False):
        """One lockstep local step (forward+backward of G clients + fused optimizer) as a replayed hipGraph.  The
        ~45 kernel launches of a step become one graph launch; everything that changes between steps lives in
        device memory the graph reads: the sample indices (copied into a static buffer), the dropout stream
        counter and the round's learning rate.  The first step of a shape runs eagerly (it also allocates every
        scratch buffer the graph will reuse), the second is captured and replayed, later ones only replay — same
        kernels, same arguments, same results as the eager path.  With ``cids_dev`` (engines that take the client
        ids from device memory) the ids are one more refilled buffer and the key drops them."""
        sdev = self._seed_dev if seed_dev is None else seed_dev
        ckey = tuple(int(c) for c in cids) if cids_dev is None else None
        key = (sub.theta.data_ptr(), r0, G, B, ckey, spec.key(), sdev.data_ptr(), prepacked, pack_next)
        pk = {"prepacked": prepacked, "pack_next": pack_next}
        ent = self._graphs.get(key, "new")
        if fill:
            sdev.fill_(seed)
        st = self.graph_stats
        if ent == "new":
            st["eager_first"] = st.get("eager_first", 0) + 1
            # bounded cache: with client sampling (frac < 1) every round brings new client groups; the oldest
            # captured graphs (and the memory pools they hold) are released first
            if len(self._graphs) >= self.max_graphs and getattr(self, "_streams", None):
                torch.cuda.synchronize(self.device)  # an evicted graph may still run on a side stream
            while len(self._graphs) >= self.max_graphs:
                self._graphs.pop(next(iter(self._graphs)))
            self._step(sub, r0, idx, G, B, spec, cids, 0.0, seed_dev=sdev, cids_dev=cids_dev, **pk)
            self._graphs[key] = None
            return
        if ent is None:
            idx_buf = torch.empty(G * B, dtype=torch.int32, device=self.device)
            idx_buf.copy_(idx)
            cid_buf = None
            if cids_dev is not None:
                cid_buf = torch.empty(G, dtype=torch.int32, device=self.device)
                cid_buf.copy_(cids_dev)
            torch.cuda.current_stream().synchronize()
            g = torch.cuda.CUDAGraph()
            # no garbage collection inside the capture: a dead reference cycle of an earlier run (its captured
            # graphs, tensors freed with events on other streams) released mid-capture aborts the HIP runtime
            gc_on = gc.isenabled()
            gc.disable()
            try:
                # thread_local: the RCCL watchdog thread of a multi-GPU run may query events during the capture
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._step(sub, r0, idx_buf, G, B, spec, cids, 0.0, seed_dev=sdev, cids_dev=cid_buf, **pk)
            except Exception:  # noqa: BLE001 - capture unsupported here: stay eager for this shape
                self._graphs[key] = False
                self._step(sub, r0, idx, G, B, spec, cids, 0.0, seed_dev=sdev, cids_dev=cids_dev, **pk)
                return
            finally:
                if gc_on:
                    gc.enable()
            ent = self._graphs[key] = (g, idx_buf, cid_buf)
            st["captured"] = st.get("captured", 0) + 1
        elif ent is False:
            self._step(sub, r0, idx, G, B, spec, cids, 0.0, seed_dev=sdev, cids_dev=cids_dev, **pk)
            return
        g, idx_buf, cid_buf = ent
        st["replayed"] = st.get("replayed", 0) + 1
        idx_buf.copy_(idx)
        if cid_buf is not None:
            cid_buf.copy_(cids_dev)
        g.replay()

    def local_grad(self, rs, rows, clients, round_idx, bn_train=True, tag=11):
        """Gradient of the first batch of a fresh shuffle (``next(iter(train_loader))``) into ``self.grads`` rows
        [0, len(rows)); ``bn_train=False`` = model.eval() (DisPFL ``screen_gradients``).  Running stats untouched
        (the steps run on copies of the buffer rows)."""
        plan, idx = self._plan(clients, self._epoch_chunks(round_idx, tag, 0, n_batches=1))
        seed_dev = self._seed_dev_or_zero()
        for r0, r1, s, off, n, G, B in plan:
            t = self._to_dev(rows[r0:r1])
            th, bu = gather_rows(rs.theta, t), gather_rows(rs.bufs, t)
            seed_dev.fill_(self._step_seed(round_idx, tag, 0, s))
            self.e.train_step(th, bu, self.grads[r0:r1], idx[off:off + n], G, B, self.cfg.dropout_keep,
                              self.cfg.seed << 40, cids=clients[r0:r1], seed_dev=seed_dev, bn_train=bn_train)

    def _seed_dev_or_zero(self):
        if self._seed_dev is None:
            self._seed_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._lr_dev = torch.zeros(1, dtype=torch.float32, device=self.device)
        return self._seed_dev

    # ---------------------------------------------------------------------------------------------- SNIP
    def generate_global_mask_snip(self):
        """IterSNIP saliency on every client (mean over iterations, then clients) -> global top-k mask
        (``sailentgrads_api.py:47-66``, ``snip.py:21-116``).  ``stratified_sampling``: each iteration uses a
        label-stratified mini-batch (the intent of ``sailentgrads/client.py:33-43``)."""
        t0 = time.perf_counter()
        cfg = self.cfg
        score = torch.zeros((max(1, self.C), self.P), dtype=torch.float32, device=self.device)
        self.theta.copy_(self.w_global.unsqueeze(0).expand_as(self.theta))
        saved_bufs = self.bufs.clone()
        clients = self.local
        seed_dev = self._seed_dev_or_zero()
        for it in range(cfg.itersnip_iteration):
            if cfg.stratified_sampling:
                plan, idx = self._plan(clients, lambda j, c: [self._stratified_batch(c, it, cfg.batch_size)])
            else:  # "next(iter(train_loader))": the first batch of a fresh shuffle
                plan, idx = self._plan(clients, self._epoch_chunks(-1, 0, it, n_batches=1))
            for r0, r1, s, off, n, G, B in plan:
                seed_dev.fill_(self._step_seed(-1, 1, it, s))
                th, bu, gr = self.theta[r0:r1], self.bufs[r0:r1], self.grads[r0:r1]
                self.e.train_step(th, bu, gr, idx[off:off + n], G, B, cfg.dropout_keep, cfg.seed << 40,
                                  cids=clients[r0:r1], seed_dev=seed_dev)
                self.e.saliency_acc(th, gr, score[r0:r1], 1.0 / cfg.itersnip_iteration)
        self.bufs.copy_(saved_bufs)  # SNIP runs on a model copy: running stats are discarded
        total = score.sum(0) if self.C else torch.zeros(self.P, device=self.device)
        rt.all_reduce_buckets(total, self.info)
        total /= self.N
        sel = total[self.maskable]
        sel = sel / sel.sum()
        k = int(sel.numel() * cfg.dense_ratio)
        mask = torch.ones(self.P, dtype=torch.float32, device=self.device)
        if k >= 1:
            if self.device.type == "cuda":
                m = ops.ext()
                st = torch.empty(4, dtype=torch.int32, device=self.device)
                hist = torch.empty(256, dtype=torch.int32, device=self.device)
                sel = sel.contiguous()
                m.radix_select_kth(sel.data_ptr(), sel.numel(), k, st.data_ptr(), hist.data_ptr(),
                                   ops.stream())
                keep = torch.empty_like(sel)
                m.threshold_mask(sel.data_ptr(), sel.numel(), st.data_ptr(), keep.data_ptr(),
                                 ops.stream())
            else:
                thr = torch.topk(sel, k, sorted=True).values[-1]
                keep = (sel >= thr).float()
            mask[self.maskable] = keep
        self.set_mask(mask if cfg.snip_mask else torch.ones_like(mask))
        self.timers["snip"] += time.perf_counter() - t0
        return self.mask

    def set_mask(self, mask):
        self.mask = mask
        self.mask_bits = MK.pack_bits(mask.view(1, -1))
        self._graphs = {}  # captured local steps reference the mask tensor

    # ---------------------------------------------------------------------------------------------- rounds
    def sample_clients(self, round_idx):
        per_round = max(1, int(self.N * self.cfg.frac))
        if per_round >= self.N:
            return list(range(self.N))
        np.random.seed(round_idx)
        return sorted(np.random.choice(range(self.N), per_round, replace=False).tolist())

    # ---------------------------------------------------------------------------------------------- rebalancing
    def _row_state(self):
        """Per-client device state that moves with a client: (attribute path, tensor [rows, width]).  Subclasses
        add theirs (mask bits, personal models)."""
        return [("theta", self.theta), ("bufs", self.bufs)]

    def balanced_owner(self, sampled):
        """Owner map for this round: start from the current owners and move sampled clients from the most to the
        least loaded rank (load = training samples of its sampled clients) while that lowers the larger of the two
        loads; the move picked is the one leaving the pair most even (ties: lowest client id).  Identical on every
        rank (pure function of the sizes, the sample and the current owners)."""
        own = self.owner.copy()
        load = np.zeros(self.info.world, dtype=np.int64)
        for c in sampled:
            load[own[c]] += self.sizes[c]
        for _ in range(len(sampled)):
            hi, lo = int(np.argmax(load)), int(np.argmin(load))
            if hi == lo:
                break
            best = None
            for c in sorted(c for c in sampled if own[c] == hi):
                peak = max(load[hi] - self.sizes[c], load[lo] + self.sizes[c])
                if peak < load[hi] and (best is None or peak < best[0]):
                    best = (peak, c)
            if best is None:
                break
            c = best[1]
            own[c] = lo
            load[hi] -= self.sizes[c]
            load[lo] += self.sizes[c]
        return own

    def rebalance(self, sampled):
        """Sampling-aware load balance (``cfg.rebalance``, multi-rank): migrate the state of sampled clients to the
        ranks :meth:`balanced_owner` picks — rows go point to point (RCCL send/recv), ownership moves with them and
        stays there until a later round moves it again.  Results do not depend on where a client trains."""
        if not (self.cfg.rebalance and self.info.enabled and self.info.world > 1):
            return
        t0 = time.perf_counter()
        self.migrate(self.balanced_owner(sampled))
        self.timers["migrate"] = self.timers.get("migrate", 0.0) + time.perf_counter() - t0

    def migrate(self, new_owner):
        new_owner = np.asarray(new_owner, dtype=np.int64)
        moving = [c for c in range(self.N) if new_owner[c] != self.owner[c]]
        if not moving:
            return
        me = self.info.rank
        needs = [[c for c in moving if new_owner[c] == r] for r in range(self.info.world)]
        new_local = sorted((c for c in range(self.N) if new_owner[c] == me), key=lambda c: (-int(self.sizes[c]), c))
        n = max(1, len(new_local))
        self._migrate_samples(needs, new_local)
        new_state = {}
        for path, t in self._row_state():
            width = t.shape[1]
            recv = rt.exchange_rows(self.info, self.owner, needs, lambda c, t=t: t[self.row_of[c]], width,
                                    self.device, t.dtype)
            nt = padded_rows(n, width, self.device, dtype=t.dtype) if t.dtype == torch.float32 else \
                torch.zeros((n, width), dtype=t.dtype, device=self.device)
            keep = [(i, self.row_of[c]) for i, c in enumerate(new_local) if c in self.row_of]
            if keep:
                di = self._to_dev([i for i, _ in keep])
                si = self._to_dev([j for _, j in keep])
                nt[di] = t[si]
            for i, c in enumerate(new_local):
                if c not in self.row_of:
                    nt[i].copy_(recv[c])
            new_state[path] = nt
        for path, nt in new_state.items():
            obj = self
            parts = path.split(".")
            for p_ in parts[:-1]:
                obj = getattr(obj, p_)
            setattr(obj, parts[-1], nt)
        self.owner = new_owner
        self.shards = [[c for c in range(self.N) if new_owner[c] == r] for r in range(self.info.world)]
        self.local = new_local
        self.row_of = {c: i for i, c in enumerate(new_local)}
        self.C = len(new_local)
        self.grads = padded_rows(n, self.P, self.device)
        self.mom_buf = padded_rows(n, self.P, self.device) if self.cfg.momentum != 0 else None
        self._after_migrate()

    def _sample_rows(self, c):
        """Store rows of client c's samples in a fixed order: train, test, then validation."""
        sp = self.splits[c]
        parts = [sp.train, sp.test] + ([sp.val] if sp.val is not None else [])
        return np.concatenate([np.asarray(p, dtype=np.int64) for p in parts])

    def _migrate_samples(self, needs, new_local):
        """Move the per-sample store rows (``engine.sample_fields``: volumes, moments, labels) of migrating clients
        with their state, point to point, and rebuild each rank's store to hold exactly its clients' samples (the
        data is sharded like the clients, never replicated).  Splits are re-based in the same order, so a client
        draws the same batches wherever it trains."""
        fields = getattr(self.e, "sample_fields", None)
        if not fields:
            return
        from .executor import ClientSplit
        rows = {c: self._sample_rows(c) for c in self.local}
        ns = {c: len(self.splits[c].train) + len(self.splits[c].test) +
              (0 if self.splits[c].val is None else len(self.splits[c].val)) for c in range(self.N)}
        for f in fields:
            F = getattr(self.e, f)
            rest = tuple(F.shape[1:])
            re_ = int(np.prod(rest)) if rest else 1
            recv = rt.exchange_rows(self.info, self.owner, needs,
                                    lambda c, F=F: F.index_select(0, torch.as_tensor(rows[c], device=F.device)).reshape(-1),
                                    lambda c, re_=re_: ns[c] * re_, F.device, F.dtype)
            parts = [F.index_select(0, torch.as_tensor(rows[c], device=F.device)) if c in rows
                     else recv[c].view((ns[c],) + rest) for c in new_local]
            setattr(self.e, f, torch.cat(parts) if parts else F[:0].clone())
            del F, parts, recv
        splits, off = list(self.splits), 0
        for c in range(self.N):
            sp = self.splits[c]
            ntr, nte = len(sp.train), len(sp.test)
            nva = None if sp.val is None else len(sp.val)
            splits[c] = ClientSplit(np.zeros(ntr, np.int64), np.zeros(nte, np.int64),
                                    None if nva is None else np.zeros(nva, np.int64))
        for c in new_local:
            sp = splits[c]
            ntr, nte, nva = len(sp.train), len(sp.test), 0 if sp.val is None else len(sp.val)
            splits[c] = ClientSplit(np.arange(off, off + ntr), np.arange(off + ntr, off + ntr + nte),
                                    None if sp.val is None else np.arange(off + ntr + nte, off + ntr + nte + nva))
            off += ntr + nte + nva
        self.splits = splits

    def _after_migrate(self):
        self._graphs = {}
        self._scratch = None
        self._eval_cache = None
        if hasattr(self, "rowset"):
            self.rowset = RowSet(self.theta, self.bufs)

    def _local_rows(self, clients):
        """(rows, clients) of the given global clients that live on this rank, in row order."""
        cs = sorted((c for c in clients if c in self.row_of), key=lambda c: self.row_of[c])
        return [self.row_of[c] for c in cs], cs

    def _fedavg_spec(self):
        spec = StepSpec()
        if self.alg == "salientgrads" and self.mask_bits is not None:
            spec = replace(spec, mask_mode=MASK_WEIGHT, bits=self.mask_bits, shared=True)
        if self.cfg.prox_mu > 0:
            spec = replace(spec, prox_mu=self.cfg.prox_mu, ref=self.w_global)
        return spec

    def local_train(self, round_idx, sampled, lr=None):
        rows, loc = self._local_rows(sampled)
        if not rows:
            return
        if _contiguous(rows):  # one broadcast launch for the whole run
            self.theta[rows[0]:rows[-1] + 1].copy_(self.w_global.expand(len(rows), -1))
            self.bufs[rows[0]:rows[-1] + 1].copy_(self.b_global.expand(len(rows), -1))
        else:
            ix = self._to_dev(rows)
            self.theta[ix] = self.w_global.unsqueeze(0).expand(len(rows), -1)
            self.bufs[ix] = self.b_global.unsqueeze(0).expand(len(rows), -1)
        # downlink: count_communication_params(w_global) per sampled client (the same state for all of them)
        down = self._rows_nnz(self.w_global.view(1, -1))[0] + self._rows_nnz(self.b_global.view(1, -1))[0]
        self.train_rows(RowSet(self.theta, self.bufs), rows, loc, round_idx, self.cfg.epochs, self._fedavg_spec(),
                        lr=lr)
        self.add_comm(down + self.state_nonzeros(self.theta, self.bufs, rows), loc)  # + uplink (the local model)

    def aggregate(self, sampled):
        if self.cfg.aggregator != "fedavg":
            return self.aggregate_robust(sampled)
        if self.cfg.update_topk > 0:
            return self.aggregate_topk(sampled)
        return self.aggregate_fedavg(sampled)

    def _topk_space(self):
        """One selection segment spanning the whole parameter row (the segmented radix select of ``sparse.hip``
        then picks a per-row top-k)."""
        if getattr(self, "_tk_space", None) is None:
            from types import SimpleNamespace
            lay = SimpleNamespace(names=["all"], offsets=[0], total=self.P, numel=lambda i: self.P)
            self._tk_space = MK.MaskSpace(lay)
        return self._tk_space

    def aggregate_topk(self, sampled):
        """Sparse-update FedAvg: client i contributes n_i/N * topk(theta_i - w_global) (fixed k per client, so
        every rank knows every rank's payload size), BN buffers are averaged densely.

        * selection: the segmented radix select (``MaskSpace.select`` REGROW_ABS over one row-wide segment, exact
          k with deterministic ties) on chunks of rows, instead of ``torch.topk``;
        * exchange: ONE all-gather of [client id | k values | k indices (int32 bits)] rows with sizes known on
          every rank (no size exchange, no host sync);
        * combine: every rank orders the gathered lists by client id and reduces duplicates with a sort-based
          coalesce (sequential per-index sums in client order, no atomics), so all ranks get identical fp32 sums."""
        n_tot = float(sum(self.sizes[c] for c in sampled))
        k = max(1, int(math.ceil(self.cfg.update_topk * self.P)))
        rows, loc = self._local_rows(sampled)
        rec = torch.zeros((len(rows), 1 + 2 * k), dtype=torch.float32, device=self.device)
        space = self._topk_space()
        # per-row client ids and FedAvg weights: one pinned non-blocking upload (no host sync in the loop below)
        meta = torch.tensor([[float(self.local[r]), self.sizes[self.local[r]] / n_tot] for r in rows],
                            dtype=torch.float32).view(-1, 2)
        meta = (meta.pin_memory().to(self.device, non_blocking=True) if self.device.type == "cuda" else meta)
        # chunks bound the [rows, P] temporaries: 8 x 46 M fp32 = 1.5 GB for the 3D ResNet-50
        chunk = max(1, min(len(rows), int(2e9 // (4 * max(1, self.P)))))
        for j0 in range(0, len(rows), chunk):
            rr = rows[j0:j0 + chunk]
            n = len(rr)
            d = padded_rows(n, self.P, self.device)
            if _contiguous(rr):
                torch.sub(self.theta[rr[0]:rr[-1] + 1, :self.P], self.w_global, out=d)
            else:
                torch.sub(self.theta.index_select(0, self._to_dev(rr))[:, :self.P], self.w_global,
                          out=d)
            bits = torch.zeros((n, self.W), dtype=torch.int32, device=self.device)
            space.select(MK.REGROW_ABS, d, bits, torch.full((n, 1), k, dtype=torch.int64))
            # exactly k set bits per row: a static-size compaction (no device->host size query)
            top = torch.nonzero_static(MK.unpack_bits(bits, self.P, torch.bool), size=n * k)[:, 1].view(n, k)
            rec[j0:j0 + n, 0] = meta[j0:j0 + n, 0]
            rec[j0:j0 + n, 1:1 + k] = d.gather(1, top) * meta[j0:j0 + n, 1:2]
            rec[j0:j0 + n, 1 + k:] = top.to(torch.int32).view(torch.float32)
        per_rank = [sum(1 for c in sampled if self.owner[c] == r) * (1 + 2 * k) for r in range(self.info.world)]
        g = rt.all_gather_sized(rec.view(-1), per_rank, self.info).view(-1, 1 + 2 * k)
        g = g.index_select(0, torch.argsort(g[:, 0]))  # fixed client order on every rank
        g_idx = g[:, 1 + k:].contiguous().view(torch.int32).to(torch.int64).reshape(1, -1)
        upd = torch.sparse_coo_tensor(g_idx, g[:, 1:1 + k].reshape(-1), (self.P,)).coalesce()
        self.w_global.index_add_(0, upd.indices()[0], upd.values())
        # BN buffers: dense weighted sum of the rows (one reduction, not one launch per client)
        bsum = (meta[:, 1:2] * self.bufs[rows, :self.Q]).sum(0) if rows else \
            torch.zeros(self.Q, dtype=torch.float32, device=self.device)
        rt.all_reduce_buckets(bsum, self.info)
        self.b_global.copy_(bsum)
        self.stat_info["aggregate_elems"] = int(2 * k * len(sampled))

    def _compact_index(self, Pp):
        """Flat indices of the aggregation buffer that can be non-zero: SalientGrads' global mask zeroes the
        pruned weights on every client after every step, so their weighted sum is exactly 0 and they need
        not travel (params kept by the mask + all BN buffers)."""
        key = (Pp, id(self.mask))
        if getattr(self, "_cidx_key", None) != key:
            keep = torch.ones(Pp + self.Q, dtype=torch.bool, device=self.device)
            keep[:self.P] = self.mask > 0
            keep[self.P:Pp] = False
            self._cidx = keep.nonzero().view(-1)
            self._cidx_key = key
        return self._cidx

    def weighted_partial(self, theta, bufs, rows, weights):
        """[Pp + Q] buffer = sum_j weights[j] * (theta[rows[j]], bufs[rows[j]]) (local partial of a FedAvg)."""
        Pp = (self.P + 63) // 64 * 64  # keep the buffer section 16-B aligned for the vectorised kernel
        buf = torch.zeros(Pp + self.Q, dtype=torch.float32, device=self.device)
        if rows:
            w = self._to_dev(weights, torch.float32)
            if self.device.type == "cuda" and _contiguous(rows):
                m, st = ops.ext(), ops.stream()
                lo = rows[0]
                m.weighted_rows_sum(theta[lo].data_ptr(), w.data_ptr(), len(rows), self.P, theta.stride(0), 0.0,
                                    buf.data_ptr(), st)
                if self.Q:  # GroupNorm models carry no buffers
                    m.weighted_rows_sum(bufs[lo].data_ptr(), w.data_ptr(), len(rows), self.Q, bufs.stride(0), 0.0,
                                        buf[Pp:].data_ptr(), st)
            else:
                ix = self._to_dev(rows)
                buf[:self.P] = (w.view(-1, 1) * theta[ix]).sum(0)
                buf[Pp:] = (w.view(-1, 1) * bufs[ix]).sum(0)
        return buf, Pp

    def aggregate_fedavg(self, sampled):
        """w_global = sum_i n_i/sum n * w_i over sampled clients (params + buffers), one all-reduce (of the
        mask-compacted coordinates when a SalientGrads mask is active)."""
        n_tot = float(sum(self.sizes[c] for c in sampled))
        rows, loc = self._local_rows(sampled)
        buf, Pp = self.weighted_partial(self.theta, self.bufs, rows, [self.sizes[c] / n_tot for c in loc])
        sparse = (self.info.enabled and self.cfg.sparse_aggregate and self.alg == "salientgrads"
                  and self.mask is not None)
        if sparse:
            idx = self._compact_index(Pp)
            packed = buf.index_select(0, idx)
            rt.all_reduce_buckets(packed, self.info)
            buf.zero_()
            buf.index_copy_(0, idx, packed)
            self.stat_info["aggregate_elems"] = int(idx.numel())
        else:
            rt.all_reduce_buckets(buf, self.info)
            self.stat_info["aggregate_elems"] = int(buf.numel())
        self.w_global.copy_(buf[:self.P])
        self.b_global.copy_(buf[Pp:])

    def aggregate_robust(self, sampled):
        """Byzantine-robust aggregation (BASELINE config 4): every sampled client's (params, buffers) row is
        all-gathered to every rank (xGMI all-gather of K x (P+Q) fp32; 128 x 10.3 MB = 1.3 GB fits HBM
        easily), then Krum / Multi-Krum / coordinate median / trimmed mean run on device with the same
        deterministic result on all ranks (``core/robustness.py``).  BN buffers follow the selected clients
        for Krum and are coordinate-aggregated otherwise."""
        from ..core import robustness as R
        rows, loc = self._local_rows(sampled)
        W = self.P + self.Q
        # one record per client: [id, params, buffers]; every rank knows how many sampled clients each rank owns,
        # so the gather needs no size exchange (no host round trip)
        lm = torch.cat([self._to_dev(loc, torch.float32).view(-1, 1), self.theta[rows, :self.P],
                        self.bufs[rows, :self.Q]], 1) if rows else torch.zeros((0, 1 + W), device=self.device)
        per_rank = [sum(1 for c in sampled if self.owner[c] == r) * (1 + W) for r in range(self.info.world)]
        allrows = rt.all_gather_sized(lm.reshape(-1).contiguous(), per_rank, self.info).view(-1, 1 + W)
        order = torch.argsort(allrows[:, 0])  # deterministic client order on every rank
        M = allrows[:, 1:].index_select(0, order)
        kind = self.cfg.aggregator
        if kind in ("krum", "multikrum"):
            m = 1 if kind == "krum" else (self.cfg.multikrum_m or max(1, M.shape[0] - self.cfg.byzantine_f))
            agg, _ = R.krum(M, f=self.cfg.byzantine_f, multi=m)
        elif kind == "median":
            agg = R.coordinate_median(M)
        elif kind == "trimmed_mean":
            agg = R.trimmed_mean(M, self.cfg.trim_ratio)
        else:
            raise ValueError("unknown aggregator %r" % kind)
        self.w_global.copy_(agg[:self.P])
        self.b_global.copy_(agg[self.P:])
        self.stat_info["aggregate_elems"] = int(M.numel())

    # ---------------------------------------------------------------------------------------------- evaluation
    def _split_of(self, c, which):
        s = self.splits[c]
        return {"test": s.test, "train": s.train, "val": getattr(s, "val", None)}[which]

    def _eval_chunk_metrics(self, logits, y):
        """Per-sample (correct, loss) of logits [..., K] (K = 1: binary head) against labels [...]."""
        if logits.shape[-1] > 1:  # multi-class models (CrossEntropy trainers of the 2D baselines)
            loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), y.reshape(-1).long(),
                                   reduction="none").view(y.shape)
            correct = (logits.argmax(-1) == y.long()).float()
            return correct, loss
        logits = logits[..., 0]
        pred = torch.sigmoid(logits)
        x = logits if self.cfg.fix_eval_loss else pred  # Q1: the reference feeds probabilities to BCEWithLogits
        loss = F.binary_cross_entropy_with_logits(x, y, reduction="none")
        correct = ((pred >= 0.5).float() == y).float()
        return correct, loss

    def _eval_rows(self, theta, bufs, clients, per_client_rows, which="test", chunk=None):
        """Per-client (correct, loss_sum, total) with reference test semantics (Q1).  Clients that share a
        model row are evaluated together in chunks of ``chunk`` (default ``test_batch``) samples, balanced so the
        last launch is not a small tail (one launch sequence each)."""
        out = np.zeros((len(clients), 3), dtype=np.float64)
        by_row = {}
        for j, r in enumerate(per_client_rows):
            by_row.setdefault(r, []).append(j)
        for r, js in by_row.items():
            tests = [self._split_of(clients[j], which) for j in js]
            owner = np.concatenate([np.full(len(t), k) for k, t in enumerate(tests)]).astype(np.int64)
            allidx = np.concatenate(tests).astype(np.int32) if tests else np.zeros(0, np.int32)
            if allidx.size == 0:
                continue
            th, bu = theta[r:r + 1], bufs[r:r + 1]
            cap = chunk or self.cfg.test_batch
            tb = -(-allidx.size // -(-allidx.size // cap))  # ceil(n / ceil(n / cap))
            acc = torch.zeros((len(js), 3), dtype=torch.float64, device=self.device)
            own_t = self._to_dev(owner)
            all_t = self._upload_i32(allidx)
            for s in range(0, allidx.size, tb):
                idx = all_t[s:s + tb]
                logits = self.e.eval_logits(th, bu, idx, 1, idx.numel()).view(idx.numel(), -1)
                y = self.e.labels.index_select(0, idx.long().to(self.e.labels.device)).to(logits.device).float()
                correct, loss = self._eval_chunk_metrics(logits, y)
                o = own_t[s:s + idx.numel()]
                acc[:, 0].index_add_(0, o, correct.double())
                acc[:, 1].index_add_(0, o, loss.double())
                acc[:, 2].index_add_(0, o, torch.ones_like(loss, dtype=torch.float64))
            out[js] = acc.cpu().numpy()
        return out

    @staticmethod
    def _pad_size(n):
        """Evaluation bucket of a split of n samples: n rounded up to a multiple of 8 (n <= 64), else to the next
        step of a 2^(1/4) ladder (<= 19 % padding, ~9 % on average)."""
        if n <= 64:
            return -(-n // 8) * 8
        return int(math.ceil(2.0 ** (math.ceil(4.0 * math.log2(n) - 1e-9) / 4.0)))

    def eval_grouped(self, theta, bufs, rows, clients, which="test", device_out=False):
        """Model row rows[j] on client clients[j]'s split, per-client (correct, loss_sum, total).

        Ragged splits (Dirichlet / site partitions give nearly every client its own size) are bucketed by padded
        size (:meth:`_pad_size`) and each bucket's clients run as grouped launches of G rows x chunk samples, the
        rows past a client's size repeating its first sample and masked out of the sums — a few launches instead
        of one small latency-bound launch per distinct size (or per test_batch chunk of a large client).  Every
        model is per-sample in eval mode (GroupNorm, BatchNorm on running statistics), so the padding cannot
        change a valid sample's logits.  ``NIDT_EVAL_PAD=0`` keeps the exact-size grouping (A/B).  ``device_out``:
        the [len(clients), 3] float64 result stays on the device (no host synchronisation)."""
        if os.environ.get("NIDT_EVAL_PAD", "1") == "0":
            r = self._eval_grouped_exact(theta, bufs, rows, clients, which)
            return torch.from_numpy(r).to(self.device) if device_out else r
        out = np.zeros((len(clients), 3), dtype=np.float64)
        splits = [self._split_of(c, which) for c in clients]
        buckets = {}
        for j, sp in enumerate(splits):
            if len(sp):
                buckets.setdefault(self._pad_size(len(sp)), []).append(j)
        tb = self.cfg.test_batch
        launches = []
        for npad, js in sorted(buckets.items()):
            # at most ~32 test batches of samples per launch (activation memory of the eval forward)
            gcap = max(1, (32 * tb) // min(npad, tb))
            for grp0 in self._groups(js):
                for grp in [grp0[i:i + gcap] for i in range(0, len(grp0), gcap)]:
                    top = max(len(splits[j]) for j in grp)  # padded to the group's largest split (equal sizes: none)
                    for s0 in range(0, top, tb):
                        launches.append((grp, s0, min(tb, top - s0)))
        lanes = self._side_streams() if (self.device.type == "cuda" and len(launches) > 2) else None
        main, used = (torch.cuda.current_stream(), set()) if lanes else (None, None)
        fork = main.record_event() if lanes else None
        pending = []
        for grp, s0, ch in launches:
            G = len(grp)
            idx = np.empty((G, ch), dtype=np.int32)
            valid = np.zeros(G, dtype=np.int64)
            for k, j in enumerate(grp):
                seg = np.asarray(splits[j][s0:s0 + ch])
                valid[k] = len(seg)
                idx[k, :len(seg)] = seg
                idx[k, len(seg):] = splits[j][0]
            st = self._lane(G, ch)[0] if lanes else None
            if st is not None and st not in used:
                st.wait_event(fork)
                used.add(st)
            with torch.cuda.stream(st) if st is not None else _nullctx():
                rr = [rows[j] for j in grp]
                if _contiguous(rr):
                    th, bu = theta[rr[0]:rr[-1] + 1], bufs[rr[0]:rr[-1] + 1]
                else:
                    t = self._to_dev(rr)
                    th, bu = gather_rows(theta, t), gather_rows(bufs, t)
                # host->device through pinned buffers, enqueued before the forward: a pageable copy here would
                # block the host until this launch's forward finished and serialise the launch sequence
                idx_d = self._upload_i32(idx.reshape(-1))
                valid_d = self._upload_i32(valid)
                logits = self.e.eval_logits(th, bu, idx_d, G, ch).view(G, ch, -1)
                y = self.e.labels.index_select(0, idx_d.long().to(self.e.labels.device)).to(logits.device).float()
                correct, loss = self._eval_chunk_metrics(logits, y.view(G, ch))
                valid_d = valid_d.to(logits.device)
                if int(valid.min()) < ch:
                    keep = (torch.arange(ch, device=logits.device).view(1, ch) < valid_d.view(G, 1)).float()
                    correct, loss = correct * keep, loss * keep
                res = torch.stack([correct.sum(1).double(), loss.sum(1).double(), valid_d.double()], 1)
            if st is not None:
                res.record_stream(main)
            pending.append((grp, res))
        for st in used or ():
            main.wait_stream(st)
        if device_out:  # accumulate on the device: no host wait (the deferred-metrics path)
            od = torch.zeros((len(clients), 3), dtype=torch.float64, device=self.device)
            if pending:
                pos = self._upload_i32(np.concatenate([np.asarray(g, dtype=np.int32) for g, _ in pending]))
                od.index_add_(0, pos.long(), torch.cat([r for _, r in pending], 0).to(self.device))
            return od
        if pending:
            host = torch.cat([r for _, r in pending], 0).cpu().numpy()
            o = 0
            for grp, _ in pending:
                out[grp] += host[o:o + len(grp)]
                o += len(grp)
        return out

    def _eval_grouped_exact(self, theta, bufs, rows, clients, which="test"):
        """Model row rows[j] on client clients[j]'s split: clients with equal split sizes are evaluated in grouped
        launches (G rows x n samples); one device->host copy at the end."""
        out = np.zeros((len(clients), 3), dtype=np.float64)
        pending = []
        sizes = {}
        for j, c in enumerate(clients):
            sizes.setdefault(len(self._split_of(c, which)), []).append(j)
        # ragged test sets (one launch per distinct size, most of them a client or two: latency-bound) run on the
        # side lanes, a shape per lane (the engine's eval scratch is per shape); eval-mode launches are independent
        lanes = self._side_streams() if (self.device.type == "cuda" and len(sizes) > 2) else None
        main, used = (torch.cuda.current_stream(), set()) if lanes else (None, None)
        fork = main.record_event() if lanes else None
        for n, js in sizes.items():
            if n == 0:
                continue
            if n > self.cfg.test_batch:
                out[js] = self._eval_rows(theta, bufs, [clients[j] for j in js], [rows[j] for j in js], which)
                continue
            for grp in self._groups(js):
                st = self._lane(len(grp), n)[0] if lanes else None
                if st is not None and st not in used:
                    st.wait_event(fork)
                    used.add(st)
                with torch.cuda.stream(st) if st is not None else _nullctx():
                    rr = [rows[j] for j in grp]
                    if _contiguous(rr):
                        th, bu = theta[rr[0]:rr[-1] + 1], bufs[rr[0]:rr[-1] + 1]
                    else:
                        t = self._to_dev(rr)
                        th, bu = gather_rows(theta, t), gather_rows(bufs, t)
                    idx = self._upload_i32(np.concatenate([self._split_of(clients[j], which) for j in grp]))
                    logits = self.e.eval_logits(th, bu, idx, len(grp), n).view(len(grp), n, -1)
                    y = self.e.labels.index_select(0, idx.long().to(self.e.labels.device)).to(logits.device).float()
                    y = y.view(len(grp), n)
                    correct, loss = self._eval_chunk_metrics(logits, y)
                    res = torch.stack([correct.sum(1), loss.sum(1), torch.full_like(loss[:, 0], float(n))], 1).double()
                if st is not None:
                    res.record_stream(main)  # consumed on the current stream after the join
                pending.append((grp, res))
        for st in used or ():
            main.wait_stream(st)
        if pending:
            host = torch.cat([r for _, r in pending], 0).cpu().numpy()
            o = 0
            for grp, _ in pending:
                out[grp] = host[o:o + len(grp)]
                o += len(grp)
        return out

    def _eval_buffers(self, k):
        if self._eval_cache is None or self._eval_cache[0].shape[0] < k:
            self._eval_cache = (padded_rows(k, self.P, self.device), padded_rows(k, self.Q, self.device))
        th, bu = self._eval_cache
        return th[:k], bu[:k]

    def _eval_global_and_personal(self, theta=None, bufs=None, device_out=False):
        """Global model and every local client's personal model on that client's test split, as grouped launches:
        the personal rows straight from the row matrix, the global model from K = min(C, 64) staged copies that
        every group of clients reuses (rows j mod K).  (Staging copies of all C personal rows next to C copies of
        the global model took a 2C-row buffer: 94 GB for config 5's 256 x 46 M parameters, which pushed its peak to
        260 GiB and the allocator into a synchronous cache flush every round.)  Per-client launch shapes stay those
        of the grouped evaluation: the engines' per-client tensors keep their 32-bit offsets.  At the AlexNet3D
        headline (64 clients) it is also slightly faster than one launch sequence over the 2C-row copy (2.2055 vs
        2.196-2.200 rounds/s); with up to 32 clients (small models) the copy's twice-as-wide launches win and are
        used (``NIDT_EVAL_STAGE=1`` / ``0`` force either form; profiles/r4_ab_eval_forms.txt)."""
        C = self.C
        theta = self.theta if theta is None else theta
        bufs = self.bufs if bufs is None else bufs
        stage = os.environ.get("NIDT_EVAL_STAGE")
        if stage == "1" or (stage is None and C <= 32 and 2 * C * (self.P + self.Q) * 4 <= (8 << 30)):
            # few clients: one grouped launch sequence over a 2C-row copy (C personal + C global rows) keeps the
            # launches twice as wide (8 clients: 14.78-14.84 vs 14.64-14.73 rounds/s, profiles/r4_ab_eval_forms.txt)
            th, bu = self._eval_buffers(2 * C)
            with torch.no_grad():
                th[:C].copy_(theta[:C])
                th[C:].copy_(self.w_global.expand(C, -1))
                bu[:C].copy_(bufs[:C])
                bu[C:].copy_(self.b_global.expand(C, -1))
            res = self.eval_grouped(th, bu, list(range(2 * C)), self.local + self.local, device_out=device_out)
            return res[C:], res[:C]
        pers = self.eval_grouped(theta, bufs, list(range(C)), self.local, device_out=device_out)
        K = min(C, 64)
        th, bu = self._eval_buffers(K)
        with torch.no_grad():
            th.copy_(self.w_global.expand(K, -1))
            bu.copy_(self.b_global.expand(K, -1))
        glob = self.eval_grouped(th, bu, [j % K for j in range(C)], self.local, device_out=device_out)
        return glob, pers

    def gather_metrics(self, clients, arr, device_out=False):
        """Per-client metric rows of this rank's clients -> [N, k] on every rank (one all-reduce): numpy, or with
        ``device_out`` a device tensor (``arr`` may then be a device tensor too: nothing waits for the device)."""
        k = arr.shape[1] if arr.ndim == 2 else 1
        res = torch.zeros((self.N, k), dtype=torch.float64, device=self.device)
        if len(clients):
            src = arr if torch.is_tensor(arr) else torch.from_numpy(np.asarray(arr, dtype=np.float64))
            res.index_copy_(0, self._upload_i32(list(clients)).to(self.device).long(),
                            src.to(self.device, torch.float64).reshape(len(clients), k))
        rt.all_reduce_buckets(res, self.info)
        return res if device_out else res.cpu().numpy()

    @staticmethod
    def mean_acc_loss(r, cols=(0, 1, 2)):
        ok = r[:, cols[2]] > 0
        if not ok.any():
            return 0.0, 0.0
        return float(np.mean(r[ok, cols[0]] / r[ok, cols[2]])), float(np.mean(r[ok, cols[1]] / r[ok, cols[2]]))

    def _defer_metrics(self):
        """Timed GPU runs without a logger read a round's metrics one round later (pinned copy + event) instead of
        waiting for the device at the end of every round; with a logger (reference log order) or on the CPU they are
        read at once.  ``NIDT_DEFER_METRICS=0`` disables the deferral."""
        env = os.environ.get("NIDT_DEFER_METRICS", "1")
        return env == "force" or (self.device.type == "cuda" and self.log is None and env != "0")

    def _flush_metrics(self, ready_only=False):
        """Fold the evaluations still in flight into ``stat_info`` (in round order); ``ready_only``: only those whose
        device result has already arrived (never waits)."""
        while self._pending_metrics:
            if ready_only and self._pending_metrics[0][2] is not None and not self._pending_metrics[0][2].query():
                break
            round_idx, host, ev, holder, *rec = self._pending_metrics.pop(0)
            if ev is not None:
                ev.synchronize()
            holder["res"] = (rec[0] if rec else self._record_metrics)(round_idx, host.numpy().copy())
            if ev is not None:
                self._pinned_free.append(host)

    def _defer_result(self, round_idx, r, recorder=None):
        """Queue the device metric matrix ``r`` of a round: a pinned copy + event now, folded into ``stat_info`` by
        ``recorder(round_idx, host_matrix)`` (default :meth:`_record_metrics`) when first looked at."""
        if self.device.type == "cuda":
            host = next((h for h in self._pinned_free if h.shape == r.shape), None)
            if host is not None:
                self._pinned_free.remove(host)
            else:
                host = torch.empty(r.shape, dtype=r.dtype, pin_memory=True)
            host.copy_(r, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:  # NIDT_DEFER_METRICS=force on the CPU (tests of the deferred bookkeeping)
            host, ev = r.clone(), None
        holder = {}
        self._pending_metrics.append((round_idx, host, ev, holder) + ((recorder,) if recorder else ()))
        return LazyMetrics(self, holder)

    def _record_metrics(self, round_idx, r):
        sl = dict.__getitem__  # the raw lists: this IS the flush
        g_acc, g_loss = self.mean_acc_loss(r, (0, 1, 2))
        p_acc, p_loss = self.mean_acc_loss(r, (3, 4, 5))
        sl(self.stat_info, "global_test_acc").append(g_acc)
        sl(self.stat_info, "global_test_loss").append(g_loss)
        sl(self.stat_info, "person_test_acc").append(p_acc)
        sl(self.stat_info, "person_test_loss").append(p_loss)
        if self.log is not None and self.info.is_main:
            self.log.info("################global_test_on_all_clients : {}".format(round_idx))
            self.log.info({"global_test_acc": g_acc, "global_test_loss": g_loss})
            self.log.info({"person_test_acc": p_acc, "person_test_loss": p_loss})
        return dict(global_test_acc=g_acc, global_test_loss=g_loss, person_test_acc=p_acc, person_test_loss=p_loss)

    def evaluate(self, round_idx, theta=None, bufs=None):
        t0 = time.perf_counter()
        if self._defer_metrics():
            self._flush_metrics(ready_only=True)  # earlier rounds whose copies have landed: no wait
            if self.C:
                glob, pers = self._eval_global_and_personal(theta, bufs, device_out=True)
                loc = torch.cat([glob, pers], 1)
            else:
                loc = torch.zeros((0, 6), dtype=torch.float64, device=self.device)
            r = self.gather_metrics(self.local, loc, device_out=True)
            self.timers["eval"] += time.perf_counter() - t0
            return self._defer_result(round_idx, r)
        glob, pers = self._eval_global_and_personal(theta, bufs) if self.C else (np.zeros((0, 3)), np.zeros((0, 3)))
        r = self.gather_metrics(self.local, np.concatenate([glob, pers], 1))
        self._flush_metrics()
        res = self._record_metrics(round_idx, r)
        self.timers["eval"] += time.perf_counter() - t0
        return res

    # ---------------------------------------------------------------------------------------------- driver
    def _heartbeat(self):
        """Lazily started failure detector (multi-rank runs with ``cfg.heartbeat_s`` > 0), else None."""
        if self.cfg.heartbeat_s <= 0 or self.info.world <= 1:
            return None
        if getattr(self, "_hb", None) is None:
            from ..comm.failure import HeartbeatMonitor, default_store
            store = default_store()
            self._hb = HeartbeatMonitor(store, self.info.rank, self.info.world, self.cfg.heartbeat_s,
                                        30.0 * self.cfg.heartbeat_s) if store is not None else False
        return self._hb or None

    def _round_start(self, round_idx):
        hb = self._heartbeat()
        if hb is not None:
            hb.check_or_raise()  # before the round's collectives: a dead peer would block them until the timeout
        if self.log is not None and self.info.is_main:
            self.log.info("################Communication round : {}".format(round_idx))

    def _eval_due(self, round_idx):
        f = self.cfg.frequency_of_the_test
        return bool(f) and (round_idx % f == 0 or round_idx == self.cfg.comm_round - 1)

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        self._round_start(round_idx)
        sampled = self.sample_clients(round_idx)
        if self.log is not None and self.info.is_main:
            self.log.info("client_indexes = " + str(np.array(sampled)))
        self.rebalance(sampled)
        self.local_train(round_idx, sampled)
        if sync_timers:
            self._sync()
        t1 = time.perf_counter()
        self.aggregate(sampled)
        if sync_timers:
            self._sync()
        t2 = time.perf_counter()
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        self.stat_info["sum_training_flops"] += int(self.cfg.epochs * sum(self.sizes[c] for c in sampled))
        self.end_of_training(round_idx, sampled)
        res = None
        if self._eval_due(round_idx):
            res = self.evaluate(round_idx)
            if sync_timers:
                self._sync()
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return res

    def end_of_training(self, round_idx, clients):
        """Round bookkeeping after local training: the reference's per-client log lines and, when logging (or on
        the CPU), ``sum_comm_params`` folded into ``stat_info``.  Timed GPU runs without a logger never sync here;
        their counts are folded in by :meth:`finish` / :meth:`sync_stats`."""
        self.flush_round_log(round_idx, clients, comm_lines=self.alg in ("salientgrads", "fedavg"))
        if self.log is not None or self.device.type != "cuda":
            self.sync_stats()

    def finetune_round(self):
        """FedAvg's final "fine-tune" pass (``fedavg_api.py:78-88``): every client trains one more local round from
        the final w_global (the reference passes round -1, so lr = lr / lr_decay) and the global model plus these
        fine-tuned personal models are evaluated; w_global is unchanged."""
        rows, loc = self._local_rows(range(self.N))
        if not rows:
            return self.evaluate(-1)
        fin = RowSet(padded_rows(self.C, self.P, self.device), padded_rows(self.C, self.Q, self.device))
        fin.theta.copy_(self.w_global.expand(self.C, -1))
        fin.bufs.copy_(self.b_global.expand(self.C, -1))
        self.train_rows(fin, rows, loc, -1, self.cfg.epochs, self._fedavg_spec(), tag=3)
        self.flush_round_log(-1, loc, comm_lines=False)
        return self.evaluate(-1, fin.theta, fin.bufs)

    def train(self):
        if self.alg == "salientgrads":
            self.generate_global_mask_snip()
        for r in range(self.cfg.comm_round):
            self.run_round(r)
        self.finish()
        return self.stat_info

    def finish(self):
        """Reference round tail: SalientGrads re-evaluates (``sailentgrads_api.py:147``), FedAvg fine-tunes every
        client once more and evaluates (``fedavg_api.py:78-88``)."""
        self.sync_stats()
        if not self.cfg.final_round:
            return None
        if self.alg == "salientgrads":
            return self.evaluate(-1)
        return self.finetune_round()
