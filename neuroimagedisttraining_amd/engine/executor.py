"""Client-batched FL executor: many virtual clients per GPU, one process per GPU, RCCL aggregation.

This is the MI355X-native replacement of the reference's sequential client loop
(``sailentgrads_api.py:86-147`` / ``fedavg_api.py:40-88``): instead of swapping one shared ``nn.Module``'s
state_dict per client and copying weights host<->device, every rank keeps its shard of clients resident
as rows of ``theta [C_local, P]`` (params) and ``bufs [C_local, Q]`` (BN running stats) and trains all of
them in lockstep — one launch sequence per local step for the whole shard.

Round semantics reproduced from the reference (SURVEY.md §2.2 "Shared algorithm behaviors"):
* client sampling ``np.random.seed(round); choice(total, per_round, replace=False)`` (all if frac=1);
* every sampled client starts from ``w_global``; SGD(lr * lr_decay**round, momentum, wd) rebuilt per round
  (momentum never carries over, Q4); ``clip_grad_norm_(10)``; SalientGrads multiplies weights by the global
  SNIP mask after every step (Q2);
* one DataLoader(shuffle=True) pass per epoch over the client's train split (last batch may be partial);
* aggregation: sample-weighted average over ALL state entries incl. BN running stats and
  ``num_batches_tracked`` (Q3) — a local weighted row-sum followed by ONE all-reduce of P+Q floats;
* evaluation: global model and each client's last local ("personal") model on that client's test split;
  logged loss uses sigmoid-then-BCEWithLogits (Q1); metrics are unweighted means over clients (Q5).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as R
from ..parallel import runtime as rt
from .flat import ParamLayout


# ------------------------------------------------------------------------------------------------
@dataclass
class ClientSplit:
    """Global sample indices of one client (into the engine's data store)."""
    train: np.ndarray
    test: np.ndarray


@dataclass
class FLConfig:
    comm_round: int = 200
    epochs: int = 2
    batch_size: int = 16
    lr: float = 0.01
    lr_decay: float = 0.998
    wd: float = 5e-4
    momentum: float = 0.0
    max_norm: float = 10.0
    frac: float = 1.0
    dense_ratio: float = 0.5
    itersnip_iteration: int = 1
    snip_mask: bool = True
    dropout_keep: float = 0.5
    frequency_of_the_test: int = 1
    seed: int = 1024
    prox_mu: float = 0.0          # FedProx proximal coefficient (0 = FedAvg/SalientGrads)
    group: int = 0                # max clients per lockstep launch (0 = all local clients)
    test_batch: int = 256
    aggregator: str = "fedavg"    # fedavg | krum | multikrum | median | trimmed_mean (BASELINE config 4)
    byzantine_f: int = 0          # Krum's assumed number of Byzantine clients
    multikrum_m: int = 0          # Multi-Krum: number of selected clients (0 = K - f)
    trim_ratio: float = 0.1       # trimmed mean: fraction cut from each end per coordinate
    sparse_aggregate: bool = True  # SalientGrads: all-reduce only the coordinates kept by the global mask
    update_topk: float = 0.0      # >0: each client sends only its top-k |update| (values + int32 indices,
                                  # k = update_topk * P) through an RCCL all-gather (BASELINE config 5)
    hip_graphs: bool = True       # capture each lockstep local step (train + optimizer) in a hipGraph and replay it
    heartbeat_s: float = 0.0      # >0: ranks publish heartbeats every heartbeat_s through the process group's store and
                                  # each round fails fast (comm.failure.PeerFailure) if a peer is silent for 30x that


# ------------------------------------------------------------------------------------------------
class HipEngine:
    """AlexNet3D_Dropout on the gfx950 kernels (ABCD-shape volumes, polyphase uint8 store)."""

    def __init__(self, template_model, x8, mom, labels, device):
        from .alexnet_hip import HipAlexNet3D
        self.players = ParamLayout.from_tensors(list(template_model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(template_model.named_buffers()))
        self.net = HipAlexNet3D(self.players, self.blayers, device)
        self.x8, self.mom, self.labels = x8, mom, labels
        self.device = torch.device(device)
        self.m = ops.ext()
        self._cid_cache = {}

    supports_graphs = True

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None):
        y = self.labels.index_select(0, idx.long())
        ct = None
        if cids is not None:
            key = tuple(int(c) for c in cids)
            ct = self._cid_cache.get(key)
            if ct is None:  # one upload per client group, reused by every step
                ct = torch.tensor(key, dtype=torch.int32, device=self.device)
                self._cid_cache[key] = ct
        return self.net.train_step(theta, bufs, grads, self.x8, self.mom, idx, y, G, B, keep, seed, ct, seed_dev)

    def eval_logits(self, theta, bufs, idx, G, B):
        return self.net.eval_logits(theta, bufs, self.x8, idx, G, B)

    # fused optimizer: clip(10) -> SGD(wd, momentum) -> w *= mask (one HIP pass per row)
    def opt_step(self, theta, grads, mom_buf, mask, lr, wd, momentum, first, max_norm, lr_dev=None, keep_grad=False):
        """Fused clip + SGD (+ momentum) + mask.  The clipped gradient is only written back with ``keep_grad`` (the
        local step overwrites ``grads`` next time; skipping the write saves 4 B/param of HBM traffic)."""
        G, P = theta.shape
        ws = self.m.clip_sgd_mask_workspace(G, P)
        if not hasattr(self, "_optws") or self._optws.numel() < ws:
            self._optws = torch.empty(ws, dtype=torch.float32, device=theta.device)
        self.m.clip_sgd_mask(theta.data_ptr(), grads.data_ptr(), mom_buf.data_ptr() if mom_buf is not None else 0,
                             mask.data_ptr() if mask is not None else 0, self._optws.data_ptr(), 0, 0, G, P,
                             theta.stride(0), float(lr), float(wd), float(momentum), int(first), float(max_norm),
                             lr_dev.data_ptr() if lr_dev is not None else 0, int(keep_grad),
                             torch.cuda.current_stream().cuda_stream)

    def saliency_acc(self, theta, grads, score, alpha):
        G, P = theta.shape
        self.m.saliency_acc(theta.data_ptr(), grads.data_ptr(), theta.stride(0), P, G, float(alpha),
                            score.data_ptr(), score.stride(0), torch.cuda.current_stream().cuda_stream)


class TorchEngine:
    """Any ``nn.Module`` (reference-semantics eager path; CPU tests, 2D CNN families, baselines).

    ``store``: float tensor ``[N, ...]`` of inputs (already scaled); ``labels``: ``[N]``.
    ``loss``: ``"bce"`` (class_num=1, logits [B,1]) or ``"ce"`` (multi-class)."""

    def __init__(self, template_model, store, labels, device, loss="bce", dtype=torch.float32, amp=False):
        self.model = template_model.to(device)
        # amp: bf16 autocast for the forward/backward (fp32 master rows, fp32 optimizer) on MIOpen
        self.amp = bool(amp) and torch.device(device).type == "cuda"
        self.players = ParamLayout.from_tensors(list(self.model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(self.model.named_buffers()))
        self.store, self.labels, self.device, self.loss, self.dtype = store, labels, torch.device(device), loss, dtype

    def _views(self, row, layout):
        return {n: row[o:o + layout.numel(i)].view(layout.shapes[i])
                for i, (n, o) in enumerate(zip(layout.names, layout.offsets))}

    def _batch(self, idx):
        x = self.store.index_select(0, idx.long().to(self.store.device)).to(self.device)
        if x.dtype == torch.uint8:
            x = x.to(self.dtype) / 255.0
        if x.dim() == 4:  # volumes without channel dim
            x = x.unsqueeze(1)
        y = self.labels.index_select(0, idx.long().to(self.labels.device)).to(self.device)
        return x.to(self.dtype), y

    def _loss(self, out, y):
        if self.loss == "bce":
            return F.binary_cross_entropy_with_logits(out.float().view(-1, 1), y.float().view(-1, 1))
        return F.cross_entropy(out.float(), y.long())

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None):
        from torch.func import functional_call
        losses = torch.zeros(G, device=theta.device)
        self.model.train()
        for g in range(G):
            # dropout stream keyed by (step seed, global client id): independent of how clients are sharded
            cid = int(cids[g]) if cids is not None else g
            torch.manual_seed((int(seed) * 1000003 + cid) & 0x7fffffffffff)
            row = theta[g].detach().clone().requires_grad_(True)
            pv = self._views(row, self.players)
            # separate buffer tensors: in-place running-stat updates on views of one row would bump a shared
            # version counter that autograd checks; results are copied back into the row afterwards
            bview = self._views(bufs[g], self.blayers)
            bv = {k: v.clone() for k, v in bview.items()}
            x, y = self._batch(idx[g * B:(g + 1) * B])
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
                out = functional_call(self.model, {**pv, **bv}, (x,))
            if isinstance(out, (list, tuple)):
                out = out[0]
            loss = self._loss(out, y)
            loss.backward()
            with torch.no_grad():
                for k, v in bv.items():
                    bview[k].copy_(v)
            grads[g].copy_(row.grad)
            losses[g] = loss.detach()
        return losses

    def eval_logits(self, theta, bufs, idx, G, B):
        from torch.func import functional_call
        self.model.eval()
        outs = []
        with torch.no_grad():
            for g in range(G):
                pv = self._views(theta[g], self.players)
                bv = self._views(bufs[g].clone(), self.blayers)
                x, _ = self._batch(idx[g * B:(g + 1) * B])
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
                    out = functional_call(self.model, {**pv, **bv}, (x,))
                if isinstance(out, (list, tuple)):
                    out = out[0]
                outs.append(out.float())
        return torch.cat(outs, 0)

    def opt_step(self, theta, grads, mom_buf, mask, lr, wd, momentum, first, max_norm):
        for g in range(theta.shape[0]):
            gn = float(grads[g].norm())
            coef = min(1.0, max_norm / (gn + 1e-6))
            d = grads[g] * coef + wd * theta[g]
            if momentum != 0 and mom_buf is not None:
                if first:
                    mom_buf[g].copy_(d)
                else:
                    mom_buf[g].mul_(momentum).add_(d)
                d = mom_buf[g]
            theta[g].add_(d, alpha=-lr)
            if mask is not None:
                theta[g].mul_(mask)

    def saliency_acc(self, theta, grads, score, alpha):
        score.add_((theta * grads).abs() * alpha)


# ------------------------------------------------------------------------------------------------
def padded_rows(n, width, device, align=64, dtype=torch.float32):
    """``[n, width]`` zero view whose row stride is a multiple of ``align`` floats (16-B aligned rows for the
    vectorised HIP kernels; P = 2,570,241 for AlexNet3D is odd)."""
    ld = (width + align - 1) // align * align
    return torch.zeros((n, ld), dtype=dtype, device=device)[:, :width]


def gather_rows(src, ix):
    out = padded_rows(ix.numel(), src.shape[1], src.device, dtype=src.dtype)
    out.copy_(src.index_select(0, ix))
    return out


def maskable_flat_mask(layout: ParamLayout, names):
    """Boolean [P] marking the maskable (conv / linear weight) entries, in layout order."""
    m = torch.zeros(layout.total, dtype=torch.bool)
    for i, n in enumerate(layout.names):
        if n in names:
            m[layout.offsets[i]:layout.offsets[i] + layout.numel(i)] = True
    return m


def snip_maskable_names(model):
    out = []
    for name, mod in model.named_modules():
        if isinstance(mod, (torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d, torch.nn.Linear)):
            out.append(name + ".weight")
    return out


class FLRunner:
    """SalientGrads / FedAvg / FedProx over client-sharded, client-batched local training."""

    def __init__(self, engine, splits, cfg: FLConfig, info: rt.DistInfo, template_model, logger=None,
                 algorithm="salientgrads"):
        self.e, self.cfg, self.info, self.log = engine, cfg, info, logger
        self.alg = algorithm
        self.N = len(splits)
        self.splits = splits
        self.device = info.device
        self.shards = rt.shard_clients([len(s.train) for s in splits], info.world)
        self.local = self.shards[info.rank]
        self.C = len(self.local)
        P, Q = engine.players.total, engine.blayers.total
        self.P, self.Q = P, Q
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
        self.mask = None
        self.maskable = maskable_flat_mask(engine.players, snip_maskable_names(template_model)).to(self.device)
        self.stat_info = dict(sum_comm_params=0, sum_training_flops=0, global_test_acc=[], person_test_acc=[],
                              global_test_loss=[], person_test_loss=[], round_time=[])
        self.timers = {"train": 0.0, "aggregate": 0.0, "eval": 0.0, "snip": 0.0}
        self._step_seed = 0
        self._graphs = {}          # (rows, G, B) -> captured local step (None until the shape repeats)
        self._lr_dev = self._seed_dev = None

    # ---------------------------------------------------------------------------------------------
    def _rng(self, *key):
        return np.random.RandomState(abs(hash((self.cfg.seed,) + tuple(int(k) for k in key))) % (2 ** 31))

    def _groups(self, rows):
        gmax = self.cfg.group or len(rows)
        return [rows[i:i + gmax] for i in range(0, len(rows), gmax)]

    def _run_batches(self, rows, clients, round_idx, epoch_tag, fn, n_batches=None):
        """Iterate lockstep local steps over ``clients`` (global ids) living in ``rows`` (local row ids).
        ``fn(row_slice_or_index, idx_tensor, G, B)`` is called per (group, step)."""
        B = self.cfg.batch_size
        orders = []
        for c in clients:
            tr = self.splits[c].train
            perm = self._rng(round_idx, c, epoch_tag).permutation(len(tr))
            orders.append(tr[perm])
        nsteps = max(int(math.ceil(len(o) / B)) for o in orders) if orders else 0
        if n_batches is not None:
            nsteps = min(nsteps, n_batches)
        # Plan every (step, group) launch first and upload all sample indices in ONE pinned, non-blocking
        # copy: a per-step pageable host->device copy would synchronise the host with the GPU every local
        # step and expose the next step's launch latency.
        plan, chunks, off = [], [], 0
        for s in range(nsteps):
            by_size = {}
            for r, o in zip(rows, orders):
                chunk = o[s * B:(s + 1) * B]
                if len(chunk):
                    by_size.setdefault(len(chunk), []).append((r, chunk))
            for bsz, items in sorted(by_size.items(), reverse=True):
                for grp in self._groups(items):
                    n = sum(len(ch) for _, ch in grp)
                    plan.append(([r for r, _ in grp], off, n, len(grp), bsz))
                    chunks.extend(ch for _, ch in grp)
                    off += n
        if not plan:
            return
        all_idx = self._upload_i32(np.concatenate(chunks))
        for rr, o, n, G, bsz in plan:
            fn(rr, all_idx[o:o + n], G, bsz)

    def _upload_i32(self, arr):
        """int32 host array -> device tensor through pinned memory, without blocking the host."""
        t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32))
        if self.device.type != "cuda":
            return t
        return t.pin_memory().to(self.device, non_blocking=True)

    def _with_rows(self, rr, body):
        """Run ``body(theta, bufs, grads, mom)`` on rows ``rr`` (in place when they are a contiguous run)."""
        lo, hi = rr[0], rr[-1] + 1
        if rr == list(range(lo, hi)):
            return body(self.theta[lo:hi], self.bufs[lo:hi], self.grads[lo:hi],
                        self.mom_buf[lo:hi] if self.mom_buf is not None else None)
        ix = torch.tensor(rr, device=self.device)
        th, bu, gr = gather_rows(self.theta, ix), gather_rows(self.bufs, ix), gather_rows(self.grads, ix)
        mo = gather_rows(self.mom_buf, ix) if self.mom_buf is not None else None
        out = body(th, bu, gr, mo)
        self.theta[ix] = th
        self.bufs[ix] = bu
        if mo is not None:
            self.mom_buf[ix] = mo
        return out

    # ---------------------------------------------------------------------------------------------
    def generate_global_mask_snip(self):
        """IterSNIP saliency on every client (mean over iterations, then clients) -> global top-k mask
        (``sailentgrads_api.py:47-66``, ``snip.py:21-116``)."""
        t0 = time.perf_counter()
        cfg = self.cfg
        score = torch.zeros((max(1, self.C), self.P), dtype=torch.float32, device=self.device)
        rows = list(range(self.C))
        self.theta.copy_(self.w_global.unsqueeze(0).expand_as(self.theta))
        saved_bufs = self.bufs.clone()
        for it in range(cfg.itersnip_iteration):
            # "next(iter(train_loader))": the first batch of a fresh shuffle
            def fn(rr, idx, G, B):
                def body(th, bu, gr, mo):
                    self._step_seed += 1
                    self.e.train_step(th, bu, gr, idx, G, B, cfg.dropout_keep, (cfg.seed << 20) + self._step_seed,
                                      cids=[self.local[r] for r in rr])
                    lo, hi = rr[0], rr[-1] + 1
                    self.e.saliency_acc(th, gr, score[lo:hi] if rr == list(range(lo, hi)) else score[rr],
                                        1.0 / cfg.itersnip_iteration)
                self._with_rows(rr, body)
            self._run_batches(rows, self.local, -1, it, fn, n_batches=1)
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
                m = self.e.m
                st = torch.empty(4, dtype=torch.int32, device=self.device)
                hist = torch.empty(256, dtype=torch.int32, device=self.device)
                sel = sel.contiguous()
                m.radix_select_kth(sel.data_ptr(), sel.numel(), k, st.data_ptr(), hist.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
                keep = torch.empty_like(sel)
                m.threshold_mask(sel.data_ptr(), sel.numel(), st.data_ptr(), keep.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
            else:
                thr = torch.topk(sel, k, sorted=True).values[-1]
                keep = (sel >= thr).float()
            mask[self.maskable] = keep
        self.mask = mask if cfg.snip_mask else torch.ones_like(mask)
        self._graphs = {}  # captured local steps reference the mask tensor
        self.timers["snip"] += time.perf_counter() - t0
        return self.mask

    # ---------------------------------------------------------------------------------------------
    def sample_clients(self, round_idx):
        per_round = max(1, int(self.N * self.cfg.frac))
        if per_round >= self.N:
            return list(range(self.N))
        np.random.seed(round_idx)
        return sorted(np.random.choice(range(self.N), per_round, replace=False).tolist())

    def local_train(self, round_idx, sampled):
        cfg = self.cfg
        loc = [c for c in self.local if c in set(sampled)]
        rows = [self.local.index(c) for c in loc]
        if not rows:
            return
        if rows == list(range(rows[0], rows[-1] + 1)):  # one broadcast launch for the whole shard
            self.theta[rows[0]:rows[-1] + 1].copy_(self.w_global.expand(len(rows), -1))
            self.bufs[rows[0]:rows[-1] + 1].copy_(self.b_global.expand(len(rows), -1))
        else:
            for r in rows:
                self.theta[r].copy_(self.w_global)
                self.bufs[r].copy_(self.b_global)
        lr = cfg.lr * (cfg.lr_decay ** round_idx)
        first = [True]
        use_graphs = (cfg.hip_graphs and getattr(self.e, "supports_graphs", False) and self.device.type == "cuda"
                      and cfg.momentum == 0)
        if use_graphs:
            if self._lr_dev is None:
                self._lr_dev = torch.zeros(1, dtype=torch.float32, device=self.device)
                self._seed_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._lr_dev.fill_(lr)
        for ep in range(cfg.epochs):
            def fn(rr, idx, G, B):
                if use_graphs and rr == list(range(rr[0], rr[-1] + 1)):
                    self._graph_step(rr, idx, G, B)
                    first[0] = False
                    return

                def body(th, bu, gr, mo):
                    self._step_seed += 1
                    if cfg.prox_mu > 0:
                        w_ref = self.w_global
                    self.e.train_step(th, bu, gr, idx, G, B, cfg.dropout_keep, (cfg.seed << 20) + self._step_seed,
                                      cids=[self.local[r] for r in rr])
                    if cfg.prox_mu > 0:
                        gr.add_(th - w_ref.unsqueeze(0), alpha=cfg.prox_mu)
                    self.e.opt_step(th, gr, mo, self.mask if self.alg == "salientgrads" else None, lr, cfg.wd,
                                    cfg.momentum, first[0], cfg.max_norm)
                self._with_rows(rr, body)
                first[0] = False
            self._run_batches(rows, loc, round_idx, ep, fn)

    def _graph_step(self, rr, idx, G, B):
        """One lockstep local step (forward+backward of G clients, FedProx term, clip+SGD+mask) as a replayed
        hipGraph.  The ~45 kernel launches of a step become one graph launch; everything that changes between
        steps lives in device memory the graph reads: the sample indices (copied into a static buffer), the
        dropout stream counter and the round's learning rate.  The first step of a (rows, G, B) shape runs
        eagerly (it also allocates every scratch buffer the graph will reuse), the second is captured and
        replayed, later ones only replay — same kernels, same arguments, same results as the eager path."""
        cfg = self.cfg
        lo, hi = rr[0], rr[-1] + 1
        key = (lo, hi, G, B)
        self._step_seed += 1
        ent = self._graphs.get(key, "new")
        th, bu, gr = self.theta[lo:hi], self.bufs[lo:hi], self.grads[lo:hi]
        mask = self.mask if self.alg == "salientgrads" else None
        cids = [self.local[r] for r in rr]
        base = cfg.seed << 20

        def step(idx_t, seed_dev):
            self.e.train_step(th, bu, gr, idx_t, G, B, cfg.dropout_keep, base, cids=cids, seed_dev=seed_dev)
            if cfg.prox_mu > 0:
                gr.add_(th - self.w_global.unsqueeze(0), alpha=cfg.prox_mu)
            self.e.opt_step(th, gr, None, mask, 0.0, cfg.wd, 0.0, True, cfg.max_norm, lr_dev=self._lr_dev)

        self._seed_dev.fill_(self._step_seed)
        if ent == "new":  # eager warm-up step: allocates the per-shape scratch the capture will reuse
            step(idx, self._seed_dev)
            self._graphs[key] = None
            return
        if ent is None:
            idx_buf = torch.empty(G * B, dtype=torch.int32, device=self.device)
            idx_buf.copy_(idx)
            torch.cuda.current_stream().synchronize()
            g = torch.cuda.CUDAGraph()
            try:
                # thread_local: the RCCL watchdog thread of a multi-GPU run may query events during the capture
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    step(idx_buf, self._seed_dev)
            except Exception:  # noqa: BLE001 - capture unsupported here: stay eager for this shape
                self._graphs[key] = False
                step(idx, self._seed_dev)
                return
            ent = self._graphs[key] = (g, idx_buf)
        elif ent is False:
            step(idx, self._seed_dev)
            return
        g, idx_buf = ent
        idx_buf.copy_(idx)
        g.replay()

    def aggregate(self, sampled):
        if self.cfg.aggregator != "fedavg":
            return self.aggregate_robust(sampled)
        if self.cfg.update_topk > 0:
            return self.aggregate_topk(sampled)
        return self.aggregate_fedavg(sampled)

    def aggregate_topk(self, sampled):
        """Sparse-update FedAvg: client i contributes n_i/N * topk(theta_i - w_global) (fixed k per client, so
        the all-gather needs no padding), BN buffers are averaged densely.  Every rank applies the same
        gathered (index, value) lists in global client order, so all ranks end with the same model."""
        sset = set(sampled)
        n_tot = float(sum(len(self.splits[c].train) for c in sampled))
        k = max(1, int(math.ceil(self.cfg.update_topk * self.P)))
        rows = [i for i, c in enumerate(self.local) if c in sset]
        vals = torch.zeros((len(rows), k), dtype=torch.float32, device=self.device)
        idx = torch.zeros((len(rows), k), dtype=torch.int32, device=self.device)
        for j, r in enumerate(rows):
            d = self.theta[r, :self.P] - self.w_global
            top = torch.topk(d.abs(), k, sorted=False).indices
            idx[j] = top.int()
            vals[j] = d.index_select(0, top) * (len(self.splits[self.local[r]].train) / n_tot)
        cid = torch.tensor([self.local[r] for r in rows], dtype=torch.float32, device=self.device)
        g_vals = rt.all_gather_cat(vals.view(-1), self.info).view(-1, k)
        g_idx = rt.all_gather_cat(idx.view(-1), self.info).view(-1, k).long()
        g_cid = rt.all_gather_cat(cid, self.info)
        order = torch.argsort(g_cid)
        upd = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        for j in order.tolist():  # fixed order: identical fp32 sums on every rank
            upd.index_add_(0, g_idx[j], g_vals[j])
        self.w_global.add_(upd)
        bsum = torch.zeros(self.Q, dtype=torch.float32, device=self.device)
        for r in rows:
            bsum.add_(self.bufs[r, :self.Q], alpha=len(self.splits[self.local[r]].train) / n_tot)
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

    def aggregate_fedavg(self, sampled):
        """w_global = sum_i n_i/sum n * w_i over sampled clients (params + buffers), one all-reduce (of the
        mask-compacted coordinates when a SalientGrads mask is active)."""
        sset = set(sampled)
        n_tot = float(sum(len(self.splits[c].train) for c in sampled))
        Pp = (self.P + 63) // 64 * 64  # keep the buffer section 16-B aligned for the vectorised kernel
        buf = torch.zeros(Pp + self.Q, dtype=torch.float32, device=self.device)
        rows = [i for i, c in enumerate(self.local) if c in sset]
        if rows:
            w = torch.tensor([len(self.splits[self.local[r]].train) / n_tot for r in rows], dtype=torch.float32,
                             device=self.device)
            ix = torch.tensor(rows, device=self.device)
            if self.device.type == "cuda" and rows == list(range(rows[0], rows[-1] + 1)):
                m, st = self.e.m, torch.cuda.current_stream().cuda_stream
                lo = rows[0]
                m.weighted_rows_sum(self.theta[lo].data_ptr(), w.data_ptr(), len(rows), self.P, self.theta.stride(0),
                                    0.0, buf.data_ptr(), st)
                m.weighted_rows_sum(self.bufs[lo].data_ptr(), w.data_ptr(), len(rows), self.Q, self.bufs.stride(0),
                                    0.0, buf[Pp:].data_ptr(), st)
            else:
                buf[:self.P] = (w.view(-1, 1) * self.theta[ix]).sum(0)
                buf[Pp:] = (w.view(-1, 1) * self.bufs[ix]).sum(0)
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
        sset = set(sampled)
        rows = [i for i, c in enumerate(self.local) if c in sset]
        ids = torch.tensor([self.local[r] for r in rows], dtype=torch.float32, device=self.device)
        W = self.P + self.Q
        loc = torch.cat([self.theta[rows, :self.P], self.bufs[rows, :self.Q]], 1) if rows else \
            torch.zeros((0, W), device=self.device)
        allrows = rt.all_gather_cat(loc.reshape(-1).contiguous(), self.info).view(-1, W)
        allids = rt.all_gather_cat(ids, self.info).long()
        order = torch.argsort(allids)  # deterministic client order on every rank
        M = allrows.index_select(0, order)
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

    def _eval_rows(self, theta, bufs, clients, per_client_rows):
        """Per-client (correct, loss_sum, total) with reference test semantics (Q1).  Clients that share a
        model row are evaluated together in chunks of ``test_batch`` samples (one launch sequence each)."""
        out = np.zeros((len(clients), 3), dtype=np.float64)
        by_row = {}
        for j, r in enumerate(per_client_rows):
            by_row.setdefault(r, []).append(j)
        for r, js in by_row.items():
            tests = [self.splits[clients[j]].test for j in js]
            owner = np.concatenate([np.full(len(t), k) for k, t in enumerate(tests)]).astype(np.int64)
            allidx = np.concatenate(tests).astype(np.int32) if tests else np.zeros(0, np.int32)
            if allidx.size == 0:
                continue
            th, bu = theta[r:r + 1], bufs[r:r + 1]
            tb = self.cfg.test_batch
            acc = torch.zeros((len(js), 3), dtype=torch.float64, device=self.device)
            own_t = torch.from_numpy(owner).to(self.device)
            all_t = self._upload_i32(allidx)
            for s in range(0, allidx.size, tb):
                idx = all_t[s:s + tb]
                logits = self.e.eval_logits(th, bu, idx, 1, idx.numel()).view(-1)
                y = self.e.labels.index_select(0, idx.long()).to(logits.device).float()
                pred = torch.sigmoid(logits)
                loss = F.binary_cross_entropy_with_logits(pred, y, reduction="none")
                correct = ((pred >= 0.5).float() == y).float()
                o = own_t[s:s + idx.numel()]
                acc[:, 0].index_add_(0, o, correct.double())
                acc[:, 1].index_add_(0, o, loss.double())
                acc[:, 2].index_add_(0, o, torch.ones_like(loss, dtype=torch.float64))
            out[js] = acc.cpu().numpy()
        return out

    def _eval_grouped(self, theta, bufs, rows, clients):
        """Personal models: clients with equal test sizes are evaluated in one grouped launch."""
        out = np.zeros((len(clients), 3), dtype=np.float64)
        pending = []  # (client positions, device result): one device->host copy at the end
        sizes = {}
        for j, c in enumerate(clients):
            sizes.setdefault(len(self.splits[c].test), []).append(j)
        for n, js in sizes.items():
            if n == 0:
                continue
            if n > self.cfg.test_batch or rows != list(range(rows[0], rows[0] + len(rows))):
                res = self._eval_rows(theta, bufs, [clients[j] for j in js], [rows[j] for j in js])
                out[js] = res
                continue
            for grp in self._groups(js):
                rr = [rows[j] for j in grp]
                lo, hi = rr[0], rr[-1] + 1
                if rr != list(range(lo, hi)):
                    out[grp] = self._eval_rows(theta, bufs, [clients[j] for j in grp], rr)
                    continue
                idx = self._upload_i32(np.concatenate([self.splits[clients[j]].test for j in grp]))
                logits = self.e.eval_logits(theta[lo:hi], bufs[lo:hi], idx, len(grp), n).view(len(grp), n)
                y = self.e.labels.index_select(0, idx.long()).to(logits.device).float().view(len(grp), n)
                pred = torch.sigmoid(logits)
                loss = F.binary_cross_entropy_with_logits(pred, y, reduction="none").sum(1)
                correct = ((pred >= 0.5).float() == y).float().sum(1)
                pending.append((grp, torch.stack([correct, loss, torch.full_like(loss, n)], 1).double()))
        if pending:
            host = torch.cat([r for _, r in pending], 0).cpu().numpy()
            o = 0
            for grp, r in pending:
                out[grp] = host[o:o + len(grp)]
                o += len(grp)
        return out

    def _eval_global_and_personal(self):
        """Global model and every local client's personal model on that client's test split, in ONE grouped
        launch sequence of 2C model rows (C personal rows + C copies of the global model).  Compared with
        evaluating the single global row in test_batch chunks (G = 1) this keeps the kernels at full-client
        shapes — it matters most at 8 clients per GPU.  Returns (glob, pers) or None when test sizes differ."""
        C = self.C
        sizes = {len(self.splits[c].test) for c in self.local}
        if len(sizes) != 1 or next(iter(sizes)) > self.cfg.test_batch or next(iter(sizes)) == 0:
            return None
        if getattr(self, "_eval_rows2", None) is None or self._eval_rows2[0].shape[0] != 2 * C:
            self._eval_rows2 = (padded_rows(2 * C, self.P, self.device), padded_rows(2 * C, self.Q, self.device))
        th, bu = self._eval_rows2
        with torch.no_grad():
            th[:C].copy_(self.theta[:C])
            th[C:].copy_(self.w_global.expand(C, -1))
            bu[:C].copy_(self.bufs[:C])
            bu[C:].copy_(self.b_global.expand(C, -1))
        res = self._eval_grouped(th, bu, list(range(2 * C)), self.local + self.local)
        return res[C:], res[:C]

    def evaluate(self, round_idx):
        t0 = time.perf_counter()
        both = self._eval_global_and_personal() if self.C else None
        if both is not None:
            glob, pers = both
        else:
            gth = padded_rows(1, self.P, self.device)
            gth.copy_(self.w_global.unsqueeze(0))
            gbu = padded_rows(1, self.Q, self.device)
            gbu.copy_(self.b_global.unsqueeze(0))
            glob = self._eval_rows(gth, gbu, self.local, [0] * self.C) if self.C else np.zeros((0, 3))
            pers = self._eval_grouped(self.theta, self.bufs, list(range(self.C)), self.local) if self.C else \
                np.zeros((0, 3))
        res = torch.zeros((self.N, 6), dtype=torch.float64, device=self.device)
        if self.C:
            res[torch.tensor(self.local, device=self.device)] = torch.from_numpy(
                np.concatenate([glob, pers], 1)).to(self.device)
        rt.all_reduce_buckets(res, self.info)
        r = res.cpu().numpy()
        ok = r[:, 2] > 0
        g_acc = float(np.mean(r[ok, 0] / r[ok, 2])) if ok.any() else 0.0
        g_loss = float(np.mean(r[ok, 1] / r[ok, 2])) if ok.any() else 0.0
        okp = r[:, 5] > 0
        p_acc = float(np.mean(r[okp, 3] / r[okp, 5])) if okp.any() else 0.0
        p_loss = float(np.mean(r[okp, 4] / r[okp, 5])) if okp.any() else 0.0
        self.stat_info["global_test_acc"].append(g_acc)
        self.stat_info["global_test_loss"].append(g_loss)
        self.stat_info["person_test_acc"].append(p_acc)
        self.stat_info["person_test_loss"].append(p_loss)
        if self.log is not None and self.info.is_main:
            self.log.info({"global_test_acc": g_acc, "global_test_loss": g_loss})
            self.log.info({"person_test_acc": p_acc, "person_test_loss": p_loss})
        self.timers["eval"] += time.perf_counter() - t0
        return dict(global_test_acc=g_acc, global_test_loss=g_loss, person_test_acc=p_acc, person_test_loss=p_loss)

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

    def run_round(self, round_idx, sync_timers=False):
        t0 = time.perf_counter()
        hb = self._heartbeat()
        if hb is not None:
            hb.check_or_raise()  # before the round's collectives: a dead peer would block them until the timeout
        sampled = self.sample_clients(round_idx)
        if self.log is not None and self.info.is_main:
            self.log.info("################Communication round : {}".format(round_idx))
            self.log.info("client_indexes = " + str(np.array(sampled)))
        self.local_train(round_idx, sampled)
        if sync_timers and self.device.type == "cuda":
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        self.aggregate(sampled)
        if sync_timers and self.device.type == "cuda":
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        self.timers["train"] += t1 - t0
        self.timers["aggregate"] += t2 - t1
        res = None
        if self.cfg.frequency_of_the_test and (round_idx % self.cfg.frequency_of_the_test == 0):
            res = self.evaluate(round_idx)
        self.stat_info["round_time"].append(time.perf_counter() - t0)
        return res

    def train(self):
        if self.alg == "salientgrads":
            self.generate_global_mask_snip()
        for r in range(self.cfg.comm_round):
            self.run_round(r)
        return self.stat_info
