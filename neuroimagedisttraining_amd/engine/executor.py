"""Client-batched FL executor: engines (the per-model compute of one lockstep step) and the run configuration.

The round driver (sharding, lockstep planning, hipGraphs, aggregation, evaluation) is ``engine/runner.py``; the
personalized / decentralized algorithms are ``engine/personalized.py``.

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
import os
import time
from dataclasses import dataclass, field
from typing import Optional

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
    val: np.ndarray = None   # FedFomo's validation split (cifar10/data_val_loader.py:275-278)


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
    # capture each lockstep local step (train + optimizer) in a hipGraph and replay it: True / False force it,
    # None = the engine's measured default (``graphs_default``: on for AlexNet3D, off for ResNet-18-GN)
    hip_graphs: Optional[bool] = None
    step_streams: int = 4         # side HIP streams for the extra launches of one lockstep step (ragged clients)
    stratified_sampling: bool = False  # IterSNIP: label-stratified SNIP batches (sailentgrads/client.py:33-43)
    fix_eval_loss: bool = False   # evaluation loss on logits instead of the reference's sigmoid-then-BCEWithLogits (Q1)
    final_round: bool = True      # reference round tail: SalientGrads final eval, FedAvg fine-tune round + eval
    # ---- personalized / decentralized algorithms (engine/personalized.py), reference flag names
    cs: str = "ring"              # D-PSGD neighbour topology: ring | random | full
    lamda: float = 0.5            # Ditto proximal pull
    local_epochs: int = 0         # Ditto personal epochs (0 = epochs)
    anneal_factor: float = 0.5    # DisPFL cosine-annealed drop ratio
    active: float = 1.0           # DisPFL client availability
    static: bool = False          # DisPFL: fixed masks (no fire / regrow)
    dis_gradient_check: bool = False  # DisPFL: random regrow instead of top |g|
    uniform: bool = False         # DisPFL: uniform instead of ERK per-layer density
    different_initial: bool = False   # DisPFL: per-client random initial masks
    diff_spa: bool = False        # DisPFL: per-client density from {0.2, 0.4, 0.6, 0.8, 1.0}
    erk_power_scale: float = 1.0
    save_masks: bool = False
    dispfl_aggregate: bool = False    # DisPFL: enable the masked neighbour average (disabled in the reference, Q10)
    each_prune_ratio: float = 0.05    # SubAvg fake_prune percentile
    dist_thresh: float = 1e-4         # SubAvg: prune only if the mask moved more than this
    acc_thresh: float = 0.5           # SubAvg: and the pruned model's local training accuracy exceeds this
    rebalance: bool = False       # multi-rank, frac < 1: before each round move the sampled clients' state (rows, masks)
                                  # and their samples (engine.sample_fields) so every rank trains about the same
                                  # number of samples; the data stays sharded like the clients
    heartbeat_s: float = 0.0      # >0: ranks publish heartbeats every heartbeat_s through the process group's store and
                                  # each round fails fast (comm.failure.PeerFailure) if a peer is silent for 30x that


# ------------------------------------------------------------------------------------------------
class HipEngine:
    """AlexNet3D_Dropout on the gfx950 kernels (ABCD-shape volumes, polyphase uint8 store)."""
    sample_fields = ("x8", "mom", "labels")  # per-sample store rows (they travel with a migrating client)

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
    input_shape = (1, 121, 145, 121)   # one sample as the model sees it (FLOP counting)

    @staticmethod
    def graphs_default_for(k):
        """Captured steps for row sets of more than NIDT_AX_EAGER_MAXG clients, eager steps with the weight-gradient
        branch below ([EAGER-BRANCH], alexnet_hip.py)."""
        from .alexnet_hip import eager_branch
        return not eager_branch(k)

    accepts_cids_dev = True  # train_step(cids_dev=...): client ids from a device buffer (graph reuse across groups)

    # [PACK-FUSE] the optimizer step may write the next train step's conv2-5 forward images (runner: pack_next /
    # prepacked, also inside captured steps: the two variants are separate graphs).  NIDT_AX_PACK_FUSE=0: off (A/B)
    fused_pack = os.environ.get("NIDT_AX_PACK_FUSE", "1") != "0"
    fused_pack_graphs = fused_pack

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True,
                   cids_dev=None, prepacked=False):
        self._last_gb = (G, B)
        y = self.labels.index_select(0, idx.long())
        ct = cids_dev
        if ct is None and cids is not None:
            key = tuple(int(c) for c in cids)
            ct = self._cid_cache.get(key)
            if ct is None:  # one upload per client group, reused by every step
                ct = torch.tensor(key, dtype=torch.int32, device=self.device)
                self._cid_cache[key] = ct
        return self.net.train_step(theta, bufs, grads, self.x8, self.mom, idx, y, G, B, keep, seed, ct, seed_dev,
                                   bn_train=bn_train, prepacked=prepacked)

    def eval_logits(self, theta, bufs, idx, G, B):
        return self.net.eval_logits(theta, bufs, self.x8, idx, G, B)

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False,
                  pack_next=False):
        """Fused per-client step (``optim.hip`` ``local_opt``): masks (shared or per-row bits, weight or gradient
        mode), FedProx proximal gradient, clip(10), SGD(wd, momentum), Ditto pull — one norm pass + one update
        pass over the rows.  The clipped gradient is written back only with ``keep_grad``.  ``pack_next``: the same
        rows train again next at this step's shape, so the update also writes their conv2-5 forward images (the next
        train step then runs with ``prepacked``)."""
        gb = getattr(self, "_last_gb", None)
        if pack_next and self.fused_pack and gb is not None and gb[0] == theta.shape[0]:
            self.local_opt_pack(theta, grads, mom_buf, spec, lr, wd, momentum, max_norm,
                                self.net.fused_plan(gb[0], gb[1], theta.shape[1]), lr_dev=lr_dev, keep_grad=keep_grad)
            return
        self.m.local_opt(*self._opt_args(theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev,
                                         keep_grad), ops.stream())

    def local_opt_pack(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, plan, lr_dev=None,
                       keep_grad=False, wt=False):
        """:meth:`local_opt` that also writes the conv layers' bf16 forward images of the next step from the updated
        weights (``optim.hip`` ``local_opt_pack``; ``plan`` = :meth:`.resnet2d_hip.WeightPacker.fused_plan`).
        ``wt``: the plan is the tiled one and the step writes the data-gradient images too (``local_opt_pack_wt``)."""
        tab, nd, nconv, rest, nrest, lds, buf = plan
        fn = self.m.local_opt_pack_wt if wt else self.m.local_opt_pack
        fn(*self._opt_args(theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev, keep_grad),
           tab.data_ptr(), nd, nconv, rest.data_ptr() if nrest else 0, nrest, lds, buf.data_ptr(), ops.stream())

    def _opt_args(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev, keep_grad):
        G, P = theta.shape
        # one workspace per row group, never freed or shared: captured graphs keep its address, and the launches of
        # one step may run concurrently on side streams (runner step_streams)
        if not hasattr(self, "_optws"):
            self._optws = {}
        wkey = (theta.data_ptr(), G, P)
        ows = self._optws.get(wkey)
        if ows is None:
            ows = self._optws[wkey] = torch.empty(self.m.clip_sgd_mask_workspace(G, P), dtype=torch.float32,
                                                  device=theta.device)
        bits = spec.bits
        if spec.mask_mode:
            assert bits is not None and bits.dtype == torch.int32 and bits.stride(1) == 1
            assert spec.shared or bits.shape[0] == G
        mstride = 0 if (bits is None or spec.shared) else bits.stride(0)
        ref = spec.ref if spec.prox_mu else None
        pref = spec.pref if spec.lamda else None
        return (theta.data_ptr(), grads.data_ptr(), mom_buf.data_ptr() if mom_buf is not None else 0,
                theta.stride(0), bits.data_ptr() if (bits is not None and spec.mask_mode) else 0, mstride,
                int(spec.mask_mode), ref.data_ptr() if ref is not None else 0,
                ref.stride(0) if (ref is not None and ref.dim() == 2) else 0, float(spec.prox_mu),
                pref.data_ptr() if pref is not None else 0,
                pref.stride(0) if (pref is not None and pref.dim() == 2) else 0, float(spec.lamda),
                ows.data_ptr(), G, P, float(lr), float(wd), float(momentum), float(max_norm),
                lr_dev.data_ptr() if lr_dev is not None else 0, int(keep_grad))

    def saliency_acc(self, theta, grads, score, alpha):
        G, P = theta.shape
        self.m.saliency_acc(theta.data_ptr(), grads.data_ptr(), theta.stride(0), P, G, float(alpha),
                            score.data_ptr(), score.stride(0), ops.stream())


class TorchEngine:
    """Any ``nn.Module`` (reference-semantics eager path; CPU tests, 2D CNN families, baselines).

    ``store``: float tensor ``[N, ...]`` of inputs (already scaled); ``labels``: ``[N]``.
    ``loss``: ``"bce"`` (class_num=1, logits [B,1]) or ``"ce"`` (multi-class)."""
    sample_fields = ("store", "labels")

    def __init__(self, template_model, store, labels, device, loss="bce", dtype=torch.float32, amp=False):
        self.model = template_model.to(device)
        # amp: bf16 autocast for the forward/backward (fp32 master rows, fp32 optimizer) on MIOpen
        self.amp = bool(amp) and torch.device(device).type == "cuda"
        self.players = ParamLayout.from_tensors(list(self.model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(self.model.named_buffers()))
        self.store, self.labels, self.device, self.loss, self.dtype = store, labels, torch.device(device), loss, dtype

    @property
    def input_shape(self):
        shp = tuple(self.store.shape[1:])
        return (1,) + shp if len(shp) == 3 else shp   # volumes without a channel dim get one (see _batch)

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

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True):
        from torch.func import functional_call
        losses = torch.zeros(G, device=theta.device)
        if seed_dev is not None:
            seed = int(seed) + int(seed_dev.item())
        self.model.train(bn_train)
        if keep >= 1.0:  # dropout off (the HIP head's keep = 1), BN still in training mode
            for mod in self.model.modules():
                if isinstance(mod, torch.nn.Dropout):
                    mod.eval()
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
            if bn_train:
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

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False):
        """Reference-order torch twin of the fused ``local_opt`` kernel (one client row at a time)."""
        from .masks import unpack_bits
        if lr_dev is not None:
            lr = float(lr_dev.item())
        G, P = theta.shape
        m = None
        if spec.mask_mode:
            m = unpack_bits(spec.bits, P)
        for g in range(G):
            mg = None if m is None else (m[0] if spec.shared else m[g])
            gr = grads[g]
            if spec.mask_mode == 2:
                gr = gr * mg
            if spec.prox_mu:
                gr = gr + spec.prox_mu * (theta[g] - spec.ref)
            gn = float(gr.norm())
            coef = min(1.0, max_norm / (gn + 1e-6))
            gr = gr * coef
            if keep_grad:
                grads[g].copy_(gr)
            d = gr + wd * theta[g]
            if momentum != 0 and mom_buf is not None:
                mom_buf[g].mul_(momentum).add_(d)
                d = mom_buf[g]
            theta[g].add_(d, alpha=-lr)
            if spec.lamda:
                theta[g].sub_(lr * spec.lamda * (theta[g] - spec.pref))
            if spec.mask_mode == 1:
                theta[g].mul_(mg)

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


def __getattr__(name):  # FLRunner moved to engine/runner.py (imports it lazily: runner imports this module)
    if name in ("FLRunner", "StepSpec", "RowSet"):
        from . import runner
        return getattr(runner, name)
    raise AttributeError(name)
