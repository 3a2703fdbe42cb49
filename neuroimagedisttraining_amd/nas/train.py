"""DARTS search and genotype training drivers (reference ``darts/train_search.py:1-315``, ``darts/train.py:1-214``).

Same flags and schedule as the reference scripts (SGD momentum 0.9, cosine LR to ``learning_rate_min``,
grad-clip 5, ``train_portion`` split of the training set into weight/arch batches, genotype logged every
epoch; eval: auxiliary tower weight, linearly ramped drop-path).  Differences, MI355X-first:

* ``nn.DataParallel`` is replaced by one process per GPU (``torchrun``): each rank takes a disjoint shard of
  every global batch and gradients (weights and alphas) are averaged with ONE coalesced all-reduce per
  update over RCCL (gloo on CPU);
* ``--channels_last`` / ``--bf16`` run the convs through MIOpen NHWC with bf16 autocast;
* data: CIFAR-10 arrays from ``--data`` (``.npz``) or the synthetic CIFAR-shape set (no network here).

Usage: ``python -m neuroimagedisttraining_amd.nas.train search|eval [flags]``.
"""
from __future__ import annotations

import argparse
import logging
import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

from . import utils as U
from .architect import Architect
from .genotypes import genotype_from_string
from .network import NetworkCIFAR
from .search import Network, Network_GumbelSoftmax

log = logging.getLogger("nas")


def search_args(argv=None):
    a = argparse.ArgumentParser("darts search")
    add = a.add_argument
    add("--run_id", type=int, default=0)
    add("--data", type=str, default="")
    add("--batch_size", type=int, default=64)
    add("--learning_rate", type=float, default=0.025)
    add("--learning_rate_min", type=float, default=0.001)
    add("--momentum", type=float, default=0.9)
    add("--weight_decay", type=float, default=3e-4)
    add("--report_freq", type=float, default=50)
    add("--gpu", type=str, default="0")
    add("--epochs", type=int, default=50)
    add("--init_channels", type=int, default=16)
    add("--layers", type=int, default=8)
    add("--model_path", type=str, default="saved_models")
    add("--cutout", action="store_true", default=False)
    add("--cutout_length", type=int, default=16)
    add("--drop_path_prob", type=float, default=0.3)
    add("--save", type=str, default="EXP")
    add("--seed", type=int, default=2)
    add("--grad_clip", type=float, default=5)
    add("--train_portion", type=float, default=0.5)
    add("--unrolled", action="store_true", default=False)
    add("--arch_learning_rate", type=float, default=3e-4)
    add("--arch_weight_decay", type=float, default=1e-3)
    add("--optimization", type=str, default="DARTS", help="DARTS | DARTS_V2")
    add("--arch_search_method", type=str, default="DARTS", help="DARTS | GDAS")
    add("--lambda_train_regularizer", type=float, default=1)
    add("--lambda_valid_regularizer", type=float, default=1)
    add("--early_stopping", type=int, default=0)
    add("--group_id", type=int, default=0)
    add("--w_update_times", type=int, default=1)
    add("--tau_max", type=float, default=10.0)
    add("--tau_min", type=float, default=0.1)
    add("--n_train", type=int, default=0, help="synthetic set size (0 = CIFAR-10 size)")
    add("--max_steps", type=int, default=0, help="stop each epoch after this many steps (0 = full epoch)")
    add("--channels_last", action="store_true")
    add("--bf16", action="store_true")
    return a.parse_args(argv)


def eval_args(argv=None):
    a = argparse.ArgumentParser("darts train")
    add = a.add_argument
    add("--data", type=str, default="")
    add("--batch_size", type=int, default=96)
    add("--learning_rate", type=float, default=0.025)
    add("--learning_rate_min", type=float, default=0.001)
    add("--momentum", type=float, default=0.9)
    add("--weight_decay", type=float, default=3e-4)
    add("--report_freq", type=float, default=50)
    add("--gpu", type=str, default="0")
    add("--epochs", type=int, default=600)
    add("--init_channels", type=int, default=36)
    add("--layers", type=int, default=20)
    add("--model_path", type=str, default="saved_models")
    add("--auxiliary", action="store_true", default=False)
    add("--auxiliary_weight", type=float, default=0.4)
    add("--cutout", action="store_true", default=False)
    add("--cutout_length", type=int, default=16)
    add("--drop_path_prob", type=float, default=0.2)
    add("--save", type=str, default="EXP")
    add("--seed", type=int, default=0)
    add("--arch", type=str, default="DARTS")
    add("--grad_clip", type=float, default=5)
    add("--n_train", type=int, default=0)
    add("--max_steps", type=int, default=0)
    add("--channels_last", action="store_true")
    add("--bf16", action="store_true")
    return a.parse_args(argv)


# ------------------------------------------------------------------------------------------------
class GradSync:
    """Average gradients over ranks with one flat all-reduce (no-op for world size 1)."""

    def __init__(self, info):
        self.info = info

    def __call__(self, grads):
        if self.info.world <= 1 or not grads:
            return
        import torch.distributed as dist
        flat = torch.cat([g.reshape(-1).float() for g in grads])
        dist.all_reduce(flat)
        flat.div_(self.info.world)
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()


def _data(args, info):
    from ..data.images import _load_arrays
    n_train = args.n_train or None
    xtr, ytr, xte, yte, n_cls = _load_arrays("cifar10", args.data, n_train=n_train,
                                             n_test=max(1000, (n_train or 50000) // 5), seed=args.seed)
    mean = xtr.mean(dim=(0, 2, 3), keepdim=True)
    std = xtr.std(dim=(0, 2, 3), keepdim=True) + 1e-6
    return (xtr - mean) / std, ytr, (xte - mean) / std, yte, n_cls


def _batches(x, y, idx, bs, info, rng, shuffle=True, cutout=None):
    """Global batches of size ``bs``; each rank takes its contiguous ``bs/world`` slice."""
    idx = np.asarray(idx)
    order = rng.permutation(len(idx)) if shuffle else np.arange(len(idx))
    per = max(1, bs // info.world)
    for s in range(0, len(idx) - bs + 1 if len(idx) >= bs else 1, bs):
        sel = idx[order[s:s + bs]][info.rank * per:(info.rank + 1) * per]
        xb = x[torch.from_numpy(sel)]
        if cutout is not None:
            xb = torch.stack([cutout(im) for im in xb])
        yield xb, y[torch.from_numpy(sel)]


def _to(xb, yb, dev, cl):
    xb = xb.to(dev, non_blocking=True)
    if cl:
        xb = xb.contiguous(memory_format=torch.channels_last)
    return xb, yb.to(dev, non_blocking=True)


def _autocast(args, dev):
    return torch.autocast(dev.type, dtype=torch.bfloat16, enabled=bool(args.bf16) and dev.type == "cuda")


def _cosine(lr0, lr_min, epoch, epochs):
    return lr_min + 0.5 * (lr0 - lr_min) * (1 + math.cos(math.pi * epoch / max(1, epochs)))


def _infer(model, x, y, info, args, dev, aux_out=False):
    model.eval()
    crit = nn.CrossEntropyLoss()
    top1, objs = U.AvgrageMeter(), U.AvgrageMeter()
    rng = np.random.RandomState(0)
    with torch.no_grad():
        for xb, yb in _batches(x, y, np.arange(len(y)), args.batch_size, info, rng, shuffle=False):
            xb, yb = _to(xb, yb, dev, args.channels_last)
            with _autocast(args, dev):
                out = model(xb)
            out = (out[0] if aux_out else out).float()
            objs.update(crit(out, yb).item(), yb.numel())
            top1.update(U.accuracy(out, yb)[0].item(), yb.numel())
    return top1.avg, objs.avg


def run_search(args, info=None):
    from ..parallel import runtime as rt
    info = info or rt.init_distributed()
    dev = info.device
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    x, y, _, _, n_cls = _data(args, info)
    crit = nn.CrossEntropyLoss()
    cls = Network_GumbelSoftmax if args.arch_search_method == "GDAS" else Network
    model = cls(args.init_channels, n_cls, args.layers, crit, dev).to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    sync = GradSync(info)
    with torch.no_grad():  # identical init on every rank
        for p in model.parameters():
            if info.world > 1:
                import torch.distributed as dist
                dist.broadcast(p, 0)
    opt = torch.optim.SGD(model.weight_parameters(), args.learning_rate, momentum=args.momentum,
                          weight_decay=args.weight_decay)
    architect = Architect(model, crit, args, dev, grad_sync=sync)
    n = len(y)
    split = int(np.floor(args.train_portion * n))
    tr_idx, va_idx = np.arange(split), np.arange(split, n)
    rng = np.random.RandomState(args.seed)
    cut = U.Cutout(args.cutout_length) if args.cutout else None
    history = []
    for epoch in range(args.epochs):
        lr = _cosine(args.learning_rate, args.learning_rate_min, epoch, args.epochs)
        for g in opt.param_groups:
            g["lr"] = lr
        if isinstance(model, Network_GumbelSoftmax):
            model.set_tau(args.tau_max - (args.tau_max - args.tau_min) * epoch / max(1, args.epochs - 1))
        genotype = model.genotype()
        if info.is_main:
            log.info("epoch %d lr %e genotype = %s", epoch, lr, genotype[0])
        model.train()
        top1, objs = U.AvgrageMeter(), U.AvgrageMeter()
        va_iter = _batches(x, y, va_idx, args.batch_size, info, rng, cutout=None)
        t0 = time.perf_counter()
        for step, (xb, yb) in enumerate(_batches(x, y, tr_idx, args.batch_size, info, rng, cutout=cut)):
            if args.max_steps and step >= args.max_steps:
                break
            xb, yb = _to(xb, yb, dev, args.channels_last)
            try:
                xv, yv = next(va_iter)
            except StopIteration:
                va_iter = _batches(x, y, va_idx, args.batch_size, info, rng)
                xv, yv = next(va_iter)
            xv, yv = _to(xv, yv, dev, args.channels_last)
            if args.optimization == "DARTS":
                architect.step(xb, yb, xv, yv, lr, opt, args.unrolled)
            else:
                architect.step_v2(xb, yb, xv, yv, args.lambda_train_regularizer, args.lambda_valid_regularizer)
            for _ in range(args.w_update_times):
                opt.zero_grad(set_to_none=True)
                with _autocast(args, dev):
                    logits = model(xb)
                loss = crit(logits.float(), yb)
                loss.backward()
                sync([p.grad for p in model.weight_parameters() if p.grad is not None])
                nn.utils.clip_grad_norm_(model.weight_parameters(), args.grad_clip)
                opt.step()
            objs.update(loss.item(), yb.numel())
            top1.update(U.accuracy(logits.float(), yb)[0].item(), yb.numel())
            if info.is_main and step % int(args.report_freq) == 0:
                log.info("train %03d %e %f", step, objs.avg, top1.avg)
        va_acc, va_loss = _infer(model, x[va_idx], y[va_idx], info, args, dev)
        history.append(dict(epoch=epoch, train_acc=top1.avg, train_loss=objs.avg, valid_acc=va_acc,
                            valid_loss=va_loss, seconds=time.perf_counter() - t0))
        if info.is_main:
            log.info("epoch %d train_acc %f valid_acc %f (%.1fs)", epoch, top1.avg, va_acc, history[-1]["seconds"])
    genotype = model.genotype()
    return model, genotype, history


def run_eval(args, info=None):
    from ..parallel import runtime as rt
    info = info or rt.init_distributed()
    dev = info.device
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    x, y, xt, yt, n_cls = _data(args, info)
    genotype = genotype_from_string(args.arch)
    model = NetworkCIFAR(args.init_channels, n_cls, args.layers, args.auxiliary, genotype).to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    if info.world > 1:
        import torch.distributed as dist
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p, 0)
    log.info("param size = %fMB", U.count_parameters_in_MB(model))
    crit = nn.CrossEntropyLoss()
    opt = torch.optim.SGD(model.parameters(), args.learning_rate, momentum=args.momentum,
                          weight_decay=args.weight_decay)
    sync = GradSync(info)
    rng = np.random.RandomState(args.seed)
    cut = U.Cutout(args.cutout_length) if args.cutout else None
    history = []
    for epoch in range(args.epochs):
        lr = _cosine(args.learning_rate, args.learning_rate_min, epoch, args.epochs)
        for g in opt.param_groups:
            g["lr"] = lr
        model.drop_path_prob = args.drop_path_prob * epoch / max(1, args.epochs)
        model.train()
        top1, objs = U.AvgrageMeter(), U.AvgrageMeter()
        for step, (xb, yb) in enumerate(_batches(x, y, np.arange(len(y)), args.batch_size, info, rng, cutout=cut)):
            if args.max_steps and step >= args.max_steps:
                break
            xb, yb = _to(xb, yb, dev, args.channels_last)
            opt.zero_grad(set_to_none=True)
            with _autocast(args, dev):
                logits, aux = model(xb)
            loss = crit(logits.float(), yb)
            if args.auxiliary and aux is not None:
                loss = loss + args.auxiliary_weight * crit(aux.float(), yb)
            loss.backward()
            sync([p.grad for p in model.parameters() if p.grad is not None])
            nn.utils.clip_grad_norm_(model.parameters(), args.grad_clip)
            opt.step()
            objs.update(loss.item(), yb.numel())
            top1.update(U.accuracy(logits.float(), yb)[0].item(), yb.numel())
        te_acc, te_loss = _infer(model, xt, yt, info, args, dev, aux_out=True)
        history.append(dict(epoch=epoch, train_acc=top1.avg, train_loss=objs.avg, test_acc=te_acc, test_loss=te_loss))
        if info.is_main:
            log.info("epoch %d lr %e train_acc %f test_acc %f", epoch, lr, top1.avg, te_acc)
    return model, history


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(message)s")
    mode = argv.pop(0) if argv and argv[0] in ("search", "eval") else "search"
    if mode == "search":
        _, g, _ = run_search(search_args(argv))
        print(g[0])
    else:
        run_eval(eval_args(argv))


if __name__ == "__main__":
    main()
