"""Rounds/s of the reference's only timed configs: ResNet-18-GN on CIFAR-10, 100 clients, on the client-batched
HIP engine (engine/resnet2d_hip.py: hand-written grouped conv kernels, lockstep clients, hipGraph steps).

Reference jobs (1x V100): SubAvg ``subavg/subavgsparsitywithoutiteration70sps.sh`` (finished 500 rounds inside
72 h -> >= 0.0019 rounds/s, ``subavg/error3437295.err``) and DisPFL ``DisPFL/dispflsparsitywithoutiteration70sps.sh``
(did not finish 500 rounds in the 2-3 day limit -> < 0.0029 rounds/s, ``DisPFL/error3469448.err``): resnet18,
cifar10, dir 0.3, batch 16, lr 0.1, lr_decay 0.998, 5 local epochs, dense_ratio 0.3, 100 clients, frac 0.1.

Data: CIFAR-10-shape synthetic uint8 images (50,000 train / 10,000 test, weak class signal) — or with ``--dataset
tiny`` Tiny-ImageNet-shape 64x64 images (100,000 / 10,000, 200 classes; ``tiny_resnet18``, the reference's
``fedml_experiments/standalone/*/tiny.sh`` presets use batch 128) — partitioned with the reference's ``dir``
partitioner (alpha 0.3) and per-client test sets drawn from the train label histogram; random-init weights.  The
reference's train-time RandomCrop(pad 4) + RandomHorizontalFlip run fused into the engine's input stage (on device,
per step / client / sample draws); ``--no-augment`` turns them off.
Usage: ``python tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

V100_BOUNDS = {"subavg": (">=", 0.0019, "subavg/error3437295.err:2-12"),
               "dispfl": ("<", 0.0029, "DisPFL/error3469448.err:3")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algorithm", default="subavg")
    ap.add_argument("--clients", type=int, default=100)
    ap.add_argument("--frac", type=float, default=0.1)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--dense-ratio", type=float, default=0.3)
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=2022)
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--dataset", default="cifar10", choices=["cifar10", "tiny"])
    ap.add_argument("--no-augment", action="store_true")
    ap.add_argument("--graphs", default="default", choices=["default", "on", "off"],
                    help="captured hipGraph local steps (FLConfig.hip_graphs; default = the engine's choice)")
    args = ap.parse_args()
    tiny = args.dataset == "tiny"
    if tiny and args.n_train == 50000:
        args.n_train = 100000

    from neuroimagedisttraining_amd.core import partition as Pt
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
    from neuroimagedisttraining_amd.models import customized_resnet18, tiny_resnet18
    from neuroimagedisttraining_amd.parallel import runtime as rt

    info = rt.init_distributed(prefer_gpu=True)
    torch.manual_seed(args.seed)
    t0 = time.perf_counter()
    n_cls = 200 if tiny else 10
    if tiny:  # 64x64 Tiny-ImageNet-shape images with a weak class signal (same generator rule as synthetic_cifar)
        g = np.random.default_rng(args.seed)
        lab = g.integers(0, n_cls, size=args.n_train + args.n_test)
        proto = g.integers(0, 256, size=(n_cls, 64, 64, 3)).astype(np.float32)
        x8 = torch.empty(len(lab), 64, 64, 3, dtype=torch.uint8)
        for s0 in range(0, len(lab), 10000):
            sl = slice(s0, s0 + 10000)
            base = g.integers(0, 256, size=(len(lab[sl]), 64, 64, 3)).astype(np.float32)
            x8[sl] = torch.from_numpy(np.clip(0.7 * base + 0.3 * proto[lab[sl]], 0, 255).astype(np.uint8))
        y = torch.from_numpy(lab.astype(np.int64))
    else:
        x8, y = synthetic_cifar(args.n_train + args.n_test, seed=args.seed)
    ytr, yte = y[:args.n_train].numpy(), y[args.n_train:].numpy()
    rng = np.random.RandomState(args.seed)
    train_map = Pt.partition_labels("dir", ytr, args.clients, 0.3, n_cls=n_cls, rng=rng)
    test_map = Pt.per_client_test_indices(ytr, yte, train_map, n_cls=n_cls, rng=rng)
    splits = []
    for c in range(args.clients):
        tr = np.asarray(train_map[c], dtype=np.int64)
        te = np.asarray(test_map[c], dtype=np.int64) + args.n_train
        if args.algorithm == "fedfomo":  # 10 % validation split (data_val_loader.py)
            nv = int(0.1 * len(tr))
            splits.append(ClientSplit(train=tr[nv:], test=te, val=tr[:nv]))
        else:
            splits.append(ClientSplit(train=tr, test=te))
    model = (tiny_resnet18 if tiny else customized_resnet18)(class_num=n_cls)
    engine = ResNetHipEngine(model, x8, y, info.device, augment=not args.no_augment)
    cfg = FLConfig(comm_round=args.warmup + args.rounds, epochs=args.epochs, batch_size=args.batch, lr=args.lr,
                   lr_decay=0.998, dense_ratio=args.dense_ratio, seed=args.seed, frac=args.frac,
                   frequency_of_the_test=0 if args.no_eval else 1, final_round=False,
                   hip_graphs={"default": None, "on": True, "off": False}[args.graphs])
    runner = make_runner(args.algorithm, engine, splits, cfg, info, model, logger=None)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    if runner.alg == "salientgrads":
        runner.generate_global_mask_snip()
    walls = []
    for r in range(args.warmup):
        t1 = time.perf_counter()
        runner.run_round(r)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t1)
        print("warmup round %d: %.2f s" % (r, walls[-1]), flush=True)
    if os.environ.get("NIDT_CIFAR_EVAL_PROBE") in ("1", "exit") and hasattr(runner, "_eval_buffers"):
        # diagnostics: time the per-round personal evaluation of every client alone (SubAvg's eval block)
        from neuroimagedisttraining_amd.engine import masks as MK
        from neuroimagedisttraining_amd.engine.personalized import RowSet
        for rep in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            th, bu = runner._eval_buffers(max(1, runner.C))
            th.copy_(runner.w_global.expand_as(th))
            bu.copy_(runner.b_global.expand_as(bu))
            th[:runner.C, :runner.P].mul_(MK.unpack_bits(runner.mbits[:runner.C], runner.P))
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            r = runner.eval_local(RowSet(th, bu), *runner.all_rows())
            torch.cuda.synchronize()
            print("eval probe %d: prepare %.1f ms, eval_local %.1f ms (%d clients, %d test samples)"
                  % (rep, (t2 - t1) * 1e3, (time.perf_counter() - t2) * 1e3, runner.C,
                     int(sum(len(sp.test) for sp in splits))), flush=True)
        if os.environ.get("NIDT_CIFAR_EVAL_PROBE") == "exit":
            return
    rt.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    each = []
    for r in range(args.warmup, args.warmup + args.rounds):
        t1 = time.perf_counter()
        res = runner.run_round(r)
        torch.cuda.synchronize()
        each.append(time.perf_counter() - t1)
        print("round %d: %.2f s" % (r, each[-1]), flush=True)
    rt.barrier(info)
    torch.cuda.synchronize()
    dt = rt.max_over_ranks(time.perf_counter() - t0, info)
    value = args.rounds / dt
    bound = V100_BOUNDS.get(args.algorithm)
    if info.is_main:
        print(json.dumps({
            "metric": "FL rounds/sec, %d-client %s ResNet-18-GN on %s-shape synth" % (
                args.clients, args.algorithm, "Tiny-ImageNet" if tiny else "CIFAR-10"),
            "value": round(value, 4), "unit": "rounds/s", "n_gpus": info.world, "rounds": args.rounds,
            "warmup": args.warmup, "s_per_round": round(dt / args.rounds, 3), "dtype": "bf16",
            "data": "synthetic", "setup_s": round(t_setup, 1), "warmup_round_s": [round(w, 2) for w in walls],
            "s_round_each": [round(w, 3) for w in each], "graph_stats": dict(getattr(runner, "graph_stats", {})),
            "phase_s_total": {k: round(v, 3) for k, v in runner.timers.items()},
            "reference_v100": ({"bound": bound[0] + str(bound[1]), "source": bound[2],
                                "vs_bound": round(value / bound[1], 1)} if (bound and not tiny) else None),
            "config": {"model": "resnet18 (GroupNorm32)", "clients": args.clients, "frac": args.frac,
                       "epochs": args.epochs, "batch": args.batch, "lr": args.lr, "dense_ratio": args.dense_ratio,
                       "partition": "dir 0.3", "train_images": args.n_train, "eval_every_round": not args.no_eval,
                       "dataset": args.dataset, "augment": not args.no_augment},
            "last_round_metrics": None if res is None else dict(res)}), flush=True)
    rt.shutdown(info)


if __name__ == "__main__":
    main()
