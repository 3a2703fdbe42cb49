"""BASELINE config 5: 3D ResNet-50 on full-resolution 1x121x145x121 volumes, many clients, sparse update exchange.

Clients are sharded over the ranks (one process per GPU, RCCL); every client trains a 3D ResNet-50 (Bottleneck
[3,4,6,3]) on its own synthetic ABCD-shape volumes and the server update is FedAvg over top-k sparsified client
updates exchanged with a fixed-size all-gather (``FLConfig.update_topk``).  ``--engine hip`` (default): the
client-batched engine (engine/resnet3d_hip.py: ``--group`` clients per lockstep launch, every bottleneck conv and
BatchNorm on the hand-written kernels); ``--engine torch``: the generic per-client TorchEngine (bf16 autocast,
stage checkpointing; ``--no-hip-convs`` = all MIOpen), the comparison row.  Client rows (params, grads, BN buffers) stay resident in HBM:
the script reports the per-GPU peak so the 288 GB sizing can be checked (256 clients x 46 M params x 8 B of
fp32 params + grads = 94 GB on one GPU, 12 GB per GPU on 8).

Round 0 of a run is not steady state (first-shape eager steps, step-table builds, allocator growth), so
``--warmup`` rounds (default 1) are reported separately (``round0_s``) and ``steady_s_per_round`` averages the rounds
after them.  The synthetic cohort is generated and synchronised before the first round.

Usage: [torchrun --nproc-per-node N] python tools/config5_resnet3d.py --clients 256 --rounds 3
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1, help="leading rounds excluded from the steady average")
    ap.add_argument("--train-per-client", type=int, default=2)
    ap.add_argument("--test-per-client", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--topk", type=float, default=0.01)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--engine", default="hip", choices=["hip", "torch"])
    ap.add_argument("--group", type=int, default=32, help="clients per lockstep launch (hip engine)")
    ap.add_argument("--test-batch", type=int, default=None,
                    help="eval chunk (default 16 on the hip engine: a client's 9 test volumes in one grouped launch of "
                         "--group clients instead of per-client chunks; 8 on the torch engine)")
    ap.add_argument("--no-hip-convs", action="store_true",
                    help="keep every Conv3d on MIOpen (default: eligible 3x3x3 convs run on the HIP kernels)")
    args = ap.parse_args()
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner, TorchEngine
    from neuroimagedisttraining_amd.models.resnet3d import resnet3d_50
    from neuroimagedisttraining_amd.parallel import runtime as rt
    info = rt.init_distributed()
    dev = info.device
    shards = rt.shard_clients([args.train_per_client] * args.clients, info.world)
    vol, labels, local = build_fl_volumes(shards[info.rank], args.clients, args.train_per_client,
                                          args.test_per_client, dev, seed=7)
    splits = [local.get(c) or ClientSplit(np.zeros(args.train_per_client, np.int64),
                                          np.zeros(args.test_per_client, np.int64)) for c in range(args.clients)]
    n_hip = 0
    if args.engine == "hip":
        from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
        model = resnet3d_50(num_classes=1, width=args.width)
        eng = ResNet3DHipEngine(model, vol, labels, dev)
        n_hip = "all bottleneck convs + BN (client-batched)"
    else:
        model = resnet3d_50(num_classes=1, checkpoint_stages=True, width=args.width)
        if dev.type == "cuda" and not args.no_hip_convs:
            from neuroimagedisttraining_amd.ops.modules import use_hip_convs
            n_hip = use_hip_convs(model)  # 13 of the 16 bottleneck 3x3x3 convs -> nidt::conv3d_k3
        eng = TorchEngine(model, vol, labels, dev, loss="bce", amp=True)
    cfg = FLConfig(comm_round=args.rounds, epochs=args.epochs, batch_size=args.batch, lr=0.01, frac=1.0,
                   seed=7, update_topk=args.topk, frequency_of_the_test=1,
                   test_batch=args.test_batch or (16 if args.engine == "hip" else 8),
                   group=args.group if args.engine == "hip" else 0)
    runner = FLRunner(eng, splits, cfg, info, model, algorithm="fedavg")
    memlog = []
    if dev.type == "cuda":  # per-phase memory: allocated after, and the peak during, each phase of a round
        def _wrap(name):
            fn = getattr(runner, name)

            def w(*a, **k):
                torch.cuda.reset_peak_memory_stats()
                out = fn(*a, **k)
                memlog.append((name, round(torch.cuda.memory_allocated() / 2 ** 30, 1),
                               round(torch.cuda.max_memory_allocated() / 2 ** 30, 1),
                               round(torch.cuda.memory_reserved() / 2 ** 30, 1)))
                return out
            setattr(runner, name, w)
        for nm in ("local_train", "aggregate", "evaluate"):
            _wrap(nm)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    rt.barrier(info)
    t0 = time.perf_counter()
    res = None
    per_round, peaks, phases = [], [], []
    for r in range(args.rounds):
        t_before = dict(runner.timers)
        tr = time.perf_counter()
        res = runner.run_round(r, sync_timers=True)
        if dev.type == "cuda":
            torch.cuda.synchronize()
            peaks.append(max((m[2] for m in memlog[-3:]), default=0.0))
        per_round.append(rt.max_over_ranks(time.perf_counter() - tr, info))
        phases.append({k: round(v - t_before.get(k, 0.0), 3) for k, v in runner.timers.items()})
        if info.is_main:
            print("round %d: %.2f s %s" % (r, per_round[-1], phases[-1]), flush=True)  # progress
    dt = rt.max_over_ranks(time.perf_counter() - t0, info)
    peak = torch.cuda.max_memory_allocated() / 2 ** 30 if dev.type == "cuda" else 0.0
    if info.is_main:
        print(json.dumps({"config": "3D ResNet-50 full-res, sparse top-k all-gather", "engine": args.engine,
                          "group": args.group if args.engine == "hip" else None, "clients": args.clients,
                          "ranks": info.world, "params": runner.P, "rounds": args.rounds,
                          "s_per_round": round(dt / args.rounds, 2),
                          "round0_s": round(sum(per_round[:args.warmup]) / max(1, min(args.warmup, args.rounds)), 2),
                          "steady_s_per_round": (round(float(np.mean(per_round[args.warmup:])), 2)
                                                 if args.rounds > args.warmup else None),
                          "s_round_each": [round(x, 2) for x in per_round], "hip_convs": n_hip,
                          "peak_hbm_gib_rank0": round(peak, 1), "peak_gib_each_round": peaks,
                          "phase_s_each_round": phases, "mem_gib_phase_alloc_peak_reserved": memlog,
                          "update_topk": args.topk, "aggregate_elems": runner.stat_info.get("aggregate_elems"),
                          "metrics": None if res is None else dict(res)}), flush=True)
    rt.shutdown(info)


if __name__ == "__main__":
    main()
