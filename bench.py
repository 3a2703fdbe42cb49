"""Headline benchmark: FL rounds/sec (whole node), 64-client SalientGrads AlexNet3D on ABCD-shape synthetic volumes.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched with
``torch.distributed.run`` (one rank per GPU, RCCL).  One *step* = one full federated round of the
reference's SalientGrads (``fedml_experiments/standalone/sailentgrads/main_sailentgrads.py`` defaults):
all 64 clients (frac=1) train 2 local epochs of batch 16 over their 144-sample train split with
SGD(lr 0.01 * 0.998^round, wd 5e-4) + clip_grad_norm(10) + global SNIP mask (dense_ratio 0.5), then
sample-weighted FedAvg of all params + BN buffers (one RCCL all-reduce), then evaluation of the global model
and every client's personal model on its 36-sample test split (frequency_of_the_test = 1).
The 64 clients are sharded over the N GPUs (strong scaling: total work per round is fixed as N grows).
The SNIP mask phase runs once before the warmup rounds (as in the reference, it is not per round).

Data: synthetic ABCD-shape (1x121x145x121 uint8) volumes with a non-IID (Dirichlet 0.3) label prior per
client, generated on device; random-init AlexNet3D_Dropout weights.  Compute: bf16 MFMA with fp32 accumulate,
fp32 master weights / optimizer / BN statistics.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Measured on MI355X (1 GPU) with tools/eager_baseline.py: PyTorch-ROCm eager fp32, reference semantics
# (sequential clients, one shared nn.Module, per-step mask multiply), same 64-client config.  See BASELINE.md.
EAGER_BASELINE_ROUNDS_PER_S = 0.04611  # fp32, steady-state (rounds 1-2), profiles/r1_eager_baseline_steady.txt


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--train-per-client", type=int, default=144)
    ap.add_argument("--test-per-client", type=int, default=36)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--group", type=int, default=0, help="max clients per lockstep launch (0 = all local)")
    ap.add_argument("--dense-ratio", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=1024)
    ap.add_argument("--no-eval", action="store_true", help="(diagnostic only) skip per-round evaluation")
    ap.add_argument("--algorithm", default="salientgrads", choices=["salientgrads", "fedavg", "fedprox"],
                    help="other BASELINE configs: fedavg (config 2: --clients 8), fedprox + --aggregator (config 4)")
    ap.add_argument("--aggregator", default="fedavg", choices=["fedavg", "krum", "multikrum", "median", "trimmed_mean"])
    ap.add_argument("--prox-mu", type=float, default=0.01)
    ap.add_argument("--phase-timers", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    from neuroimagedisttraining_amd.parallel import runtime as rt
    from neuroimagedisttraining_amd.engine.executor import FLConfig, FLRunner, HipEngine
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes, to_hip_store
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout

    info = rt.init_distributed(prefer_gpu=True)
    assert info.device.type == "cuda", "bench.py needs a GPU"
    torch.manual_seed(args.seed)
    shards = rt.shard_clients([args.train_per_client] * args.clients, info.world)
    local = shards[info.rank]
    t0 = time.perf_counter()
    vol, labels, splits_local = build_fl_volumes(local, args.clients, args.train_per_client, args.test_per_client,
                                                 info.device, seed=args.seed)
    x8, mom = to_hip_store(vol)
    del vol
    torch.cuda.synchronize()
    t_data = time.perf_counter() - t0

    # splits indexed by global client id; non-local clients only need their sizes (sampling weights)
    import numpy as np
    from neuroimagedisttraining_amd.engine.executor import ClientSplit
    splits = []
    for c in range(args.clients):
        if c in splits_local:
            splits.append(splits_local[c])
        else:
            splits.append(ClientSplit(train=np.zeros(args.train_per_client, dtype=np.int64),
                                      test=np.zeros(args.test_per_client, dtype=np.int64)))
    model = AlexNet3D_Dropout(num_classes=1)
    engine = HipEngine(model, x8, mom, labels, info.device)
    cfg = FLConfig(comm_round=args.warmup + args.steps, epochs=args.epochs, batch_size=args.batch,
                   dense_ratio=args.dense_ratio, seed=args.seed, group=args.group,
                   frequency_of_the_test=0 if args.no_eval else 1, aggregator=args.aggregator,
                   prox_mu=args.prox_mu if args.algorithm == "fedprox" else 0.0)
    alg = "salientgrads" if args.algorithm == "salientgrads" else "fedavg"
    runner = FLRunner(engine, splits, cfg, info, model, logger=None, algorithm=alg)
    t0 = time.perf_counter()
    if alg == "salientgrads":
        runner.generate_global_mask_snip()
    torch.cuda.synchronize()
    t_snip = time.perf_counter() - t0
    for r in range(args.warmup):
        runner.run_round(r)
    torch.cuda.synchronize()
    rt.barrier(info)
    torch.cuda.synchronize()
    for k in runner.timers:
        runner.timers[k] = 0.0
    t0 = time.perf_counter()
    res = None
    for r in range(args.warmup, args.warmup + args.steps):
        res = runner.run_round(r, sync_timers=args.phase_timers)
    torch.cuda.synchronize()
    rt.barrier(info)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = rt.max_over_ranks(dt, info)
    ms = dt * 1000.0 / max(1, args.steps)
    value = args.steps / dt
    headline = args.algorithm == "salientgrads" and args.clients == 64 and args.aggregator == "fedavg"
    if info.is_main:
        out = {
            "metric": ("FL rounds/sec (whole node), 64-client SalientGrads 3D-CNN on ABCD-shape synth" if headline else
                       "FL rounds/sec (whole node), %d-client %s%s 3D-CNN on ABCD-shape synth"
                       % (args.clients, args.algorithm, "" if args.aggregator == "fedavg" else "+" + args.aggregator)),
            "value": round(value, 4),
            "unit": "rounds/s",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (round(value / EAGER_BASELINE_ROUNDS_PER_S, 2)
                            if EAGER_BASELINE_ROUNDS_PER_S and headline else None),
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": "AlexNet3D_Dropout", "algorithm": {"salientgrads": "SalientGrads", "fedavg": "FedAvg",
                                                                  "fedprox": "FedProx"}[args.algorithm],
                       "aggregator": args.aggregator, "clients": args.clients,
                       "global_batch": args.batch * args.clients, "batch_per_client": args.batch,
                       "seq_len": None, "input": "1x121x145x121", "epochs": args.epochs,
                       "train_per_client": args.train_per_client, "test_per_client": args.test_per_client,
                       "dense_ratio": args.dense_ratio, "eval_every_round": not args.no_eval,
                       "parallelism": "clients-sharded-dp%d" % info.world},
            "setup_s": {"data": round(t_data, 2), "snip_mask": round(t_snip, 2)},
            "phase_s": {k: round(v, 3) for k, v in runner.timers.items()},
            "last_round_metrics": res,
        }
        print(json.dumps(out), flush=True)
    rt.shutdown(info)


if __name__ == "__main__":
    main()
