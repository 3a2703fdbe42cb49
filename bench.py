"""Headline benchmark: FL rounds/sec (whole node), 64-client SalientGrads AlexNet3D on ABCD-shape synthetic volumes.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``, one rank per GPU over RCCL.  For N>1 it
runs either under ``torch.distributed.run`` (the ranks come from RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*, and
``--gpus`` must equal WORLD_SIZE) or directly: with ``--gpus N > 1`` and no WORLD_SIZE in the environment the
parent process spawns the N ranks itself (torchrun-style env, 127.0.0.1 rendezvous) BEFORE anything touches the
GPU, forwards rank 0's JSON line and exits with the first failing rank's code.  One *step* = one full federated round of the
reference's SalientGrads (``fedml_experiments/standalone/sailentgrads/main_sailentgrads.py`` defaults):
all 64 clients (frac=1) train 2 local epochs of batch 16 over their 144-sample train split with
SGD(lr 0.01 * 0.998^round, wd 5e-4) + clip_grad_norm(10) + global SNIP mask (dense_ratio 0.5), then
sample-weighted FedAvg of all params + BN buffers (one RCCL all-reduce), then evaluation of the global model
and every client's personal model on its 36-sample test split (frequency_of_the_test = 1).
The 64 clients are sharded over the N GPUs (strong scaling: total work per round is fixed as N grows).
The SNIP mask phase runs once before the warmup rounds (as in the reference, it is not per round).

``--algorithm`` selects any other algorithm of the harness on the same executor (fedavg / fedprox [+ robust
``--aggregator``], dispfl, subavg, ditto, dpsgd, fedfomo, local) and ``--size-skew A`` gives the clients
Dirichlet(A) sizes with the same total sample count (ragged federations).

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

# Measured on MI355X (1 GPU) with tools/eager_baseline.py: PyTorch-ROCm eager, reference semantics
# (sequential clients, one shared nn.Module, per-step mask multiply), same 64-client config.  See BASELINE.md.
EAGER_BASELINE_ROUNDS_PER_S = 0.04611       # fp32 (the reference's precision), profiles/r1_eager_baseline_steady.txt
EAGER_BF16_BASELINE_ROUNDS_PER_S = 0.0640   # same eager path under bf16 autocast (equal-precision comparison)
ALGOS = ["salientgrads", "fedavg", "fedprox", "dispfl", "subavg", "ditto", "dpsgd", "fedfomo", "local"]
NAMES = {"salientgrads": "SalientGrads", "fedavg": "FedAvg", "fedprox": "FedProx", "dispfl": "DisPFL",
         "subavg": "SubAvg", "ditto": "Ditto", "dpsgd": "D-PSGD", "fedfomo": "FedFomo", "local": "Local"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = ranks (default: WORLD_SIZE under torchrun, else 1); N>1 without torchrun self-launches")
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
    ap.add_argument("--frac", type=float, default=1.0)
    ap.add_argument("--size-skew", type=float, default=0.0, help="Dirichlet alpha of per-client sizes (0 = equal)")
    ap.add_argument("--no-eval", action="store_true", help="(diagnostic only) skip per-round evaluation")
    ap.add_argument("--algorithm", default="salientgrads", choices=ALGOS)
    ap.add_argument("--aggregator", default="fedavg", choices=["fedavg", "krum", "multikrum", "median", "trimmed_mean"])
    ap.add_argument("--prox-mu", type=float, default=0.01)
    ap.add_argument("--cs", default="ring", help="D-PSGD topology")
    ap.add_argument("--phase-timers", action="store_true", help="synchronised per-phase timers (adds syncs)")
    ap.add_argument("--dump-rows", default="", help="after the run, save this rank's client rows (each client's "
                    "last locally trained params, i.e. the rows before the last aggregation) to <prefix>.rank<r>.pt "
                    "(sharding-parity checks: tools/compare_rows.py)")
    ap.add_argument("--step-streams", type=int, default=4,
                    help="side streams for the extra (ragged) launches of one lockstep step (1 = serial)")
    ap.add_argument("--rebalance", type=int, default=0,
                    help="1: move sampled clients (state and samples) between ranks to even the per-round load "
                         "(off by default: no measurement has shown a net gain, profiles/r2_s2_rehearse_2ranks.txt)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: launcher/plumbing diagnostic only -- a tiny 3-D CNN on 15^3 volumes on the CPU twin "
                         "engine with gloo collectives (NOT the headline config)")
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n, argv):
    """Spawn ``n`` ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, one per GPU).

    Called before any GPU call in this process (it makes none: the device-count check runs in each rank); the
    children inherit stdout, so rank 0's JSON line is the only line printed.  When a rank fails the others are
    terminated (they would otherwise wait in a collective until its timeout).  Returns the exit code."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / cross-process tensors)
        # stdout: rank 0's through a pipe (its JSON line is re-emitted on our stdout, anything else the libraries print
        # there goes to stderr); the other ranks print nothing on stdout
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True, bufsize=1))

    def forward(pipe):
        for line in pipe:
            out = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            out.write(line)
            out.flush()

    import threading
    fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fwd.start()
    rc = 0
    try:
        live = list(procs)
        while live:
            time.sleep(0.2)
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in live:
                        q.send_signal(signal.SIGTERM)
    finally:
        deadline = time.time() + 30
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
        fwd.join(timeout=10)
    return rc


def _cpu_tiny_setup(args, info):
    """``--device cpu``: the same runner on the CPU twin engine (a small 3-D CNN, 15^3 uint8 volumes), so the
    launcher and the gloo collectives can be checked without a GPU."""
    import numpy as np
    from torch import nn
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, TorchEngine

    class Tiny3D(nn.Module):
        def __init__(self):
            super().__init__()
            self.features = nn.Sequential(nn.Conv3d(1, 4, 3, 2), nn.BatchNorm3d(4), nn.ReLU(inplace=True),
                                          nn.Conv3d(4, 8, 3), nn.BatchNorm3d(8), nn.ReLU(inplace=True))
            self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(8, 1))

        def forward(self, x):
            return self.classifier(self.features(x).amax((2, 3, 4)))

    per = args.train_per_client + args.test_per_client
    g = torch.Generator().manual_seed(args.seed)
    N = args.clients * per
    vols = torch.randint(0, 256, (N, 15, 15, 15), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, 2, (N,), generator=g).float()
    splits = [ClientSplit(np.arange(c * per, c * per + args.train_per_client),
                          np.arange(c * per + args.train_per_client, (c + 1) * per)) for c in range(args.clients)]
    torch.manual_seed(args.seed)
    model = Tiny3D()
    return model, TorchEngine(model, vols, labels, "cpu"), splits, [args.train_per_client] * args.clients


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(world_env) if world_env else 1
    if args.gpus > 1 and world_env is None:
        # no HIP call in the launcher (children must be spawned by a process that never touched the GPU): each rank
        # checks the visible device count itself and exits non-zero, which stops the others
        sys.exit(self_launch(args.gpus, argv))
    run(args)


def run(args):
    import numpy as np
    from neuroimagedisttraining_amd.parallel import runtime as rt
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, HipEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes, skewed_sizes, to_hip_store
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout

    # NIDT_DIST_BACKEND=gloo rehearses the multi-rank layout with every rank on the one visible GPU (not a scaling run)
    if (args.device == "cuda" and args.gpus > 1 and torch.cuda.device_count() < args.gpus
            and os.environ.get("NIDT_DIST_BACKEND") != "gloo"):
        raise SystemExit("bench.py: --gpus %d but only %d GPU(s) visible" % (args.gpus, torch.cuda.device_count()))
    info = rt.init_distributed(prefer_gpu=args.device == "cuda")
    if info.world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d ranks" % (args.gpus, info.world))
    cuda = args.device == "cuda"
    if cuda:
        assert info.device.type == "cuda", "bench.py needs a GPU (--device cpu: CPU plumbing diagnostic)"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    torch.manual_seed(args.seed)
    rebalance = bool(args.rebalance)
    t0 = time.perf_counter()
    if cuda:
        per = args.train_per_client + args.test_per_client
        tot = skewed_sizes(args.clients, per, args.size_skew, seed=args.seed)
        n_test = [max(1, int(round(t * args.test_per_client / per))) for t in tot]
        n_train = [t - e for t, e in zip(tot, n_test)]
        shards = rt.shard_clients(n_train, info.world)
        local = shards[info.rank]  # data is sharded like the clients (rebalancing moves a client's samples with it)
        vol, labels, splits_local = build_fl_volumes(local, args.clients, n_train, n_test, info.device,
                                                     seed=args.seed)
        x8, mom = to_hip_store(vol)
        del vol
        nval = None
        if args.algorithm == "fedfomo":  # validation split: 10 % of client 0's train size (data_val_loader.py:275)
            nval = int(0.1 * n_train[0])
            splits_local = {c: ClientSplit(s.train[nval:], s.test, s.train[:nval]) for c, s in splits_local.items()}
            n_train = [n - nval for n in n_train]
        # splits indexed by global client id; non-local clients only need their sizes (sampling weights)
        splits = [splits_local[c] if c in splits_local else
                  ClientSplit(train=np.zeros(n_train[c], dtype=np.int64), test=np.zeros(n_test[c], dtype=np.int64),
                              val=None if nval is None else np.zeros(nval, dtype=np.int64))
                  for c in range(args.clients)]
        model = AlexNet3D_Dropout(num_classes=1)
        engine = HipEngine(model, x8, mom, labels, info.device)
    else:
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // info.world))  # ranks share the host's cores
        model, engine, splits, n_train = _cpu_tiny_setup(args, info)
    sync()
    t_data = time.perf_counter() - t0
    cfg = FLConfig(comm_round=args.warmup + args.steps, epochs=args.epochs, batch_size=args.batch,
                   dense_ratio=args.dense_ratio, seed=args.seed, group=args.group, frac=args.frac,
                   frequency_of_the_test=0 if args.no_eval else 1, aggregator=args.aggregator,
                   prox_mu=args.prox_mu if args.algorithm == "fedprox" else 0.0, cs=args.cs, final_round=False,
                   rebalance=rebalance, step_streams=args.step_streams,
                   hip_graphs=None if cuda else False)  # None: the engine's per-launch-size default
    runner = make_runner(args.algorithm, engine, splits, cfg, info, model, logger=None)
    t0 = time.perf_counter()
    if runner.alg == "salientgrads":
        runner.generate_global_mask_snip()
    sync()
    t_snip = time.perf_counter() - t0
    for r in range(args.warmup):
        runner.run_round(r)
    sync()
    rt.barrier(info)
    sync()
    for k in runner.timers:
        runner.timers[k] = 0.0
    runner.record_train_events, runner.train_events = True, []
    t0 = time.perf_counter()
    res = None
    for r in range(args.warmup, args.warmup + args.steps):
        res = runner.run_round(r, sync_timers=args.phase_timers)
    if hasattr(runner, "_flush_metrics"):
        runner._flush_metrics()   # the last round's deferred evaluation metrics land on the host inside the timing
    sync()
    t_local = time.perf_counter() - t0   # this rank's own work (before waiting for the slowest rank)
    rt.barrier(info)
    sync()
    dt = time.perf_counter() - t0
    per_rank = rt.all_gather_cat(torch.tensor([t_local], dtype=torch.float64, device=info.device), info)
    per_rank = [round(float(x), 4) for x in per_rank.cpu()]
    # GPU time each rank spent in local training (CUDA events, no syncs in the timed loop): the load balance
    t_train = sum(a.elapsed_time(b) for a, b in runner.train_events) / 1000.0
    per_rank_train = rt.all_gather_cat(torch.tensor([t_train], dtype=torch.float64, device=info.device), info)
    per_rank_train = [round(float(x), 4) for x in per_rank_train.cpu()]
    dt = rt.max_over_ranks(dt, info)
    # caching-allocator peak of any rank (every engine buffer, incl. one scratch set per distinct (G, B) launch shape)
    peak_gib = rt.max_over_ranks(torch.cuda.max_memory_allocated(info.device) / 2 ** 30 if cuda else 0.0,
                                info)
    ms = dt * 1000.0 / max(1, args.steps)
    value = args.steps / dt
    headline = (cuda and args.algorithm == "salientgrads" and args.clients == 64 and args.aggregator == "fedavg"
                and args.size_skew == 0 and args.frac == 1.0)
    if info.is_main:
        out = {
            "metric": ("FL rounds/sec (whole node), 64-client SalientGrads 3D-CNN on ABCD-shape synth" if headline else
                       "FL rounds/sec (whole node), %d-client %s%s 3D-CNN on ABCD-shape synth%s"
                       % (args.clients, NAMES[args.algorithm],
                          "" if args.aggregator == "fedavg" else "+" + args.aggregator,
                          "" if args.size_skew == 0 else " (size skew %.2f)" % args.size_skew)
                       + ("" if cuda else " [CPU plumbing diagnostic: tiny 3-D CNN, 15^3 volumes]")),
            "value": round(value, 4),
            "unit": "rounds/s",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "strong",
            # equal-precision ratio (the reference publishes no number): vs the reference-semantics eager path under bf16
            # autocast; the fp32-eager ratio mixes precisions and is reported separately, labelled as such
            "vs_baseline": (round(value / EAGER_BF16_BASELINE_ROUNDS_PER_S, 2) if headline else None),
            "vs_bf16_eager": (round(value / EAGER_BF16_BASELINE_ROUNDS_PER_S, 2) if headline else None),
            "vs_fp32_eager_cross_precision": (round(value / EAGER_BASELINE_ROUNDS_PER_S, 2) if headline else None),
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic",
            "config": {"model": "AlexNet3D_Dropout" if cuda else "Tiny3D (CPU diagnostic)", "algorithm": NAMES[args.algorithm],
                       "aggregator": args.aggregator, "clients": args.clients, "frac": args.frac,
                       "global_batch": args.batch * args.clients, "batch_per_client": args.batch,
                       "seq_len": None, "input": "1x121x145x121" if cuda else "1x15x15x15", "epochs": args.epochs,
                       "train_per_client": args.train_per_client, "test_per_client": args.test_per_client,
                       "size_skew": args.size_skew, "samples_train_total": int(sum(n_train)),
                       "dense_ratio": args.dense_ratio, "eval_every_round": not args.no_eval,
                       "rebalance": rebalance,
                       "parallelism": "clients-sharded-dp%d" % info.world},
            "setup_s": {"data": round(t_data, 2), "snip_mask": round(t_snip, 2)},
            "rank_wall_s": per_rank,
            "rank_train_gpu_s": per_rank_train,
            "rank_imbalance": (round(max(per_rank_train) / (sum(per_rank_train) / len(per_rank_train)), 3)
                               if per_rank_train and sum(per_rank_train) > 0 else None),
            "peak_hbm_gib": round(peak_gib, 2),
            "last_round_metrics": None if res is None else dict(res),
        }
        if args.phase_timers:
            out["phase_s"] = {k: round(v, 3) for k, v in runner.timers.items()}
        print(json.dumps(out), flush=True)
    if args.dump_rows:
        rows, loc = runner._local_rows(range(args.clients))
        dump = {int(c): runner.theta[r, :runner.P].detach().cpu() for r, c in zip(rows, loc)}
        if getattr(runner, "mask", None) is not None:
            dump[-1] = runner.mask.detach().float().cpu()  # the global SNIP mask the rows trained under
        torch.save(dump, "%s.rank%d.pt" % (args.dump_rows, info.rank))
    rt.shutdown(info)


if __name__ == "__main__":
    main()
