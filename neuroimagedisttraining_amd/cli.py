"""Standalone experiment entry points (reference ``fedml_experiments/standalone/<algo>/main_<algo>.py``).

Flags, defaults and the ``args.identity`` string (the log file name, ``LOG/<dataset>/<identity>.log``) follow
the reference entry points.  Added flags:

* ``--engine {auto,hip,torch}``: every algorithm (SalientGrads, FedAvg, FedProx, DisPFL, SubAvg, Ditto, D-PSGD,
  FedFomo, Local) runs on the client-batched MI355X executor (HIP kernels, clients sharded over ranks, RCCL
  collectives) when ``hip`` (``auto`` = hip if a GPU and the extension are available) for 3DCNN (AlexNet3D) and
  3D ResNet-50 (``--model resnet3d_50``) on ABCD-shape volumes and ResNet-18-GN (``--model resnet18``) on
  CIFAR-10/100 — the reference defaults of every entry point;
  ``torch`` = the reference-semantics sequential eager path (also the CPU path).
* ``--synthetic_abcd 1``, ``--n_per_client``: synthetic ABCD-shape cohort (no HDF5 needed); ``--synthetic_abcd 0
  --data_dir <cohort.nidtvol | dir>`` trains on the real cohort (site clients) on either path;
  ``--synthetic_size N``: N synthetic train images (N/5 test) for CIFAR/Tiny without data files.
* FedProx / robust aggregation: ``--fedprox_mu``, ``--aggregator {fedavg,krum,multikrum,median,trimmed_mean}``,
  ``--byzantine_f``, ``--trim_ratio``.
* ``--checkpoint_dir`` / ``--checkpoint_every`` / ``--keep_last`` / ``--resume`` for the HIP executor (background-written,
  indexed, world-size independent checkpoints: ``utils/checkpoint.py``).

Run under ``torchrun`` for multi-GPU; single process otherwise.
"""
from __future__ import annotations

import argparse
import logging
import os
import random

import numpy as np
import torch

ALGOS = ("sailentgrads", "fedavg", "fedprox", "dispfl", "subavg", "ditto", "dpsgd", "fedfomo", "local")

_DEFAULTS = {  # per-entry-point defaults that differ
    "sailentgrads": dict(model="3DCNN", dataset="ABCD", batch_size=16, lr=0.01, epochs=2, client_num_in_total=4,
                         frac=1.0, comm_round=200, seed=1024, cs="v0"),
    "fedavg": dict(model="3DCNN", dataset="ABCD", batch_size=16, lr=0.001, epochs=5, client_num_in_total=4,
                   frac=0.9, comm_round=200, seed=0),
    "fedprox": dict(model="3DCNN", dataset="ABCD", batch_size=16, lr=0.001, epochs=5, client_num_in_total=128,
                    frac=1.0, comm_round=200, seed=0, partition_method="dir", fedprox_mu=0.01),
    "dispfl": dict(model="3DCNN", dataset="ABCD", batch_size=16, lr=0.001, epochs=5, client_num_in_total=21,
                   frac=0.1, comm_round=10, seed=1024, cs="random"),
    "subavg": dict(model="resnet18", dataset="cifar10", batch_size=128, lr=0.1, epochs=5, client_num_in_total=100,
                   frac=0.1, comm_round=1000, seed=0),
    "ditto": dict(model="resnet18", dataset="cifar10", batch_size=128, lr=0.1, epochs=2, client_num_in_total=100,
                  frac=0.1, comm_round=1000, seed=0),
    "dpsgd": dict(model="resnet18", dataset="cifar10", batch_size=128, lr=0.1, epochs=5, client_num_in_total=100,
                  frac=0.1, comm_round=50, seed=0, cs="ring"),
    "fedfomo": dict(model="resnet18", dataset="cifar10", batch_size=128, lr=0.1, epochs=5, client_num_in_total=100,
                    frac=0.1, comm_round=1000, seed=0),
    "local": dict(model="resnet18", dataset="cifar10", batch_size=128, lr=0.1, epochs=5, client_num_in_total=100,
                  frac=1.0, comm_round=10, seed=1024),
}


def str2bool(v):
    return str(v).lower() in ("1", "true", "yes", "y")


def add_args(parser, algo):
    d = _DEFAULTS[algo]
    a = parser.add_argument
    a("--model", type=str, default=d["model"])
    a("--dataset", type=str, default=d["dataset"])
    a("--data_dir", type=str, default="")
    # Tiny-ImageNet: reproduce the reference loader's reshape(-1, 3, 64, 64) pixel scramble (PARITY.md §2.5)
    a("--tiny_ref_pixel_order", type=int, default=0)
    a("--partition_method", type=str, default=d.get("partition_method", "dir"))
    a("--partition_alpha", type=float, default=0.3)
    a("--batch_size", type=int, default=d["batch_size"])
    a("--client_optimizer", type=str, default="sgd")
    a("--lr", type=float, default=d["lr"])
    a("--lr_decay", type=float, default=0.998)
    a("--wd", type=float, default=5e-4)
    a("--momentum", type=float, default=0)
    a("--epochs", type=int, default=d["epochs"])
    a("--client_num_in_total", type=int, default=d["client_num_in_total"])
    a("--frac", type=float, default=d["frac"])
    a("--comm_round", type=int, default=d["comm_round"])
    a("--frequency_of_the_test", type=int, default=1)
    a("--gpu", type=int, default=0)
    a("--ci", type=int, default=0)
    a("--seed", type=int, default=d["seed"])
    a("--tag", type=str, default="test")
    if algo in ("sailentgrads", "dispfl"):
        a("--dense_ratio", type=float, default=0.5)
        a("--anneal_factor", type=float, default=0.5)
        a("--cs", type=str, default=d["cs"])
        a("--active", type=float, default=1.0)
        a("--public_portion", type=float, default=0)
        a("--erk_power_scale", type=float, default=1)
        for f in ("dis_gradient_check", "strict_avg", "static", "uniform", "save_masks", "different_initial",
                  "record_mask_diff", "diff_spa", "global_test"):
            a("--" + f, action="store_true")
        a("--dispfl_aggregate", type=int, default=0)
    if algo == "sailentgrads":
        a("--itersnip_iteration", type=int, default=1)
        a("--stratified_sampling", action="store_true")
        a("--snip_mask", type=str2bool, default=True)  # reference: type=bool (cannot be disabled, Q6)
        a("--logfile", type=str, default="logfile")
    if algo == "subavg":
        a("--dense_ratio", type=float, default=0.5)
        a("--each_prune_ratio", type=float, default=0.05)
        a("--dist_thresh", type=float, default=1e-4)
        a("--acc_thresh", type=float, default=0.5)
        a("--record_mask_diff", action="store_true")
    if algo == "ditto":
        a("--local_epochs", type=int, default=3)
        a("--lamda", type=float, default=0.5)
    if algo == "dpsgd":
        a("--cs", type=str, default=d["cs"])
        a("--type", type=str, default="epoch")
    # additions (not in the reference)
    a("--engine", type=str, default="auto", choices=["auto", "hip", "torch"])
    a("--synthetic_abcd", type=int, default=1)
    a("--n_per_client", type=int, default=180)
    a("--synthetic_size", type=int, default=0)
    a("--rebalance", type=int, default=0)  # 1: (HIP, multi-rank, frac < 1) move sampled clients + samples to even the load
    a("--heartbeat_s", type=float, default=0.0)  # >0: multi-rank failure detection (comm/failure.py)
    a("--augment", type=int, default=1)  # image datasets: the reference's train-time RandomCrop(pad 4) + flip
    a("--fedprox_mu", type=float, default=d.get("fedprox_mu", 0.0))
    a("--aggregator", type=str, default="fedavg")
    a("--byzantine_f", type=int, default=0)
    a("--trim_ratio", type=float, default=0.1)
    a("--update_topk", type=float, default=0.0, help="send only the top-k fraction of each client's update")
    a("--group", type=int, default=0)
    a("--checkpoint_dir", type=str, default="")
    a("--checkpoint_every", type=int, default=1,
      help="save every N rounds (and after the last round); saves are written in the background and become the "
           "resume point once written, so a crash loses at most N rounds plus the rounds one save takes to write")
    a("--keep_last", type=int, default=2, help="complete checkpoint rounds kept on disk (0 = all)")
    a("--resume", type=int, default=0)
    a("--log_dir", type=str, default="LOG")
    a("--results_dir", type=str, default=os.environ.get("NIDT_RESULTS_DIR", "results"),
      help="record_information target: <results_dir>/<dataset>/<identity>.json (+ .npz for large arrays); "
           "default $NIDT_RESULTS_DIR or ./results")
    return parser


def identity(args, algo):
    part = args.partition_method + ("" if args.partition_method == "homo" else str(args.partition_alpha))
    args.client_num_per_round = int(args.client_num_in_total * args.frac)
    if algo == "sailentgrads":
        s = "SailentGrads-" + args.dataset + "-" + part + "-mdl" + args.model + "customized" + "lowbatch" + "-cs" + args.cs
        s += "-masks" if args.save_masks else ""
        s += "-diff_spa" if args.diff_spa else ""
        s += "-uniform_init" if args.uniform else "-ERK_init"
        s += "-diff_init" if args.different_initial else "-same_init"
        s += "-g" if args.global_test else ""
        s += "-RSM" if args.static else "-DST"
        s += "-cm%s-total_clnt%s" % (args.comm_round, args.client_num_in_total)
        s += "-neighbor%s-dr%s-active%s-seed%s-lr%s-batchsize%s-iteration%s-stratified%s" % (
            args.client_num_per_round, args.dense_ratio, args.active, args.seed, args.lr, args.batch_size,
            args.itersnip_iteration, args.stratified_sampling)
        return s
    if algo in ("fedavg", "fedprox"):
        s = ("fedavg" if algo == "fedavg" else "fedprox") + "-" + part + "-mdl" + args.model
        s += "-batchsize%s-cm%s-total_clnt%s-neighbor%s-seed%s-lr%s" % (
            args.batch_size, args.comm_round, args.client_num_in_total, args.client_num_per_round, args.seed, args.lr)
        return s + ("-mu%s-agg%s" % (args.fedprox_mu, args.aggregator) if algo == "fedprox" else "")
    if algo == "dispfl":  # main_dispfl.py:203-238
        s = "DisPFL-" + args.dataset + "-" + part + "-mdl" + args.model + "-cs" + args.cs
        s += "-masks" if args.save_masks else ""
        s += "-diff_spa" if args.diff_spa else ""
        s += "-uniform_init" if args.uniform else "-ERK_init"
        s += "-diff_init" if args.different_initial else "-same_init"
        s += "-g" if args.global_test else ""
        s += "-RSM" if args.static else "-DST"
        s += "-cm%s-total_clnt%s-neighbor%s-dr%s-batchsize%s-active%s-lr%s-seed%s" % (
            args.comm_round, args.client_num_in_total, args.client_num_per_round, args.dense_ratio, args.batch_size,
            args.active, args.lr, args.seed)
        return s
    if algo == "subavg":  # main_subavg.py:177-186 (no "-" between the name and the partition)
        return "SubAVG%s-mdl%s-batchsize%s-cm%s-total_clnt%s-neighbor%s-seed%s-dr%s" % (
            part, args.model, args.batch_size, args.comm_round, args.client_num_in_total, args.client_num_per_round,
            args.seed, args.dense_ratio)
    if algo == "ditto":  # main_ditto.py:165-174
        return "ditto-%s-mdl%s-ge%s-le%s-batchsize%s-lambda%s-cm%s-total_clnt%s-neighbor%s-seed%s" % (
            part, args.model, args.epochs, args.local_epochs, args.batch_size, args.lamda, args.comm_round,
            args.client_num_in_total, args.client_num_per_round, args.seed)
    if algo == "dpsgd":  # main_dpsgd.py:167-175
        return "dpsgd-%s-%s-mdl%s-cs%s-batchsize%s-cm%s-total_clnt%s-neighbor%s-seed%s-type%s" % (
            args.dataset, part, args.model, args.cs, args.batch_size, args.comm_round, args.client_num_in_total,
            args.client_num_per_round, args.seed, args.type)
    if algo == "fedfomo":  # main_fedfomo.py:170-176
        return "fedfomo-%s-mdl%s-cm%s-total_clnt%s-batchsize%s-neighbor%s-seed%s" % (
            part, args.model, args.comm_round, args.client_num_in_total, args.batch_size, args.client_num_per_round,
            args.seed)
    if algo == "local":  # main_local.py:163-168
        return "local-%s-cm%s-total_clnt%s-neighbor%s-seed%s" % (
            part, args.comm_round, args.client_num_in_total, args.client_num_per_round, args.seed)
    raise ValueError(algo)


def load_data(args, dataset_name, logger=None):
    from .data import abcd, images
    if dataset_name == "ABCD":
        if args.synthetic_abcd or not args.data_dir:
            return abcd.load_partition_data_abcd_synthetic(args.client_num_in_total, args.partition_method,
                                                           args.partition_alpha, args.batch_size,
                                                           n_per_client=args.n_per_client, seed=args.seed,
                                                           logger=logger)
        return abcd.load_partition_data_abcd(args.data_dir, args.partition_method, args.partition_alpha,
                                             args.client_num_in_total, args.batch_size, logger)
    if dataset_name in ("cifar10", "cifar100", "tiny"):
        n = getattr(args, "synthetic_size", 0) or None
        return images.load_partition_data(dataset_name, args.data_dir, args.partition_method, args.partition_alpha,
                                          args.client_num_in_total, args.batch_size, logger, seed=args.seed,
                                          with_val=getattr(args, "algo", "") == "fedfomo", n_train=n,
                                          n_test=n // 5 if n else None, augment=bool(getattr(args, "augment", 1)),
                                          ref_pixel_order=bool(getattr(args, "tiny_ref_pixel_order", 0)))
    if dataset_name == "synthetic":
        return images.load_partition_data_synthetic_tabular(args.client_num_in_total, args.batch_size)
    raise ValueError(dataset_name)


RESNET3D_NAMES = ("resnet3d_50", "3dresnet50")
IMAGE_DATASETS = ("cifar10", "cifar100", "tiny")
# the other image models of the reference entry points (main_subavg.py:143-158): client-batched via vmap
ZOO2D_NAMES = ("lenet5", "cnn_cifar10", "cnn_cifar100", "vgg11", "vgg16")


def hip_family(args):
    """Model family of the client-batched MI355X executor for these flags, or None (eager only):
    ``alexnet3d`` (3DCNN on ABCD: engine/executor.HipEngine), ``resnet2d`` (resnet18 = ResNet-18-GN on 32x32
    CIFAR-10/100 or 64x64 Tiny-ImageNet — ``customized_resnet18`` / ``tiny_resnet18``: engine/resnet2d_hip),
    ``resnet3d`` (3D ResNet-50 on ABCD: engine/resnet3d_hip), ``batched2d`` (lenet5 / cnn_cifar10 / cnn_cifar100 /
    vgg11 / vgg16 on CIFAR: engine/batched2d, clients vmapped into grouped library calls + the fused optimizer)."""
    model = args.model.lower()
    if args.dataset == "ABCD" and model in ("3dcnn", "alexnet3d", "alexnet3d_dropout"):
        # the AlexNet3D kernels are built for the ABCD volume (1x121x145x121: polyphase 61x73x61 store, conv1's
        # compile-time tiling); a cohort file of another shape runs on the eager engine (loudly, see _use_hip)
        shape = _cohort_shape(args)
        return "alexnet3d" if shape in (None, ABCD_SHAPE) else None
    if args.dataset in IMAGE_DATASETS and model == "resnet18":
        return "resnet2d"
    if args.dataset in ("cifar10", "cifar100") and model in ZOO2D_NAMES:
        return "batched2d"
    if args.dataset == "ABCD" and model in RESNET3D_NAMES:
        return "resnet3d"
    return None


ABCD_SHAPE = (121, 145, 121)


def _cohort_shape(args):
    """Volume shape of the ``--data_dir`` cohort file (None: synthetic ABCD-shape data or no readable file)."""
    if getattr(args, "synthetic_abcd", True) or not getattr(args, "data_dir", None):
        return None
    try:
        from .data.volume_file import VolumeFile
        return tuple(VolumeFile(_resolve_cohort(args.data_dir)).shape)
    except Exception:  # noqa: BLE001 - unreadable here: the loader reports it
        return None


def _use_hip(args, algo):
    """Every algorithm of the harness runs on the client-batched MI355X executor for the model families of
    :func:`hip_family` (the reference defaults of every entry point: 3DCNN + ABCD, resnet18 + cifar10)."""
    if hip_family(args) is None:
        shape = _cohort_shape(args) if args.dataset == "ABCD" else None
        why = ("the cohort's volumes are %s, the AlexNet3D kernels need %s" % (shape, ABCD_SHAPE)
               if shape not in (None, ABCD_SHAPE) else
               "--engine hip supports --model 3DCNN / %s --dataset ABCD, --model resnet18 --dataset %s and "
               "--model %s --dataset cifar10 / cifar100"
               % (" / ".join(RESNET3D_NAMES), " / ".join(IMAGE_DATASETS), " / ".join(ZOO2D_NAMES)))
        if args.engine == "hip":
            raise RuntimeError(why + "; use --engine torch")
        logging.getLogger(__name__).warning("running on the eager PyTorch engine: %s", why)
        return False
    if args.engine == "torch":
        return False
    try:
        from . import ops
        ok = torch.cuda.is_available() and ops.available()
    except Exception:  # noqa: BLE001
        ok = False
    if args.engine == "hip" and not ok:
        raise RuntimeError("--engine hip needs a GPU and the built HIP extension")
    return ok


def _resolve_cohort(data_dir):
    """NIDTVOL1 cohort file for ``--data_dir`` (a ``.nidtvol`` file or a directory holding
    ``alldatain8bitsnormalized.nidtvol``); raises instead of silently substituting synthetic data."""
    path = data_dir
    if os.path.isdir(path):
        path = os.path.join(path, "alldatain8bitsnormalized.nidtvol")
    if not os.path.exists(path) or not str(path).endswith(".nidtvol"):
        raise FileNotFoundError(
            "--synthetic_abcd 0 needs a NIDTVOL1 cohort (got --data_dir %r); convert the reference HDF5 once with "
            "`python -m neuroimagedisttraining_amd.data.volume_file convert alldatain8bitsnormalized.h5 "
            "alldatain8bitsnormalized.nidtvol`" % data_dir)
    return path


def hip_cohort(args, info, logger=None, with_val=False, raw=False):
    """(x8, mom, labels, splits) for the HIP engine: this rank's clients' subjects resident in HBM in the engine's
    polyphase layout (``raw``: plain uint8 ``[N, D, H, W]`` volumes, ``mom`` None — the 3D ResNet engine),
    ``splits[c]`` indexing that local store (non-local clients keep only their sizes).

    * real cohort (``--synthetic_abcd 0``): the reference ABCD loader's site-as-client split (21 sites, seeded
      80/20, ``ABCD/data_loader.py:67-102,157-212``) read from a NIDTVOL1 file by the native reader and streamed
      into HBM (gather / H2D / polyphase overlapped, ``data/volume_file.py``);
    * synthetic cohort (default): ``--n_per_client`` ABCD-shape volumes per client with a Dirichlet label prior.
    ``with_val``: 10 % of client 0's train size moved from every client's train split into a validation split
    (``cifar10/data_val_loader.py:275-278``; FedFomo)."""
    from .core import partition as PT
    from .data.synthetic_fl import build_fl_volumes, to_hip_store
    from .engine.executor import ClientSplit
    from .parallel import runtime as rt
    N = args.client_num_in_total
    if not args.synthetic_abcd:
        from .data.volume_file import VolumeFile, stream_to_device
        vf = VolumeFile(_resolve_cohort(args.data_dir))
        train, test, _ = PT.partition_by_site(vf.sites, max_clients=21)
        if len(train) != N:
            (logger or logging.getLogger(__name__)).info(
                "ABCD site split gives %d clients (--client_num_in_total %d ignored, quirk Q9)", len(train), N)
            N = args.client_num_in_total = len(train)
            args.client_num_per_round = int(N * args.frac)
        tr = [np.asarray(train[c]) for c in range(N)]
        te = [np.asarray(test[c]) for c in range(N)]
        shards = rt.shard_clients([len(t) for t in tr], info.world)
        mine = shards[info.rank]  # rebalancing moves a client's samples with it: the store is never replicated
        subj = np.concatenate([np.concatenate([tr[c], te[c]]) for c in mine]) if mine else np.zeros(0, np.int64)
        if raw:
            x8, mom = stream_to_device(vf, subj, info.device), None
        else:
            x8, mom = stream_to_device(vf, subj, info.device, hip_store=True)
        labels = torch.from_numpy(vf.labels[subj].astype(np.float32)).to(info.device)
        local, off = {}, 0
        for c in mine:
            local[c] = ClientSplit(np.arange(off, off + len(tr[c])), np.arange(off + len(tr[c]),
                                                                              off + len(tr[c]) + len(te[c])))
            off += len(tr[c]) + len(te[c])
        sizes = [(len(tr[c]), len(te[c])) for c in range(N)]
    else:
        n_test = max(1, int(round(args.n_per_client * 0.2)))
        n_train = args.n_per_client - n_test
        shards = rt.shard_clients([n_train] * N, info.world)
        mine = shards[info.rank]
        vol, labels, local = build_fl_volumes(mine, N, n_train, n_test, info.device, seed=args.seed,
                                              alpha=args.partition_alpha)
        if raw:
            x8, mom = vol, None
        else:
            x8, mom = to_hip_store(vol)
        del vol
        sizes = [(n_train, n_test)] * N
    nval = None
    if with_val:
        nval = int(0.1 * sizes[0][0])
        for c, sp in local.items():
            local[c] = ClientSplit(sp.train[nval:], sp.test, sp.train[:nval])
        sizes = [(a - nval, b) for a, b in sizes]
    splits = [local.get(c) or ClientSplit(np.zeros(sizes[c][0], np.int64), np.zeros(sizes[c][1], np.int64),
                                          None if nval is None else np.zeros(nval, np.int64))
              for c in range(N)]
    return x8, mom, labels, splits


def fl_config(args, algo):
    """FLConfig from the reference flags of any entry point."""
    from .engine.executor import FLConfig
    g = lambda k, d=None: getattr(args, k, d)  # noqa: E731
    return FLConfig(comm_round=args.comm_round, epochs=args.epochs, batch_size=args.batch_size, lr=args.lr,
                    lr_decay=args.lr_decay, wd=args.wd, momentum=args.momentum, frac=args.frac,
                    dense_ratio=g("dense_ratio", 1.0), itersnip_iteration=g("itersnip_iteration", 1),
                    snip_mask=g("snip_mask", True), frequency_of_the_test=args.frequency_of_the_test, seed=args.seed,
                    prox_mu=args.fedprox_mu if algo == "fedprox" else 0.0, group=args.group,
                    aggregator=args.aggregator, byzantine_f=args.byzantine_f, trim_ratio=args.trim_ratio,
                    update_topk=args.update_topk, heartbeat_s=args.heartbeat_s,
                    rebalance=bool(g("rebalance", 0)),
                    stratified_sampling=bool(g("stratified_sampling", False)),
                    cs=g("cs", "ring") if algo == "dpsgd" else "random", lamda=g("lamda", 0.5),
                    local_epochs=g("local_epochs", 0) or 0, anneal_factor=g("anneal_factor", 0.5),
                    active=g("active", 1.0), static=bool(g("static", False)),
                    dis_gradient_check=bool(g("dis_gradient_check", False)), uniform=bool(g("uniform", False)),
                    different_initial=bool(g("different_initial", False)), diff_spa=bool(g("diff_spa", False)),
                    erk_power_scale=g("erk_power_scale", 1.0), save_masks=bool(g("save_masks", False)),
                    dispfl_aggregate=bool(g("dispfl_aggregate", 0)), each_prune_ratio=g("each_prune_ratio", 0.05),
                    dist_thresh=g("dist_thresh", 1e-4), acc_thresh=g("acc_thresh", 0.5))


def image_cohort(args, info, with_val=False):
    """(x8, labels, splits, n_cls) for the client-batched ResNet-18-GN engine: the CIFAR-10/100 (32x32) or
    Tiny-ImageNet (64x64) train and test images as uint8 ``[N, S, S, 3]`` in one device store (train first, test at
    ``+n_train``), split exactly as the eager loaders do (``data/images.load_partition_data``: same partitioner, same
    RandomState stream, per-client test sets drawn from the train label histogram, FedFomo's 10 % validation split).

    Pixels: uint8 HWC images (the reference's dataset directories, ``data/image_files.py``, or a uint8 ``.npz``) are
    used as is (the engine applies the dataset's mean/std normalisation on device, as the eager loaders do on the
    host, ``images.NORM``); float images (the synthetic loader's, or a float ``.npz``) are taken to be normalised
    NCHW tensors and mapped back to uint8 pixels."""
    from .core import partition as PT
    from .data import images
    from .engine.executor import ClientSplit
    MEAN, STD = images.NORM[args.dataset]
    n = getattr(args, "synthetic_size", 0) or None
    xtr, ytr, xte, yte, n_cls = images.load_raw(args.dataset, args.data_dir, n, n // 5 if n else None, args.seed,
                                                 bool(getattr(args, "tiny_ref_pixel_order", 0)))

    def to_u8(x):
        if x.dtype == torch.uint8:
            return x
        mean = torch.tensor(MEAN).view(1, 3, 1, 1)
        std = torch.tensor(STD).view(1, 3, 1, 1)
        return ((x * std + mean) * 255.0).round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous()

    xtr, xte = to_u8(xtr), to_u8(xte)
    side = 64 if args.dataset == "tiny" else 32
    assert tuple(xtr.shape[1:]) == (side, side, 3), xtr.shape
    N = args.client_num_in_total
    rng = np.random.RandomState(args.seed)
    train_map = images.partition_data(ytr.numpy(), args.partition_method, N, args.partition_alpha, n_cls, rng)
    test_map = PT.per_client_test_indices(ytr.numpy(), yte.numpy(), train_map, n_cls=n_cls, rng=rng)
    ntr = len(ytr)
    splits = []
    nval = int(0.1 * len(train_map[0])) if with_val else 0
    for c in range(N):
        tr = np.asarray(train_map[c], dtype=np.int64)
        te = np.asarray(test_map[c], dtype=np.int64) + ntr
        if with_val:
            pick = rng.choice(len(tr), min(nval, len(tr)), replace=False)
            splits.append(ClientSplit(train=np.delete(tr, pick), test=te, val=tr[pick]))
        else:
            splits.append(ClientSplit(train=tr, test=te))
    x8 = torch.cat([xtr, xte]).to(info.device)
    y = torch.cat([ytr, yte]).long().to(info.device)
    return x8, y, splits, n_cls


def build_hip_engine(args, algo, info, logger=None):
    """(engine, template model, client splits) of the client-batched executor for this model family."""
    fam = hip_family(args)
    if fam == "resnet2d":
        from .data.images import NORM
        from .engine.resnet2d_hip import ResNetHipEngine
        from .models import customized_resnet18, tiny_resnet18
        x8, y, splits, n_cls = image_cohort(args, info, with_val=algo == "fedfomo")
        # main_subavg.py:149-152: resnet18 is tiny_resnet18 on Tiny-ImageNet (AdaptiveAvgPool2d), else
        # customized_resnet18 — same parameters, the engine pools the whole final map in both
        model = (tiny_resnet18 if args.dataset == "tiny" else customized_resnet18)(class_num=n_cls)
        desc = "%s %s images (%d clients)" % ("synthetic" if not args.data_dir else args.data_dir, args.dataset,
                                              len(splits))
        mean, std = NORM[args.dataset]
        eng = ResNetHipEngine(model, x8, y, info.device, mean=mean, std=std, augment=bool(getattr(args, "augment", 1)))
        return eng, model, splits, desc
    if fam == "batched2d":
        from .data.images import NORM
        from .engine.batched2d import BatchedModuleEngine
        from .models import create_model
        x8, y, splits, n_cls = image_cohort(args, info, with_val=algo == "fedfomo")
        model = create_model(args.model, dataset=args.dataset, class_num=n_cls)
        desc = "%s %s images (%d clients), %s vmapped over clients" % (
            "synthetic" if not args.data_dir else args.data_dir, args.dataset, len(splits), args.model)
        mean, std = NORM[args.dataset]
        eng = BatchedModuleEngine(model, x8, y, info.device, mean, std, augment=bool(getattr(args, "augment", 1)))
        return eng, model, splits, desc
    if fam == "resnet3d":
        from .engine.resnet3d_hip import ResNet3DHipEngine
        from .models.resnet3d import resnet3d_50
        x8, _, labels, splits = hip_cohort(args, info, logger, with_val=algo == "fedfomo", raw=True)
        model = resnet3d_50(num_classes=1)
        desc = "NIDTVOL1 %s" % _resolve_cohort(args.data_dir) if not args.synthetic_abcd else "synthetic ABCD-shape"
        return ResNet3DHipEngine(model, x8, labels, info.device), model, splits, desc
    from .engine.executor import HipEngine
    from .models.alexnet3d import AlexNet3D_Dropout
    x8, mom, labels, splits = hip_cohort(args, info, logger, with_val=algo == "fedfomo")
    model = AlexNet3D_Dropout(num_classes=1)
    desc = "NIDTVOL1 %s" % _resolve_cohort(args.data_dir) if not args.synthetic_abcd else "synthetic ABCD-shape"
    return HipEngine(model, x8, mom, labels, info.device), model, splits, desc


def run_hip(args, algo, logger):
    """Any algorithm of the harness on the client-batched MI355X executor (HIP kernels, clients sharded over
    ranks, RCCL collectives) for the model families of :func:`hip_family`."""
    from .engine.personalized import make_runner
    from .parallel import runtime as rt
    from .utils import checkpoint as ck
    info = rt.init_distributed()
    eng, model, splits, desc = build_hip_engine(args, algo, info, logger)
    logger.info("HIP cohort (%s): %s, %d clients, train sizes %s" % (
        hip_family(args), desc, len(splits), [len(s.train) for s in splits]))
    cfg = fl_config(args, algo)
    runner = make_runner(algo, eng, splits, cfg, info, model, logger=logger)
    start = 0
    if args.resume and args.checkpoint_dir and ck.latest_round(args.checkpoint_dir) is not None:
        start = ck.load_runner(runner, args.checkpoint_dir)
        logger.info("resumed from %s at round %d", args.checkpoint_dir, start)
    elif runner.alg == "salientgrads":
        runner.generate_global_mask_snip()
    saver = (ck.Checkpointer(args.checkpoint_dir, info, every=args.checkpoint_every, keep_last=args.keep_last)
             if args.checkpoint_dir else None)
    for r in range(start, cfg.comm_round):
        runner.run_round(r)
        if saver is not None:
            saver.maybe_save(runner, r + 1, last=r + 1 == cfg.comm_round)
    if saver is not None:
        saver.close()
    runner.finish()
    if info.is_main:
        _record(args, algo, runner.stat_info, logger)
    rt.shutdown(info)
    return runner.stat_info


# algorithms whose reference API persists stat_info at the end (subavg_api.py:92, fedfomo_api.py:118, local_api.py:84)
RECORDED = ("subavg", "fedfomo", "local")


def _record(args, algo, stat_info, logger):
    """``record_information`` without pickle (JSON + npz), into a directory that is created (quirk Q13)."""
    if algo not in RECORDED:
        return None
    from .utils.records import record_information
    path = record_information(stat_info, args.results_dir, args.dataset, args.identity)
    logger.info("stat_info recorded to %s", path)
    return path


def run_reference(args, algo, logger, device):
    from .algorithms import personalized as PZ
    from .algorithms.fedavg import FedAvgAPI, FedProxAPI
    from .algorithms.salientgrads import SailentGradsAPI
    from .algorithms.trainers import ClassificationTrainer, VolumeTrainer
    from .models import create_model
    ds_name = "ABCD" if algo == "sailentgrads" else args.dataset
    dataset = load_data(args, ds_name, logger)
    class_num = 1 if ds_name == "ABCD" else dataset[8 if len(dataset) > 8 else 7]
    in_shape = None
    model = create_model(args.model, ds_name, class_num, in_shape=in_shape).to(device)
    trainer = (VolumeTrainer if ds_name == "ABCD" else ClassificationTrainer)(model, args, logger)
    cls = {"sailentgrads": SailentGradsAPI, "fedavg": FedAvgAPI, "fedprox": FedProxAPI, "dispfl": PZ.DisPFLAPI,
           "subavg": PZ.SubAvgAPI, "ditto": PZ.DittoAPI, "dpsgd": PZ.DPSGDAPI, "fedfomo": PZ.FedFomoAPI,
           "local": PZ.LocalAPI}[algo]
    api = cls(dataset, device, args, trainer, logger)
    api.train()
    _record(args, algo, api.stat_info, logger)
    return api.stat_info


def main(algo, argv=None):
    from .utils.logger import logger_config
    parser = add_args(argparse.ArgumentParser(description="%s (neuroimagedisttraining_amd)" % algo), algo)
    args = parser.parse_args(argv)
    args.algo = algo
    args.identity = identity(args, algo)
    log_path = os.path.join(args.log_dir, args.dataset, args.identity + ".log")
    logger = logger_config(log_path=log_path, logging_name=args.identity)
    logger.info(args)
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(args.seed)
    if _use_hip(args, algo):
        return run_hip(args, algo, logger)
    device = torch.device("cuda:%d" % args.gpu if torch.cuda.is_available() else "cpu")
    logger.info(device)
    return run_reference(args, algo, logger, device)
