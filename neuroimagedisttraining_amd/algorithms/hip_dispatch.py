"""The reference-compatible API classes (``SailentGradsAPI(dataset, device, args, trainer, logger).train()`` and the
other algorithms' ``*API``) on the client-batched MI355X executor.

A reference script builds its dataset tuple with the loaders (``load_partition_data_abcd``, the CIFAR /
Tiny-ImageNet loaders), a model, a ``ModelTrainer`` and then calls ``API(...).train()``
(``main_sailentgrads.py:272-280``, ``main_subavg.py:221-222``).  On a GPU with the HIP extension built, ``train()``
hands the whole run to the same ``FLRunner`` / ``make_runner`` the command-line entry points use: the tuple's
client loaders are turned into one device store plus per-client index splits —

* ABCD ``IndexLoader``s (``data/abcd.py``) already index one ``VolumeStore``: its uint8 volumes become the engine's
  polyphase store (AlexNet3D) or raw volumes (3D ResNet-50), the loaders' indices the splits;
* the image loaders' ``TensorDataset`` / ``AugmentedTensorDataset`` hold normalised float copies of each client's
  images: they are concatenated and mapped back to the uint8 pixels the image engines normalise on device
  (``round((x * std + mean) * 255)``, exact for pixels that were uint8) —

and the trainer's model is the template (its weights are the initial global model; the final global model is
loaded back into it).  ``stat_info`` gets the runner's records (same keys and reference log lines).

The eager implementation stays the oracle: ``args.engine = "torch"`` (or ``NIDT_API_ENGINE=torch``), a CPU device,
a missing extension or a model / data layout the kernels do not cover keep the sequential eager loop.
``args.engine = "hip"`` (``NIDT_API_ENGINE=hip``) makes an unsupported case an error instead.
"""
from __future__ import annotations

import argparse
import logging
import os

import numpy as np
import torch

log = logging.getLogger(__name__)

# reference API name -> harness algorithm
ALGO_OF = {"SailentGradsAPI": "sailentgrads", "FedAvgAPI": "fedavg", "FedProxAPI": "fedprox", "DisPFLAPI": "dispfl",
           "SubAvgAPI": "subavg", "DittoAPI": "ditto", "DPSGDAPI": "dpsgd", "FedFomoAPI": "fedfomo",
           "LocalAPI": "local"}


def _mode(args):
    m = os.environ.get("NIDT_API_ENGINE") or getattr(args, "engine", None) or "auto"
    return {"eager": "torch"}.get(m, m)


def _full_args(args, algo):
    """The caller's ``args`` over this package's defaults of ``algo`` (a reference script's parser lacks the
    executor's own flags: group, step streams, ...)."""
    from .. import cli
    base = cli.add_args(argparse.ArgumentParser(add_help=False), algo).parse_args([])
    merged = vars(base)
    merged.update(vars(args) if not isinstance(args, dict) else args)
    ns = argparse.Namespace(**merged)
    ns.algo = algo
    return ns


def _family(model):
    from ..models.alexnet3d import AlexNet3D_Dropout
    name = type(model).__name__.lower()
    if isinstance(model, AlexNet3D_Dropout):
        return "alexnet3d"
    if "resnet" in name and any(isinstance(m, torch.nn.Conv3d) for m in model.modules()):
        return "resnet3d"
    if "resnet" in name:
        return "resnet2d"
    return None


def _abcd_cohort(api, device):
    from ..engine.executor import ClientSplit
    trn, tst = api.train_data_local_dict, api.test_data_local_dict
    store = trn[0].store
    N = len(trn)
    splits = [ClientSplit(np.asarray(trn[c].indices, np.int64), np.asarray(tst[c].indices, np.int64))
              for c in range(N)]
    val = api.val_data_local_dict
    if val is not None:
        splits = [ClientSplit(s.train, s.test, np.asarray(val[c].indices, np.int64)) for c, s in enumerate(splits)]
    return store, splits


def _image_tensors(loader):
    ds = loader.dataset
    if hasattr(ds, "tensors"):
        return ds.tensors[0], ds.tensors[1]
    if hasattr(ds, "x") and hasattr(ds, "y"):
        return ds.x, ds.y
    raise TypeError("unsupported image loader dataset %s" % type(ds).__name__)


def _image_cohort(api, mean, std):
    """One uint8 HWC store of every client's train / test (/ val) images and the index splits into it."""
    from ..engine.executor import ClientSplit
    N = len(api.train_data_local_dict)
    xs, ys, splits, off = [], [], [], 0
    mean_t = torch.tensor(mean).view(1, -1, 1, 1)
    std_t = torch.tensor(std).view(1, -1, 1, 1)

    def take(loader):
        nonlocal off
        x, y = _image_tensors(loader)
        x = x.detach().cpu().float()
        u8 = ((x * std_t + mean_t) * 255.0).round().clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous()
        xs.append(u8)
        ys.append(torch.as_tensor(y).long().cpu())
        ix = np.arange(off, off + len(u8), dtype=np.int64)
        off += len(u8)
        return ix

    for c in range(N):
        tr = take(api.train_data_local_dict[c])
        te = take(api.test_data_local_dict[c])
        va = take(api.val_data_local_dict[c]) if api.val_data_local_dict is not None else None
        splits.append(ClientSplit(tr, te, va) if va is not None else ClientSplit(tr, te))
    return torch.cat(xs), torch.cat(ys), splits


def build_engine(api, args, info):
    """(engine, splits) for the API's dataset tuple and trainer model, or None when the kernels do not cover them."""
    from ..data.abcd import IndexLoader
    model = api.model_trainer.model
    fam = _family(model)
    first = api.train_data_local_dict[0]
    if fam in ("alexnet3d", "resnet3d") and isinstance(first, IndexLoader):
        store, splits = _abcd_cohort(api, info.device)
        vol = store.volumes
        if vol.dtype != torch.uint8 or tuple(vol.shape[1:]) != (121, 145, 121):
            return None
        if fam == "alexnet3d":
            from ..data.synthetic_fl import to_hip_store
            from ..engine.executor import HipEngine
            x8, mom = to_hip_store(vol.to(info.device))
            return HipEngine(model, x8, mom, store.labels.float().to(info.device), info.device), splits
        from ..engine.resnet3d_hip import ResNet3DHipEngine
        return ResNet3DHipEngine(model, vol.to(info.device), store.labels.float().to(info.device),
                                 info.device), splits
    if fam == "resnet2d" and not isinstance(first, IndexLoader):
        from ..data.images import NORM
        from ..engine.resnet2d_hip import ResNetHipEngine
        x0, _ = _image_tensors(first)
        side = x0.shape[-1]
        ds = args.dataset if args.dataset in NORM else ("tiny" if side == 64 else "cifar10")
        mean, std = NORM[ds]
        x8, y, splits = _image_cohort(api, mean, std)
        if tuple(x8.shape[1:]) not in ((32, 32, 3), (64, 64, 3)):
            return None
        eng = ResNetHipEngine(model, x8.to(info.device), y.to(info.device), info.device, mean=mean, std=std,
                              augment=bool(getattr(args, "augment", 1)))
        return eng, splits
    return None


def try_train_on_hip(api):
    """Runs ``api``'s whole training on the client-batched executor when possible; returns True if it did."""
    algo = ALGO_OF.get(type(api).__name__)
    mode = _mode(api.args)
    if algo is None or mode == "torch":
        return False
    dev = torch.device(api.device) if not isinstance(api.device, torch.device) else api.device
    try:
        from .. import ops
        ok = dev.type == "cuda" and torch.cuda.is_available() and ops.available()
    except Exception:  # noqa: BLE001
        ok = False
    if not ok:
        if mode == "hip":
            raise RuntimeError("engine 'hip' needs a CUDA device and the built HIP extension")
        return False
    from .. import cli
    from ..engine.personalized import make_runner
    from ..parallel import runtime as rt
    args = _full_args(api.args, algo)
    info = rt.init_distributed()
    built = build_engine(api, args, info)
    if built is None:
        if mode == "hip":
            raise RuntimeError("engine 'hip': no client-batched kernels for %s on this dataset"
                               % type(api.model_trainer.model).__name__)
        api.logger.warning("%s: no client-batched kernels for %s on this data; running the eager loop",
                           type(api).__name__, type(api.model_trainer.model).__name__)
        return False
    eng, splits = built
    cfg = cli.fl_config(args, algo)
    model = api.model_trainer.model
    runner = make_runner(algo, eng, splits, cfg, info, model, logger=api.logger)
    api.logger.info("%s: %d clients on the client-batched MI355X executor (%s)", type(api).__name__, len(splits),
                    type(eng).__name__)
    if runner.alg == "salientgrads":
        runner.generate_global_mask_snip()
    for r in range(cfg.comm_round):
        runner.run_round(r)
    runner.finish()
    api.stat_info.update(dict(runner.stat_info))
    with torch.no_grad():  # the final global model back into the caller's trainer
        sd = dict(eng.players.unflatten(runner.w_global))
        sd.update(eng.blayers.unflatten(runner.b_global))
        model.load_state_dict({k: v.to(next(model.parameters()).device) for k, v in sd.items()}, strict=False)
    api.engine_used = "hip"
    api.runner = runner
    return True
