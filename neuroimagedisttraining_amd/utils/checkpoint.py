"""FL checkpoint / resume (absent in the reference).

A checkpoint holds the global model, every local client's personal row, BN buffers, the SalientGrads mask,
the next round index and the stat_info history.  Each rank writes its own shard (``rank{r}.pt``) of client
rows plus rank 0 the global state; files are written atomically (tmp + rename) and loaded with
``torch.load(weights_only=True)`` (no unpickling of arbitrary objects).
"""
from __future__ import annotations

import json
import os

import torch


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_runner(runner, directory, next_round):
    os.makedirs(directory, exist_ok=True)
    r = runner.info.rank
    shard = {"theta": runner.theta.detach().cpu().contiguous(), "bufs": runner.bufs.detach().cpu().contiguous(),
             "local": torch.tensor(runner.local, dtype=torch.int64)}
    _atomic_save(shard, os.path.join(directory, "rank%d.pt" % r))
    if runner.info.is_main:
        glob = {"w_global": runner.w_global.detach().cpu(), "b_global": runner.b_global.detach().cpu(),
                "mask": None if runner.mask is None else runner.mask.detach().cpu(),
                "next_round": torch.tensor(next_round)}
        _atomic_save(glob, os.path.join(directory, "global.pt"))
        with open(os.path.join(directory, "stat_info.json.tmp"), "w") as f:
            json.dump({k: v for k, v in runner.stat_info.items() if isinstance(v, (list, int, float))}, f)
        os.replace(os.path.join(directory, "stat_info.json.tmp"), os.path.join(directory, "stat_info.json"))


def load_runner(runner, directory):
    """Restore a runner in place; returns the round index to resume from."""
    glob = torch.load(os.path.join(directory, "global.pt"), map_location="cpu", weights_only=True)
    shard = torch.load(os.path.join(directory, "rank%d.pt" % runner.info.rank), map_location="cpu",
                       weights_only=True)
    if shard["local"].tolist() != list(runner.local):
        raise ValueError("checkpoint client shard does not match this rank's clients")
    runner.w_global.copy_(glob["w_global"].to(runner.device))
    runner.b_global.copy_(glob["b_global"].to(runner.device))
    if glob["mask"] is not None:
        runner.set_mask(glob["mask"].to(runner.device))
    runner.theta.copy_(shard["theta"].to(runner.device))
    runner.bufs.copy_(shard["bufs"].to(runner.device))
    p = os.path.join(directory, "stat_info.json")
    if os.path.exists(p):
        with open(p) as f:
            runner.stat_info.update(json.load(f))
    return int(glob["next_round"])


def save_state_dict(sd, path):
    _atomic_save({k: v.detach().cpu() for k, v in sd.items()}, path)


def load_state_dict(path):
    return torch.load(path, map_location="cpu", weights_only=True)
