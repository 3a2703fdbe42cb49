"""FL checkpoint / resume (absent in the reference): world-size independent and crash consistent.

Layout of ``<dir>``::

    round_<R>/clients_rank<r>.pt   per-client state of the clients rank r held, keyed by global client id
    round_<R>/global.pt            w_global, b_global, SalientGrads mask, runner state (RNG streams, affinities)
    round_<R>/stat_info.json
    latest                         text file "<R>" — written last (atomic rename) after a barrier

A round directory only becomes visible through ``latest`` once every rank has written its shard, so a crash
mid-save leaves the previous checkpoint intact.  Per-client rows are keyed by client id, so a run checkpointed
on 4 ranks resumes on 2 (or 1, or 8): each rank loads the rows of the clients it now owns from whichever shard
holds them.  Everything is loaded with ``torch.load(weights_only=True)`` — no unpickling of arbitrary objects.
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import torch

from ..parallel import runtime as rt


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _client_state(runner):
    """{client id: {name: tensor}} of this rank's clients (rows of every per-client matrix the runner keeps)."""
    out = {}
    mats = {"theta": runner.theta, "bufs": runner.bufs}
    if getattr(runner, "mbits", None) is not None:
        mats["mbits"] = runner.mbits
    if getattr(runner, "shared_bits", None) is not None:
        mats["shared_bits"] = runner.shared_bits
    if hasattr(runner, "pers"):
        mats["pers_theta"] = runner.pers.theta
        mats["pers_bufs"] = runner.pers.bufs
    for c in runner.local:
        i = runner.row_of[c]
        out[int(c)] = {k: (m[i, :runner.P] if k in ("theta", "pers_theta") else
                           m[i, :runner.Q] if k in ("bufs", "pers_bufs") else m[i]).detach().cpu().clone()
                       for k, m in mats.items()}
    return out


def _runner_state(runner):
    st = {}
    if hasattr(runner, "np_rng"):
        kind, keys, pos, has_gauss, cached = runner.np_rng.get_state()
        st["np_rng_keys"] = torch.from_numpy(keys.astype(np.int64))
        st["np_rng_meta"] = torch.tensor([pos, has_gauss], dtype=torch.int64)
        st["np_rng_cached"] = torch.tensor([cached], dtype=torch.float64)
    if hasattr(runner, "py_rng"):
        v, state, g = runner.py_rng.getstate()
        st["py_rng"] = torch.tensor(list(state), dtype=torch.int64)
        st["py_rng_meta"] = torch.tensor([v, -1 if g is None else 0], dtype=torch.int64)
        if g is not None:
            st["py_rng_gauss"] = torch.tensor([g], dtype=torch.float64)
    for k in ("weights_locals", "p_choose", "dist_locals"):
        if hasattr(runner, k):
            st[k] = torch.from_numpy(np.asarray(getattr(runner, k), dtype=np.float64))
    return st


def save_runner(runner, directory, next_round):
    """Checkpoint after round ``next_round - 1`` (collective: every rank calls it)."""
    info = runner.info
    rdir = os.path.join(directory, "round_%d" % next_round)
    os.makedirs(rdir, exist_ok=True)
    _atomic_save({"next_round": torch.tensor(next_round), "clients": _client_state(runner)},
                 os.path.join(rdir, "clients_rank%d.pt" % info.rank))
    if info.is_main:
        glob_ = {"w_global": runner.w_global.detach().cpu(), "b_global": runner.b_global.detach().cpu(),
                 "mask": None if runner.mask is None else runner.mask.detach().cpu(),
                 "next_round": torch.tensor(next_round), "world": torch.tensor(info.world),
                 "runner": _runner_state(runner)}
        _atomic_save(glob_, os.path.join(rdir, "global.pt"))
        with open(os.path.join(rdir, "stat_info.json.tmp"), "w") as f:
            json.dump({k: v for k, v in runner.stat_info.items() if isinstance(v, (list, int, float))}, f)
        os.replace(os.path.join(rdir, "stat_info.json.tmp"), os.path.join(rdir, "stat_info.json"))
    rt.barrier(info)  # every shard of this round is on disk before the round becomes the latest
    if info.is_main:
        with open(os.path.join(directory, "latest.tmp"), "w") as f:
            f.write(str(next_round))
        os.replace(os.path.join(directory, "latest.tmp"), os.path.join(directory, "latest"))
    rt.barrier(info)


def latest_round(directory):
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return int(f.read().strip())


def load_runner(runner, directory):
    """Restore a runner in place from the latest complete checkpoint (any world size); returns the round to
    resume from."""
    r = latest_round(directory)
    if r is None:
        raise FileNotFoundError("no complete checkpoint in %s" % directory)
    rdir = os.path.join(directory, "round_%d" % r)
    g = torch.load(os.path.join(rdir, "global.pt"), map_location="cpu", weights_only=True)
    runner.w_global.copy_(g["w_global"].to(runner.device))
    runner.b_global.copy_(g["b_global"].to(runner.device))
    if g["mask"] is not None:
        runner.set_mask(g["mask"].to(runner.device))
    need = set(int(c) for c in runner.local)
    for path in sorted(glob.glob(os.path.join(rdir, "clients_rank*.pt"))):
        shard = torch.load(path, map_location="cpu", weights_only=True)
        if int(shard["next_round"]) != r:
            raise ValueError("checkpoint shard %s belongs to another round" % path)
        for c, st in shard["clients"].items():
            c = int(c)
            if c not in need:
                continue
            i = runner.row_of[c]
            runner.theta[i, :runner.P].copy_(st["theta"].to(runner.device))
            runner.bufs[i, :runner.Q].copy_(st["bufs"].to(runner.device))
            if "mbits" in st:
                runner.mbits[i].copy_(st["mbits"].to(runner.device))
            if "shared_bits" in st:
                runner.shared_bits[i].copy_(st["shared_bits"].to(runner.device))
            if "pers_theta" in st:
                runner.pers.theta[i, :runner.P].copy_(st["pers_theta"].to(runner.device))
                runner.pers.bufs[i, :runner.Q].copy_(st["pers_bufs"].to(runner.device))
            need.discard(c)
    if need:
        raise ValueError("checkpoint has no state for clients %s" % sorted(need))
    st = g.get("runner", {})
    if "np_rng_keys" in st:
        pos, has_gauss = (int(x) for x in st["np_rng_meta"])
        runner.np_rng.set_state(("MT19937", st["np_rng_keys"].numpy().astype(np.uint32), pos, has_gauss,
                                 float(st["np_rng_cached"][0])))
    if "py_rng" in st:
        v, gflag = (int(x) for x in st["py_rng_meta"])
        runner.py_rng.setstate((v, tuple(int(x) for x in st["py_rng"]),
                                None if gflag < 0 else float(st["py_rng_gauss"][0])))
    for k in ("weights_locals", "p_choose", "dist_locals"):
        if k in st:
            setattr(runner, k, st[k].numpy().copy())
    p = os.path.join(rdir, "stat_info.json")
    if os.path.exists(p):
        with open(p) as f:
            runner.stat_info.update(json.load(f))
    return r


def save_state_dict(sd, path):
    _atomic_save({k: v.detach().cpu() for k, v in sd.items()}, path)


def load_state_dict(path):
    return torch.load(path, map_location="cpu", weights_only=True)
