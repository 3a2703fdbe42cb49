"""FL checkpoint / resume (absent in the reference): world-size independent, crash consistent, indexed
and written in the background.

Layout of ``<dir>``::

    round_<R>/clients_rank<r>.pt   rank r's clients: ids [C] + one [C, width] matrix per per-client state
    round_<R>/global.pt            w_global, b_global, SalientGrads mask, runner state (RNG streams, affinities),
                                   the world size and the client -> shard index
    round_<R>/stat_info.json
    latest                         text file "<R>" — written last (atomic rename), after every rank's shard is on disk

* **Crash consistency.**  A round directory becomes visible only through ``latest``, which rank 0 rewrites after a
  barrier that every rank reaches only once its shard is complete; a crash mid-save leaves the previous checkpoint
  intact.  Shards of a crashed run with more ranks that linger in a round directory are never read: the loader
  reads exactly the shards named by the index of the ``global.pt`` it resumes from (and rank 0 removes
  ``clients_rank<r>`` files with r >= world when it commits).
* **World-size independence.**  Rows are keyed by global client id, so a run checkpointed on 4 ranks resumes on 2
  (or 1, or 8).  The index maps every client to the shard that holds it, so each rank opens only the shards its
  clients live in (not every shard, which at config 5 — 256 clients x 46 M params — would be ~47 GB per rank).
* **Interval and retention.**  :class:`Checkpointer` saves every ``every`` rounds (and at the end) and keeps the
  ``keep_last`` newest complete round directories.
* **Background writes.**  The device rows are copied into pinned host buffers on the current stream (ordered
  before the next round's kernels, no host sync), and a writer thread serialises them once the copy event has
  completed.  The barrier + ``latest`` commit of a round runs on the main thread at the next save (or at
  :meth:`Checkpointer.close`), after the writer has finished: collectives never run off the main thread.
Everything is loaded with ``torch.load(weights_only=True)`` — no unpickling of arbitrary objects.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import re
import shutil

import numpy as np
import torch

from ..parallel import runtime as rt


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _row_mats(runner):
    """name -> (device matrix, width) of every per-client state the runner keeps (rows = runner.local order)."""
    mats = {"theta": (runner.theta, runner.P), "bufs": (runner.bufs, runner.Q)}
    if getattr(runner, "mbits", None) is not None:
        mats["mbits"] = (runner.mbits, runner.mbits.shape[1])
    if getattr(runner, "shared_bits", None) is not None:
        mats["shared_bits"] = (runner.shared_bits, runner.shared_bits.shape[1])
    if hasattr(runner, "pers"):
        mats["pers_theta"] = (runner.pers.theta, runner.P)
        mats["pers_bufs"] = (runner.pers.bufs, runner.Q)
    return mats


def _runner_state(runner):
    st = {}
    if hasattr(runner, "np_rng"):
        kind, keys, pos, has_gauss, cached = runner.np_rng.get_state()
        st["np_rng_keys"] = torch.from_numpy(np.array(keys, dtype=np.int64, copy=True))
        st["np_rng_meta"] = torch.tensor([pos, has_gauss], dtype=torch.int64)
        st["np_rng_cached"] = torch.tensor([cached], dtype=torch.float64)
    if hasattr(runner, "py_rng"):
        v, state, g = runner.py_rng.getstate()
        st["py_rng"] = torch.tensor(list(state), dtype=torch.int64)
        st["py_rng_meta"] = torch.tensor([v, -1 if g is None else 0], dtype=torch.int64)
        if g is not None:
            st["py_rng_gauss"] = torch.tensor([g], dtype=torch.float64)
    for k in ("weights_locals", "p_choose", "dist_locals"):
        if hasattr(runner, k):  # a COPY: the writer thread may serialise it after the next round changed it in place
            st[k] = torch.from_numpy(np.array(getattr(runner, k), dtype=np.float64, copy=True))
    return st


def _round_dirs(directory):
    out = []
    for name in os.listdir(directory) if os.path.isdir(directory) else ():
        m = re.fullmatch(r"round_(\d+)", name)
        if m:
            out.append(int(m.group(1)))
    return sorted(out)


def latest_round(directory):
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return int(f.read().strip())


class Checkpointer:
    """Periodic, background-written checkpoints of an FL runner (collective: every rank makes the same calls).

    ``every``: save after every ``every``-th round (``maybe_save``) — 0 disables periodic saves; ``keep_last``:
    complete round directories kept (older ones are deleted by rank 0 at commit; 0 keeps all); ``async_write``:
    serialise on a writer thread (device -> pinned copy on the stream, file write off the critical path)."""

    def __init__(self, directory, info, every=1, keep_last=2, async_write=True):
        self.dir, self.info = directory, info
        self.every, self.keep_last = int(every), int(keep_last)
        self.async_write = bool(async_write)
        self._pool = cf.ThreadPoolExecutor(1) if self.async_write else None
        self._pending = None      # (next_round, future) of a written-but-uncommitted round
        self._pinned = {}         # name -> reusable pinned host buffer
        os.makedirs(directory, exist_ok=True)

    # ------------------------------------------------------------------------------------------ snapshot
    def _host(self, name, src):
        """Host copy of a device matrix view: pinned + non-blocking on a GPU (buffers reused across saves)."""
        if src.device.type != "cuda":
            return src.detach().clone()
        buf = self._pinned.get(name)
        if buf is None or buf.shape != src.shape or buf.dtype != src.dtype:
            buf = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            self._pinned[name] = buf
        buf.copy_(src, non_blocking=True)
        return buf

    def _snapshot(self, runner, next_round):
        info = self.info
        if hasattr(runner, "sync_stats"):
            runner.sync_stats()  # device-side counters (sum_comm_params) into stat_info: collective, every rank
        C = runner.C
        shard = {"next_round": torch.tensor(next_round), "world": torch.tensor(info.world),
                 "rank": torch.tensor(info.rank), "ids": torch.tensor([int(c) for c in runner.local], dtype=torch.int64),
                 "mats": {k: self._host(k, m[:C, :w]) for k, (m, w) in _row_mats(runner).items()}}
        glob_ = None
        if info.is_main:
            glob_ = {"w_global": runner.w_global.detach().cpu().clone(),
                     "b_global": runner.b_global.detach().cpu().clone(),
                     "mask": None if runner.mask is None else runner.mask.detach().cpu().clone(),
                     "next_round": torch.tensor(next_round), "world": torch.tensor(info.world),
                     "index": torch.from_numpy(np.asarray(runner.owner, dtype=np.int64)).clone(),
                     "runner": _runner_state(runner)}
            glob_["stat_info"] = json.dumps({k: v for k, v in runner.stat_info.items()
                                             if isinstance(v, (list, int, float))})
        event = None
        if runner.device.type == "cuda":
            event = torch.cuda.Event()
            event.record()
        return shard, glob_, event

    def _write(self, next_round, shard, glob_, event):
        if event is not None:
            event.synchronize()  # the pinned copies have landed
        rdir = os.path.join(self.dir, "round_%d" % next_round)
        os.makedirs(rdir, exist_ok=True)
        _atomic_save(shard, os.path.join(rdir, "clients_rank%d.pt" % self.info.rank))
        if glob_ is not None:
            stat = glob_.pop("stat_info")
            _atomic_save(glob_, os.path.join(rdir, "global.pt"))
            with open(os.path.join(rdir, "stat_info.json.tmp"), "w") as f:
                f.write(stat)
            os.replace(os.path.join(rdir, "stat_info.json.tmp"), os.path.join(rdir, "stat_info.json"))

    # ------------------------------------------------------------------------------------------ commit
    def _commit(self):
        """Make the pending round the latest: wait for this rank's writer, barrier (every shard on disk), rank 0
        renames ``latest`` and prunes, barrier."""
        if self._pending is None:
            return
        next_round, fut = self._pending
        self._pending = None
        err = None
        if fut is not None:
            try:
                fut.result()
            except Exception as e:  # noqa: BLE001 - re-raised below on every rank together
                err = e
        # every rank learns whether every writer succeeded (a failed rank must not leave the others waiting in the
        # barrier until the collective timeout), then all raise together
        ok = torch.tensor([0.0 if err is not None else 1.0], dtype=torch.float64, device=self.info.device)
        if self.info.enabled:
            import torch.distributed as dist
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if float(ok.item()) < 1.0:
            raise RuntimeError("checkpoint of round %d failed on %s" % (next_round, "this rank: %r" % (err,)
                                                                          if err is not None else "another rank"))
        rt.barrier(self.info)
        if self.info.is_main:
            with open(os.path.join(self.dir, "latest.tmp"), "w") as f:
                f.write(str(next_round))
            os.replace(os.path.join(self.dir, "latest.tmp"), os.path.join(self.dir, "latest"))
            self._prune(next_round)
        rt.barrier(self.info)

    def _prune(self, latest):
        rdir = os.path.join(self.dir, "round_%d" % latest)
        for name in os.listdir(rdir):  # shards a crashed run with more ranks left behind
            m = re.fullmatch(r"clients_rank(\d+)\.pt(\.tmp)?", name)
            if m and (int(m.group(1)) >= self.info.world or m.group(2)):
                os.remove(os.path.join(rdir, name))
        if self.keep_last <= 0:
            return
        rounds = _round_dirs(self.dir)
        keep = set([r for r in rounds if r <= latest][-self.keep_last:])
        for r in rounds:
            if r not in keep:  # older complete rounds, and stale dirs of a crashed run past `latest`
                shutil.rmtree(os.path.join(self.dir, "round_%d" % r), ignore_errors=True)

    # ------------------------------------------------------------------------------------------ API
    def save(self, runner, next_round):
        """Checkpoint the state after round ``next_round - 1`` (commits the previous pending save first)."""
        self._commit()
        snap = self._snapshot(runner, next_round)
        if self._pool is not None:
            self._pending = (next_round, self._pool.submit(self._write, next_round, *snap))
        else:
            self._write(next_round, *snap)
            self._pending = (next_round, None)
            self._commit()

    def maybe_save(self, runner, next_round, last=False):
        """Called after every round.  Besides saving every ``every``-th round it commits a background save whose
        file writes finished (``latest`` advances then, not only at the next save: a crash loses at most ``every``
        rounds plus the rounds a save takes to write).  The readiness test is agreed on by all ranks (collective)."""
        if (self.every > 0 and next_round % self.every == 0) or last:
            self.save(runner, next_round)
        elif self._pending is not None:
            done = self._pending[1] is None or self._pending[1].done()
            flag = torch.tensor([1.0 if done else 0.0], dtype=torch.float64, device=self.info.device)
            if self.info.enabled:
                import torch.distributed as dist
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if float(flag.item()) == 1.0:
                self._commit()

    def close(self):
        """Commit any pending save (collective)."""
        self._commit()
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None


def save_runner(runner, directory, next_round, keep_last=0):
    """Synchronous checkpoint after round ``next_round - 1`` (collective: every rank calls it)."""
    ck = Checkpointer(directory, runner.info, every=1, keep_last=keep_last, async_write=False)
    ck.save(runner, next_round)
    ck.close()


def load_runner(runner, directory):
    """Restore a runner in place from the latest complete checkpoint (any world size); returns the round to
    resume from.  Each rank reads only the shards (named by the checkpoint's client index) holding its clients."""
    r = latest_round(directory)
    if r is None:
        raise FileNotFoundError("no complete checkpoint in %s" % directory)
    rdir = os.path.join(directory, "round_%d" % r)
    g = torch.load(os.path.join(rdir, "global.pt"), map_location="cpu", weights_only=True)
    if "index" not in g or "world" not in g:  # the earlier per-client-dict layout (no client index)
        raise ValueError("checkpoint %s uses an unsupported (pre-index) format: it has no client index; re-run from "
                         "scratch or convert it with the version that wrote it" % rdir)
    runner.w_global.copy_(g["w_global"].to(runner.device))
    runner.b_global.copy_(g["b_global"].to(runner.device))
    if g["mask"] is not None:
        runner.set_mask(g["mask"].to(runner.device))
    need = set(int(c) for c in runner.local)
    index = g["index"].numpy()
    world = int(g["world"])
    shards = sorted(set(int(index[c]) for c in need))
    assert all(0 <= s < world for s in shards), "corrupt client index in %s" % rdir
    mats = _row_mats(runner)
    for s in shards:
        shard = torch.load(os.path.join(rdir, "clients_rank%d.pt" % s), map_location="cpu", weights_only=True)
        if "ids" not in shard or "mats" not in shard:
            raise ValueError("checkpoint shard %s uses an unsupported (pre-index) format" % rdir)
        if int(shard["next_round"]) != r or int(shard["world"]) != world or int(shard["rank"]) != s:
            raise ValueError("checkpoint shard %d of %s belongs to another save" % (s, rdir))
        ids = shard["ids"].tolist()
        take = [(j, int(c)) for j, c in enumerate(ids) if int(c) in need]
        if not take:
            continue
        src = torch.tensor([j for j, _ in take], dtype=torch.long)
        dst = torch.tensor([runner.row_of[c] for _, c in take], dtype=torch.long, device=runner.device)
        for k, t in shard["mats"].items():
            m, w = mats[k]
            m[dst, :w] = t.index_select(0, src).to(runner.device)
        need.difference_update(c for _, c in take)
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
