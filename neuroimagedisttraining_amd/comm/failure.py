"""Failure detection for the one-process-per-GPU runtime: store-based heartbeats.

The reference has no failure handling beyond ``MPI.COMM_WORLD.Abort()`` (``fedml_api/utils/context.py:9-18``,
``server_manager.py:61-64``).  Here a rank that dies (OOM kill, node loss) would leave the others
blocked inside an RCCL collective until the process-group timeout.  :class:`HeartbeatMonitor` lets every rank
publish a heartbeat into a ``torch.distributed`` key-value store (the process group's own TCPStore, or any
``Store``) from a daemon thread, and lets any rank ask which peers went silent — the FL executor checks before
each round's collectives and fails fast with :class:`PeerFailure` naming the dead ranks.

Heartbeats are monotonically increasing counters written with ``store.set`` (no clocks are compared across
hosts): a peer is dead when its counter has not advanced for ``timeout_s`` of the observer's own clock.
"""
from __future__ import annotations

import threading
import time


class PeerFailure(RuntimeError):
    def __init__(self, dead):
        self.dead = sorted(dead)
        super().__init__("ranks %s stopped sending heartbeats" % self.dead)


def default_store():
    """The default process group's store (None without an initialised process group)."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001 - private API: degrade to "no monitor"
        return None


class HeartbeatMonitor:
    """Publish this rank's heartbeat every ``interval_s``; report peers silent for longer than ``timeout_s``."""

    def __init__(self, store, rank, world, interval_s=1.0, timeout_s=30.0, prefix="nidt/hb/"):
        self.store, self.rank, self.world = store, rank, world
        self.interval_s, self.timeout_s, self.prefix = float(interval_s), float(timeout_s), prefix
        self._beat = 0
        self._seen = {}  # rank -> (counter, local time it last changed)
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._publish()
        self._th = threading.Thread(target=self._loop, name="nidt-heartbeat-%d" % rank, daemon=True)
        self._th.start()

    def _key(self, r):
        return "%s%d" % (self.prefix, r)

    def _publish(self):
        self._beat += 1
        self.store.set(self._key(self.rank), str(self._beat))

    def _loop(self):
        while not self._stop.wait(self.interval_s):
            try:
                self._publish()
            except Exception:  # noqa: BLE001 - the store (rank 0's server) may be gone: stop beating
                break

    def stop(self):
        """Stop publishing (a stopped monitor looks dead to its peers after ``timeout_s``)."""
        self._stop.set()
        self._th.join(timeout=5)

    def dead_ranks(self, now=None):
        """Ranks whose counter has not advanced for ``timeout_s`` (never-seen ranks count from first check)."""
        now = time.monotonic() if now is None else now
        dead = []
        with self._lock:
            for r in range(self.world):
                if r == self.rank:
                    continue
                try:
                    cur = int(self.store.get(self._key(r))) if self.store.check([self._key(r)]) else 0
                except Exception:  # noqa: BLE001 - unreachable store: treat the peer as silent
                    cur = None
                last = self._seen.get(r)
                if last is None or (cur is not None and cur != last[0]):
                    self._seen[r] = (cur, now)
                elif now - last[1] > self.timeout_s:
                    dead.append(r)
        return dead

    def check_or_raise(self):
        dead = self.dead_ranks()
        if dead:
            raise PeerFailure(dead)

    def wait_all_alive(self, timeout_s=None):
        """Block until every peer has published at least one heartbeat (start-up barrier without collectives)."""
        t_end = time.monotonic() + (self.timeout_s if timeout_s is None else timeout_s)
        keys = [self._key(r) for r in range(self.world)]
        while time.monotonic() < t_end:
            if self.store.check(keys):
                return True
            time.sleep(min(0.05, self.interval_s))
        return False
