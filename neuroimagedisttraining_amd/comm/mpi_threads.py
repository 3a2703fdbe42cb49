"""MPI-style communication manager: a send thread and a receive thread around an ``mpi4py``-like ``comm``
(reference ``fedml_core/distributed/communication/mpi/{com_manager.py:13-98, mpi_send_thread.py:20-31,
mpi_receive_thread.py:19-28}``).

``comm`` is duck-typed: anything with ``send(obj, dest=...)`` and ``recv()`` — ``mpi4py.MPI.COMM_WORLD`` when
mpi4py is installed (it is not in this image), or :class:`TorchP2PComm`, which carries the same string payloads
through per-rank mailboxes in the torch.distributed TCPStore of the one-process-per-GPU runtime.

Differences from the reference (same observable behaviour, no busy polling, clean shutdown):

* the send thread blocks on its queue (``get(timeout)``) instead of sleeping 3 ms between ``empty()`` checks;
* the receive loop delivers messages as they arrive instead of polling every 0.3 s;
* threads stop through an event plus a sentinel message to self, not ``PyThreadState_SetAsyncExc``.
"""
from __future__ import annotations

import logging
import queue
import threading
import traceback

import torch

from .message import BaseCommunicationManager, Message, Observer

log = logging.getLogger(__name__)

_STOP = "__nidt_stop__"


class TorchP2PComm:
    """``send(str, dest)`` / ``recv() -> str`` over the torch.distributed control-plane store.

    Every rank owns a mailbox in the job's c10d TCPStore: a sender reserves slot ``i`` with an atomic
    ``add`` on the receiver's tail counter and writes the payload to ``<prefix>/<dest>/<i>``; the receiver
    consumes its slots in order (``check`` with back-off polling, then ``get`` + ``delete_key``).  Control messages therefore never
    share the gloo/RCCL data channels, a blocked receive can always be ended (timed waits), and a message to
    self (the stop sentinel) needs no peer — properties gloo point-to-point lacks (no self-send; a timed-out
    receive tears the pair down)."""

    def __init__(self, store=None, prefix="nidt/mbox"):
        import torch.distributed as dist
        self.dist = dist
        self.store = store if store is not None else dist.distributed_c10d._get_default_store()
        self.prefix = prefix
        self.rank = dist.get_rank()
        self.head = 0

    def Get_rank(self):  # noqa: N802 (mpi4py spelling)
        return self.rank

    def Get_size(self):  # noqa: N802
        return self.dist.get_world_size()

    def send(self, obj, dest):
        slot = int(self.store.add("%s/%d/tail" % (self.prefix, dest), 1)) - 1
        self.store.set("%s/%d/%d" % (self.prefix, dest, slot), str(obj).encode())

    def recv(self, max_poll_s=0.02):
        import time
        key = "%s/%d/%d" % (self.prefix, self.rank, self.head)
        delay = 1e-4
        while not self.store.check([key]):  # non-blocking probe (a timed store.wait logs every timeout)
            time.sleep(delay)
            delay = min(max_poll_s, delay * 2)
        data = self.store.get(key)
        self.store.delete_key(key)
        self.head += 1
        return data.decode()


class MPISendThread(threading.Thread):
    """Drains ``q`` and sends every message's JSON to its receiver."""

    def __init__(self, comm, rank, size, name, q):
        super().__init__(name=name, daemon=True)
        self.comm, self.rank, self.size, self.q = comm, rank, size, q
        self._stop_event = threading.Event()

    def run(self):
        log.debug("Starting %s. Process ID = %d", self.name, self.rank)
        while not self._stop_event.is_set():
            try:
                msg = self.q.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                self.comm.send(msg.to_json() if isinstance(msg, Message) else msg,
                               dest=msg.get(Message.MSG_ARG_KEY_RECEIVER) if isinstance(msg, Message) else self.rank)
            except Exception:  # noqa: BLE001 - keep the thread alive like the reference
                traceback.print_exc()

    def stop(self):
        self._stop_event.set()

    def stopped(self):
        return self._stop_event.is_set()


class MPIReceiveThread(threading.Thread):
    """Blocks in ``comm.recv()`` and queues decoded :class:`Message` objects."""

    def __init__(self, comm, rank, size, name, q):
        super().__init__(name=name, daemon=True)
        self.comm, self.rank, self.size, self.q = comm, rank, size, q
        self._stop_event = threading.Event()

    def run(self):
        log.debug("Starting Thread: %s. Process ID = %d", self.name, self.rank)
        while not self._stop_event.is_set():
            try:
                s = self.comm.recv()
            except Exception:  # noqa: BLE001
                if self._stop_event.is_set():
                    break
                traceback.print_exc()
                continue
            if s == _STOP:
                break
            try:
                m = Message()
                m.init_from_json_string(s)
            except Exception:  # noqa: BLE001 - a malformed message must not kill the receive loop
                traceback.print_exc()
                continue
            self.q.put(m)

    def stop(self):
        self._stop_event.set()

    def stopped(self):
        return self._stop_event.is_set()


class MpiCommunicationManager(BaseCommunicationManager):
    """Reference-signature MPI manager (``MpiCommunicationManager(comm, rank, size, node_type)``)."""

    def __init__(self, comm, rank, size, node_type="client"):
        if comm is None:
            try:
                from mpi4py import MPI
                comm = MPI.COMM_WORLD
            except ImportError:
                comm = TorchP2PComm()
        self.comm, self.rank, self.size, self.node_type = comm, rank, size, node_type
        self._observers = []
        self.q_sender, self.q_receiver = queue.Queue(0), queue.Queue(0)
        role = "Server" if node_type == "server" else "Client"
        self.send_thread = MPISendThread(comm, rank, size, role + "SendThread", self.q_sender)
        self.receive_thread = MPIReceiveThread(comm, rank, size, role + "ReceiveThread", self.q_receiver)
        self.send_thread.start()
        self.receive_thread.start()
        self.is_running = True

    def send_message(self, msg: Message):
        self.q_sender.put(msg)

    def add_observer(self, observer: Observer):
        self._observers.append(observer)

    def remove_observer(self, observer: Observer):
        self._observers.remove(observer)

    def notify(self, msg):
        for o in list(self._observers):
            o.receive_message(msg.get_type(), msg)

    def poll_once(self, timeout=0.0):
        try:
            msg = self.q_receiver.get(timeout=timeout) if timeout else self.q_receiver.get_nowait()
        except queue.Empty:
            return False
        self.notify(msg)
        return True

    def handle_receive_message(self):
        self.is_running = True
        while self.is_running:
            self.poll_once(timeout=0.05)
        log.info("handle_receive_message stopped")

    def stop_receive_message(self):
        self.is_running = False
        self.send_thread.stop()
        self.receive_thread.stop()
        try:  # unblock our own recv() with a sentinel to self
            self.comm.send(_STOP, dest=self.rank)
        except Exception:  # noqa: BLE001
            pass
        self.send_thread.join(timeout=5)
        self.receive_thread.join(timeout=5)
