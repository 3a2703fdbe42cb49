"""MQTT backend without paho: a small MQTT 3.1.1 client and broker over plain sockets.

The reference's ``MqttCommManager`` (``fedml_core/distributed/communication/mqtt/mqtt_comm_manager.py:14-126``)
drives ``paho.mqtt.client`` against an external broker.  paho is not part of this image, so the wire protocol
is implemented here directly (MQTT 3.1.1, OASIS standard, QoS 0 publish; QoS 1 subscribe acks):

* :class:`MqttClient` — CONNECT / CONNACK, SUBSCRIBE / SUBACK, PUBLISH (QoS 0), PINGREQ keep-alive,
  DISCONNECT; one reader thread dispatches ``on_message(topic, payload)``.  Interoperates with any 3.1.1
  broker (mosquitto, EMQX, ...).
* :class:`MqttBroker` — a threaded in-process broker (topic filters with ``+`` / ``#`` wildcards) for tests
  and single-node runs where no external broker exists.
* :class:`MqttCommManager` — the reference's topic scheme: the server (id 0) subscribes ``topic<client>`` for
  every client and publishes to ``topic0_<receiver>``; client ``i`` publishes to ``topic<i>`` and subscribes
  ``topic0_<i>``.  Payloads are ``Message.to_json()`` strings, as in the reference (``:110-120``).

Unlike the reference (which returns from ``__init__`` before the subscription is acknowledged, ``:60-70``),
the manager waits for SUBACK so a message published right after construction is not lost.
"""
from __future__ import annotations

import logging
import queue
import socket
import struct
import threading
import time

from .message import BaseCommunicationManager, Message, Observer

log = logging.getLogger(__name__)

CONNECT, CONNACK, PUBLISH, SUBSCRIBE, SUBACK, PINGREQ, PINGRESP, DISCONNECT = 1, 2, 3, 8, 9, 12, 13, 14


def _enc_len(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n % 128
        n //= 128
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _enc_str(s) -> bytes:
    b = s.encode() if isinstance(s, str) else bytes(s)
    return struct.pack("!H", len(b)) + b


def _packet(ptype: int, flags: int, body: bytes) -> bytes:
    return bytes([(ptype << 4) | flags]) + _enc_len(len(body)) + body


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("mqtt: connection closed")
        buf += chunk
    return bytes(buf)


def read_packet(sock):
    """Read one control packet; returns ``(type, flags, body)``."""
    h = _recv_exact(sock, 1)[0]
    mult, n = 1, 0
    for _ in range(4):
        b = _recv_exact(sock, 1)[0]
        n += (b & 0x7F) * mult
        if not b & 0x80:
            break
        mult *= 128
    else:
        raise ValueError("mqtt: malformed remaining length")
    return h >> 4, h & 0x0F, _recv_exact(sock, n) if n else b""


def topic_matches(filt: str, topic: str) -> bool:
    """MQTT topic-filter match (``+`` one level, ``#`` the rest)."""
    fp, tp = filt.split("/"), topic.split("/")
    for i, f in enumerate(fp):
        if f == "#":
            return True
        if i >= len(tp) or (f != "+" and f != tp[i]):
            return False
    return len(fp) == len(tp)


def _parse_publish(flags: int, body: bytes):
    tl = struct.unpack("!H", body[:2])[0]
    topic = body[2:2 + tl].decode()
    pos = 2 + tl
    if (flags >> 1) & 3:  # QoS > 0 carries a packet id
        pos += 2
    return topic, body[pos:]


class MqttClient:
    """Minimal MQTT 3.1.1 client (QoS 0 publish, blocking subscribe)."""

    def __init__(self, client_id: str, host="127.0.0.1", port=1883, keepalive=60, on_message=None, timeout=10.0):
        self.client_id = str(client_id)
        self.on_message = on_message
        self._sock = socket.create_connection((host, port), timeout=timeout)
        self._sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._wlock = threading.Lock()
        self._mid = 0
        self._acks = {}
        self._cv = threading.Condition()
        self._closed = False
        body = _enc_str("MQTT") + bytes([4, 0x02]) + struct.pack("!H", keepalive) + _enc_str(self.client_id)
        self._sock.sendall(_packet(CONNECT, 0, body))
        t, _, b = read_packet(self._sock)
        if t != CONNACK or len(b) < 2 or b[1] != 0:
            raise ConnectionError("mqtt: CONNACK refused (%r)" % (b,))
        self.connack_rc = b[1]
        self._sock.settimeout(None)
        self._keepalive = keepalive
        self._rx = threading.Thread(target=self._loop, name="mqtt-rx-%s" % self.client_id, daemon=True)
        self._rx.start()
        if keepalive:
            self._ping = threading.Thread(target=self._ping_loop, daemon=True)
            self._ping.start()

    def _send(self, data: bytes):
        with self._wlock:
            self._sock.sendall(data)

    def subscribe(self, topic: str, qos: int = 0, timeout=10.0) -> int:
        with self._cv:
            self._mid = self._mid % 65535 + 1
            mid = self._mid
        body = struct.pack("!H", mid) + _enc_str(topic) + bytes([qos])
        self._send(_packet(SUBSCRIBE, 0x02, body))
        with self._cv:
            if not self._cv.wait_for(lambda: mid in self._acks or self._closed, timeout):
                raise TimeoutError("mqtt: no SUBACK for %r" % topic)
            return self._acks.pop(mid, 0x80)

    def publish(self, topic: str, payload):
        data = payload.encode() if isinstance(payload, str) else bytes(payload)
        self._send(_packet(PUBLISH, 0, _enc_str(topic) + data))

    def _loop(self):
        try:
            while True:
                t, flags, body = read_packet(self._sock)
                if t == PUBLISH:
                    topic, payload = _parse_publish(flags, body)
                    if self.on_message is not None:
                        try:
                            self.on_message(topic, payload)
                        except Exception:  # noqa: BLE001 - a bad message must not kill the reader
                            log.exception("mqtt: on_message failed")
                elif t == SUBACK:
                    mid = struct.unpack("!H", body[:2])[0]
                    with self._cv:
                        self._acks[mid] = body[2] if len(body) > 2 else 0
                        self._cv.notify_all()
        except (ConnectionError, OSError, ValueError):
            pass
        finally:
            with self._cv:
                self._closed = True
                self._cv.notify_all()

    def _ping_loop(self):
        while not self._closed:
            time.sleep(max(1.0, self._keepalive / 2))
            if self._closed:
                break
            try:
                self._send(_packet(PINGREQ, 0, b""))
            except OSError:
                break

    def disconnect(self):
        if self._closed:
            return
        try:
            self._send(_packet(DISCONNECT, 0, b""))
        except OSError:
            pass
        self._closed = True
        try:
            self._sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self._sock.close()


class MqttBroker:
    """Threaded MQTT 3.1.1 broker (QoS 0 delivery, no retained messages / sessions).  ``port=0`` picks a free
    port (``broker.port``)."""

    def __init__(self, host="127.0.0.1", port=0):
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self._srv.listen(64)
        self.host, self.port = self._srv.getsockname()
        self._subs = {}  # conn -> set of filters
        self._locks = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._accept, name="mqtt-broker", daemon=True)
        self._th.start()

    def _accept(self):
        while not self._stop.is_set():
            try:
                conn, _ = self._srv.accept()
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _write(self, conn, data):
        lk = self._locks.get(conn)
        if lk is None:
            return
        with lk:
            conn.sendall(data)

    def _serve(self, conn):
        try:
            t, _, body = read_packet(conn)
            if t != CONNECT:
                conn.close()
                return
            with self._lock:
                self._subs[conn] = set()
                self._locks[conn] = threading.Lock()
            self._write(conn, _packet(CONNACK, 0, b"\x00\x00"))
            while True:
                t, flags, body = read_packet(conn)
                if t == PUBLISH:
                    topic, payload = _parse_publish(flags, body)
                    out = _packet(PUBLISH, 0, _enc_str(topic) + payload)
                    with self._lock:
                        targets = [c for c, fs in self._subs.items() if any(topic_matches(f, topic) for f in fs)]
                    for c in targets:
                        try:
                            self._write(c, out)
                        except OSError:
                            pass
                elif t == SUBSCRIBE:
                    mid = body[:2]
                    pos, granted = 2, bytearray()
                    while pos < len(body):
                        tl = struct.unpack("!H", body[pos:pos + 2])[0]
                        filt = body[pos + 2:pos + 2 + tl].decode()
                        pos += 3 + tl
                        with self._lock:
                            self._subs[conn].add(filt)
                        granted.append(0)
                    self._write(conn, _packet(SUBACK, 0, mid + bytes(granted)))
                elif t == PINGREQ:
                    self._write(conn, _packet(PINGRESP, 0, b""))
                elif t == DISCONNECT:
                    break
        except (ConnectionError, OSError, ValueError):
            pass
        finally:
            with self._lock:
                self._subs.pop(conn, None)
                self._locks.pop(conn, None)
            try:
                conn.close()
            except OSError:
                pass

    def close(self):
        self._stop.set()
        try:
            self._srv.close()
        except OSError:
            pass
        with self._lock:
            conns = list(self._subs)
        for c in conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass


class MqttCommManager(BaseCommunicationManager):
    """The reference's MQTT manager (same constructor, topic scheme and JSON payloads) on :class:`MqttClient`.

    Incoming messages are queued by the socket reader and delivered to observers by
    :meth:`handle_receive_message` (or :meth:`poll_once`), like the other backends here; the reference calls
    observers from paho's network thread instead."""

    def __init__(self, host, port, topic="fedml", client_id=0, client_num=0):
        self._observers = []
        self._topic = topic
        self._client_id = client_id
        self.client_num = client_num
        self.q = queue.Queue()
        self._running = False
        self._client = MqttClient("fedml_%s_%s" % (topic, client_id), host or "127.0.0.1", int(port or 1883),
                                  on_message=self._on_message)
        if client_id == 0:
            for cid in range(1, client_num + 1):
                self._client.subscribe(self._topic + str(cid), 0)
        else:
            self._client.subscribe(self._topic + "0_" + str(client_id), 0)

    @property
    def client_id(self):
        return self._client_id

    @property
    def topic(self):
        return self._topic

    def _on_message(self, topic, payload):
        m = Message()
        m.init_from_json_string(payload.decode("utf-8"))
        self.q.put(m)

    def add_observer(self, observer: Observer):
        self._observers.append(observer)

    def remove_observer(self, observer: Observer):
        self._observers.remove(observer)

    def send_message(self, msg: Message):
        if self._client_id == 0:
            self._client.publish(self._topic + "0_" + str(msg.get_receiver_id()), msg.to_json())
        else:
            self._client.publish(self._topic + str(self._client_id), msg.to_json())

    def poll_once(self, timeout=0.0):
        try:
            msg = self.q.get(timeout=timeout) if timeout else self.q.get_nowait()
        except queue.Empty:
            return False
        for o in list(self._observers):
            o.receive_message(msg.get_type(), msg)
        return True

    def handle_receive_message(self):
        self._running = True
        while self._running:
            self.poll_once(timeout=0.05)

    def stop_receive_message(self):
        self._running = False
        self._client.disconnect()
