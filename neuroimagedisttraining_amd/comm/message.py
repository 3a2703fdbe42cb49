"""Control-plane message and observer API (reference ``fedml_core/distributed/communication/{message,observer,
base_com_manager}.py``).

A :class:`Message` is a dict with ``msg_type``, ``sender``, ``receiver`` and arbitrary params.  JSON
serialisation encodes tensors / numpy arrays as ``{"__tensor__": dtype, "shape": [...], "data": [...]}`` so a
state dict round-trips exactly (the reference's ``to_json`` just dumps the dict and breaks on tensors).
Bulk tensor payloads on the MI355X path do not go through JSON at all — they ride RCCL collectives
(:mod:`neuroimagedisttraining_amd.parallel.runtime`); messages carry only control data.
"""
from __future__ import annotations

import abc
import json

import numpy as np
import torch


def _enc(v):
    if torch.is_tensor(v):
        t = v.detach().cpu()
        return {"__tensor__": str(t.dtype).replace("torch.", ""), "shape": list(t.shape),
                "data": t.reshape(-1).tolist()}
    if isinstance(v, np.ndarray):
        return {"__ndarray__": str(v.dtype), "shape": list(v.shape), "data": v.reshape(-1).tolist()}
    if isinstance(v, dict):
        return {"__dict__": [[_enc(k), _enc(x)] for k, x in v.items()]}
    if isinstance(v, (list, tuple)):
        return [_enc(x) for x in v]
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    return v


def _dec(v):
    if isinstance(v, dict):
        if "__tensor__" in v:
            dt = getattr(torch, v["__tensor__"])
            return torch.tensor(v["data"], dtype=dt).reshape(v["shape"])
        if "__ndarray__" in v:
            return np.asarray(v["data"], dtype=v["__ndarray__"]).reshape(v["shape"])
        if "__dict__" in v:
            return {_dec(k): _dec(x) for k, x in v["__dict__"]}
        return {k: _dec(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_dec(x) for x in v]
    return v


class Message:
    MSG_ARG_KEY_OPERATION = "operation"
    MSG_ARG_KEY_TYPE = "msg_type"
    MSG_ARG_KEY_SENDER = "sender"
    MSG_ARG_KEY_RECEIVER = "receiver"

    MSG_OPERATION_SEND = "send"
    MSG_OPERATION_RECEIVE = "receive"
    MSG_OPERATION_BROADCAST = "broadcast"
    MSG_OPERATION_REDUCE = "reduce"

    MSG_ARG_KEY_MODEL_PARAMS = "model_params"

    def __init__(self, type=0, sender_id=0, receiver_id=0):  # noqa: A002 (reference signature)
        self.type = type
        self.sender_id = sender_id
        self.receiver_id = receiver_id
        self.msg_params = {self.MSG_ARG_KEY_TYPE: type, self.MSG_ARG_KEY_SENDER: sender_id,
                           self.MSG_ARG_KEY_RECEIVER: receiver_id}

    def init(self, msg_params):
        self.msg_params = msg_params
        self.type = msg_params.get(self.MSG_ARG_KEY_TYPE, 0)
        self.sender_id = msg_params.get(self.MSG_ARG_KEY_SENDER, 0)
        self.receiver_id = msg_params.get(self.MSG_ARG_KEY_RECEIVER, 0)

    def init_from_json_string(self, json_string):
        self.init(_dec(json.loads(json_string)))

    def get_sender_id(self):
        return self.sender_id

    def get_receiver_id(self):
        return self.receiver_id

    def add_params(self, key, value):
        self.msg_params[key] = value

    def get_params(self):
        return self.msg_params

    def add(self, key, value):
        self.msg_params[key] = value

    def get(self, key):
        return self.msg_params.get(key)

    def get_type(self):
        return self.msg_params[self.MSG_ARG_KEY_TYPE]

    def to_string(self):
        return self.msg_params

    def to_json(self):
        return json.dumps(_enc(self.msg_params))

    def get_content(self):
        return "%s" % {k: v for k, v in self.msg_params.items() if k != self.MSG_ARG_KEY_MODEL_PARAMS}


class Observer(abc.ABC):
    @abc.abstractmethod
    def receive_message(self, msg_type, msg_params) -> None:
        ...


class BaseCommunicationManager(abc.ABC):
    @abc.abstractmethod
    def send_message(self, msg: Message):
        ...

    @abc.abstractmethod
    def add_observer(self, observer: Observer):
        ...

    @abc.abstractmethod
    def remove_observer(self, observer: Observer):
        ...

    @abc.abstractmethod
    def handle_receive_message(self):
        ...

    @abc.abstractmethod
    def stop_receive_message(self):
        ...
