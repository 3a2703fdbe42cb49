"""Compat shim for the reference's protoc output ``grpc_comm_manager_pb2.py``: the same messages built from
the same descriptor (``neuroimagedisttraining_amd.comm.grpc_proto``), wire compatible."""
from neuroimagedisttraining_amd.comm.grpc_proto import DESCRIPTOR, CommRequest, CommResponse  # noqa: F401
