"""Compat shim: reference ``fedml_core/distributed/communication/gRPC/grpc_server.py`` (``GRPCCOMMServicer``)."""
from neuroimagedisttraining_amd.comm.managers import GRPCCOMMServicer  # noqa: F401
