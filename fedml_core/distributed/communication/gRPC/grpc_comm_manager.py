"""Compat shim: reference import path ``fedml_core/distributed/communication/gRPC/grpc_comm_manager.py`` -> ``neuroimagedisttraining_amd.comm.managers``."""
from neuroimagedisttraining_amd.comm.managers import GRPCCommManager  # noqa: F401
