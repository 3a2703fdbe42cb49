"""Compat shim for the reference's ``grpc_comm_manager_pb2_grpc.py`` (service stub / servicer / registration)."""
from neuroimagedisttraining_amd.comm.grpc_proto import (  # noqa: F401
    add_gRPCCommManagerServicer_to_server, gRPCCommManagerServicer, gRPCCommManagerStub)
