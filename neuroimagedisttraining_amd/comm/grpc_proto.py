"""Wire-compatible gRPC messages and service for the reference's ``grpc_comm_manager.proto``
(``fedml_core/distributed/communication/gRPC/proto/grpc_comm_manager.proto:1-16``)::

    service gRPCCommManager {
      rpc sendMessage (CommRequest) returns (CommResponse);
      rpc handleReceiveMessage(CommRequest) returns (CommResponse);
    }
    message CommRequest  { int32 client_id = 1; string message = 2; }
    message CommResponse { int32 client_id = 1; string message = 2; }

The reference ships protoc output (``grpc_comm_manager_pb2.py`` / ``_pb2_grpc.py``).  ``grpc_tools`` / protoc
are not available here, so the same file descriptor is built programmatically and registered in the default
protobuf pool; the message classes, the ``gRPCCommManagerStub`` client, the ``gRPCCommManagerServicer`` base
class and ``add_gRPCCommManagerServicer_to_server`` follow protoc's naming, and the bytes on the wire are the
same, so peers running the reference's generated code interoperate.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool
try:  # protobuf >= 4
    from google.protobuf.message_factory import GetMessageClass as _get_cls
except ImportError:  # pragma: no cover - older protobuf
    from google.protobuf import message_factory as _mf
    _get_cls = _mf.MessageFactory().GetPrototype

SERVICE = "gRPCCommManager"
_FILE = "grpc_comm_manager.proto"


def _build_file():
    fd = descriptor_pb2.FileDescriptorProto(name=_FILE, syntax="proto3")
    for mname in ("CommRequest", "CommResponse"):
        m = fd.message_type.add(name=mname)
        m.field.add(name="client_id", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, json_name="clientId")
        m.field.add(name="message", number=2, type=descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, json_name="message")
    svc = fd.service.add(name=SERVICE)
    for meth in ("sendMessage", "handleReceiveMessage"):
        svc.method.add(name=meth, input_type=".CommRequest", output_type=".CommResponse")
    return fd


_pool = descriptor_pool.Default()
try:
    DESCRIPTOR = _pool.FindFileByName(_FILE)
except KeyError:
    DESCRIPTOR = _pool.Add(_build_file()) if hasattr(_pool, "Add") else None
    DESCRIPTOR = _pool.FindFileByName(_FILE)

CommRequest = _get_cls(DESCRIPTOR.message_types_by_name["CommRequest"])
CommResponse = _get_cls(DESCRIPTOR.message_types_by_name["CommResponse"])


class gRPCCommManagerStub:  # noqa: N801 (protoc naming)
    """Client stub: ``stub.sendMessage(CommRequest(...), timeout=...) -> CommResponse``."""

    def __init__(self, channel):
        self.sendMessage = channel.unary_unary(
            "/%s/sendMessage" % SERVICE, request_serializer=CommRequest.SerializeToString,
            response_deserializer=CommResponse.FromString)
        self.handleReceiveMessage = channel.unary_unary(
            "/%s/handleReceiveMessage" % SERVICE, request_serializer=CommRequest.SerializeToString,
            response_deserializer=CommResponse.FromString)


class gRPCCommManagerServicer:  # noqa: N801
    """Service base class; override ``sendMessage`` / ``handleReceiveMessage``."""

    def sendMessage(self, request, context):  # noqa: N802
        import grpc
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        raise NotImplementedError("sendMessage")

    def handleReceiveMessage(self, request, context):  # noqa: N802
        import grpc
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        raise NotImplementedError("handleReceiveMessage")


def add_gRPCCommManagerServicer_to_server(servicer, server):  # noqa: N802
    import grpc
    handlers = {
        "sendMessage": grpc.unary_unary_rpc_method_handler(
            servicer.sendMessage, request_deserializer=CommRequest.FromString,
            response_serializer=CommResponse.SerializeToString),
        "handleReceiveMessage": grpc.unary_unary_rpc_method_handler(
            servicer.handleReceiveMessage, request_deserializer=CommRequest.FromString,
            response_serializer=CommResponse.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
