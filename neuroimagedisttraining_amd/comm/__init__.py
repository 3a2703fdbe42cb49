"""Control-plane communication: messages, managers/backends, topologies."""
from .message import BaseCommunicationManager, Message, Observer
from .managers import (ClientManager, GRPCCommManager, InProcCommManager, MpiCommunicationManager, MqttCommManager,
                       ServerManager, TorchDistCommManager, make_comm_manager)
from .topology import (AsymmetricTopologyManager, BaseTopologyManager, SymmetricTopologyManager, mixing_matrix,
                       ring_lattice)
