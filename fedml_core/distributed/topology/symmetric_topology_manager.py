"""Compat shim: reference import path ``fedml_core/distributed/topology/symmetric_topology_manager.py`` -> ``neuroimagedisttraining_amd.comm.topology``."""
from neuroimagedisttraining_amd.comm.topology import SymmetricTopologyManager  # noqa: F401
