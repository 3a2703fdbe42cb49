"""Compat shim: reference import path ``fedml_core/distributed/topology/asymmetric_topology_manager.py`` -> ``neuroimagedisttraining_amd.comm.topology``."""
from neuroimagedisttraining_amd.comm.topology import AsymmetricTopologyManager  # noqa: F401
