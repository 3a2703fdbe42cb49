"""Compat shim: reference import path ``fedml_core/distributed/topology/base_topology_manager.py`` -> ``neuroimagedisttraining_amd.comm.topology``."""
from neuroimagedisttraining_amd.comm.topology import BaseTopologyManager  # noqa: F401
