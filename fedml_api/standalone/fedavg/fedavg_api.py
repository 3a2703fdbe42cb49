"""Compat shim: reference import path ``fedml_api/standalone/fedavg/fedavg_api.py``."""
from neuroimagedisttraining_amd.algorithms.fedavg import FedAvgAPI, FedProxAPI  # noqa: F401
