"""Compat shim: reference ``fedml_api/model/cv/darts/model.py``."""
from neuroimagedisttraining_amd.nas.network import AuxiliaryHeadCIFAR, AuxiliaryHeadImageNet, Cell, NetworkCIFAR, NetworkImageNet  # noqa: F401
