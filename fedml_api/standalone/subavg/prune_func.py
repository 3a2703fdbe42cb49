"""Compat shim: reference import path ``fedml_api/standalone/subavg/prune_func.py``."""
from neuroimagedisttraining_amd.algorithms.sparse import dist_masks, fake_prune, print_pruning, real_prune  # noqa: F401
