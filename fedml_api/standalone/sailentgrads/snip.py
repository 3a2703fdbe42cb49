"""Compat shim: reference import path ``fedml_api/standalone/sailentgrads/snip.py`` (its public names with the
reference signatures, plus this package's functional forms)."""
from neuroimagedisttraining_amd.algorithms.snip import (  # noqa: F401
    get_mask_from_grads, get_mean_sailency_scores, get_mean_snip_scores, get_snip_scores, global_threshold,
    mask_from_scores, mean_scores, snip_forward_conv3d, snip_forward_linear, snip_scores)
