"""Compat shim: reference import path ``fedml_api/standalone/turboaggregate/TA_trainer.py``."""
from neuroimagedisttraining_amd.algorithms.turboaggregate import TurboAggregateTrainer  # noqa: F401
