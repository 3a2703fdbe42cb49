"""Compat shim: reference import path ``fedml_core/trainer/model_trainer.py`` -> ``neuroimagedisttraining_amd.core.trainer``."""
from neuroimagedisttraining_amd.core.trainer import ModelTrainer  # noqa: F401
