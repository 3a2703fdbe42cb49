"""Compat shim: reference import path ``fedml_api/standalone/subavg/my_model_trainer.py``."""
from neuroimagedisttraining_amd.algorithms.trainers import ClassificationTrainer as MyModelTrainer  # noqa: F401
