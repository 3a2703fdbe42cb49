"""Compat shim: reference import path ``fedml_api/standalone/fedfomo/my_model_trainer_my.py``."""
from neuroimagedisttraining_amd.algorithms.trainers import ClassificationTrainer as MyModelTrainer  # noqa: F401
