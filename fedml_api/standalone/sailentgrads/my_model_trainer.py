"""Compat shim: reference import path ``fedml_api/standalone/sailentgrads/my_model_trainer.py``."""
from neuroimagedisttraining_amd.algorithms.trainers import VolumeTrainer as MyModelTrainer  # noqa: F401
