"""Trainer abstraction (reference: ``fedml_core/trainer/model_trainer.py:8-58``).

A ``ModelTrainer`` owns one ``nn.Module`` shared by every simulated client; clients swap their
parameters in and out through :meth:`get_model_params` / :meth:`set_model_params`.  The
accounting helpers delegate to :mod:`neuroimagedisttraining_amd.utils.flops`, which (unlike the
reference, quirk Q15) counts ``Conv3d`` and uses the dataset's true input shape.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import torch


class ModelTrainer(ABC):
    """Framework-agnostic trainer interface used by every algorithm's ``Client``."""

    def __init__(self, model, args=None):
        self.model = model
        self.id = 0
        self.args = args

    def set_id(self, trainer_id):
        self.id = trainer_id

    @abstractmethod
    def get_model_params(self):
        ...

    @abstractmethod
    def set_model_params(self, model_parameters):
        ...

    @abstractmethod
    def train(self, train_data, device, args=None):
        ...

    @abstractmethod
    def test(self, test_data, device, args=None):
        ...

    def test_on_the_server(self, train_data_local_dict, test_data_local_dict, device, args=None) -> bool:
        return False

    # ---- accounting (reference model_trainer.py:39-53) ----
    def _dataset_name(self):
        return getattr(self.args, "dataset", "ABCD") if self.args is not None else "ABCD"

    def count_training_flops_per_sample(self):
        from ..utils.flops import count_training_flops
        return count_training_flops(self.model, self._dataset_name())

    def count_full_flops_per_sample(self):
        from ..utils.flops import count_training_flops
        return count_training_flops(self.model, self._dataset_name(), full=True)

    def count_inference_flops(self, w):
        from ..utils.flops import count_inference_flops
        self.set_model_params(w)
        return count_inference_flops(self.model, self._dataset_name())

    @staticmethod
    def count_communication_params(update_to_server):
        """Number of non-zero entries in a state dict — the reference's only comm metric."""
        total = 0
        for v in update_to_server.values():
            if torch.is_tensor(v):
                total += int(torch.count_nonzero(v).item())
        return total
