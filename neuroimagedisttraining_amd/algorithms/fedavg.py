"""FedAvg and FedProx (reference ``fedml_api/standalone/fedavg/fedavg_api.py:40-173``).

Per round: sample clients, each trains from ``w_global``, sample-weighted average of all keys,
evaluate the global model and each client's personal (last local) model.  After the last round
every client runs one extra local "fine-tune" pass from ``w_global`` and a final evaluation
(``fedavg_api.py:78-88``).

FedProx (new; BASELINE.json config 4) is FedAvg with the proximal term ``mu/2 ||w - w_g||^2``
added to each local loss (``args.fedprox_mu``) and an optional robust aggregator
(``args.aggregator`` in {``fedavg``, ``krum``, ``multikrum``, ``median``, ``trimmed_mean``}).
"""
from __future__ import annotations

import time

import numpy as np

from .common import APIBase
from ..core import robustness as R


class FedAvgAPI(APIBase):

    def _aggregate(self, w_locals):
        kind = getattr(self.args, "aggregator", "fedavg") or "fedavg"
        if kind == "fedavg":
            return super()._aggregate(w_locals)
        return R.robust_aggregate(kind, w_locals, f=int(getattr(self.args, "byzantine_f", 0) or 0),
                                  trim_ratio=float(getattr(self.args, "trim_ratio", 0.1) or 0.1))

    def _local_kwargs(self, w_global):
        if float(getattr(self.args, "fedprox_mu", 0.0) or 0.0) > 0:
            return {"prox_ref": w_global}
        return {}

    def train(self):
        w_global = self.model_trainer.get_model_params()
        w_per_mdls = [dict(w_global) for _ in range(self.args.client_num_in_total)]
        for round_idx in range(self.args.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            idx = np.sort(self._client_sampling(round_idx, self.args.client_num_in_total,
                                                self.args.client_num_per_round))
            w_locals = []
            for c in idx:
                client = self.client_list[c]
                w, flops, comm = client.train(w_global, round_idx, None, **self._local_kwargs(w_global))
                w_per_mdls[c] = w
                w_locals.append((client.get_sample_number(), w))
                self.stat_info["sum_training_flops"] += flops
                self.stat_info["sum_comm_params"] += comm
            w_global = self._aggregate(w_locals)
            freq = max(1, int(getattr(self.args, "frequency_of_the_test", 1) or 1))
            if round_idx % freq == 0 or round_idx == self.args.comm_round - 1:
                self._test_on_all_clients(w_global, w_per_mdls, round_idx)
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        if getattr(self.args, "final_finetune", True):
            for c in range(self.args.client_num_in_total):
                w, _, _ = self.client_list[c].train(w_global, self.args.comm_round, None)
                w_per_mdls[c] = w
            self._test_on_all_clients(w_global, w_per_mdls, -1)
        self.w_global = w_global
        return w_global


class FedProxAPI(FedAvgAPI):
    """FedAvg with a proximal local objective; ``args.fedprox_mu`` defaults to 0.01."""

    def __init__(self, dataset, device, args, model_trainer, logger=None):
        if not getattr(args, "fedprox_mu", 0):
            args.fedprox_mu = 0.01
        super().__init__(dataset, device, args, model_trainer, logger)
