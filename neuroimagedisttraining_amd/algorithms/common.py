"""Shared FL-simulation pieces: client wrapper, sampling, aggregation, evaluation, stats.

Reference behaviours reproduced (SURVEY.md §2.2 "Shared algorithm behaviors"):
* sampling: all clients when ``total == per_round`` else ``np.random.seed(round);
  np.random.choice(total, per_round, replace=False)`` (``sailentgrads_api.py:152-160``);
* aggregation: ``n_i / sum n`` weights over **every** state-dict key incl. BN running stats and
  ``num_batches_tracked`` (Q3, ``sailentgrads_api.py:212-227``);
* evaluation: unweighted mean over clients of ``correct_i/total_i`` and ``loss_i/total_i`` (Q5);
  ``--ci 1`` evaluates one client and averages over the clients actually evaluated (fixes the
  reference's IndexError).
"""
from __future__ import annotations

import copy
import functools
import logging

import numpy as np
import torch

log = logging.getLogger(__name__)


def client_sampling(round_idx, client_num_in_total, client_num_per_round):
    if client_num_in_total == client_num_per_round:
        return list(range(client_num_in_total))
    # at least one client: int(total * frac) is 0 for small federations with the reference's default frac 0.1,
    # where the reference aggregates an empty list and crashes (the identity string keeps the reference's count)
    n = max(1, min(client_num_per_round, client_num_in_total))
    np.random.seed(round_idx)
    return list(np.random.choice(range(client_num_in_total), n, replace=False))


def weighted_average(w_locals):
    """``w_locals``: list of ``(n_samples, state_dict)`` -> sample-weighted average (all keys)."""
    total = float(sum(n for n, _ in w_locals))
    out = {}
    keys = list(w_locals[0][1].keys())
    for k in keys:
        acc = None
        for n, sd in w_locals:
            t = sd[k].float() * (n / total) if not sd[k].is_floating_point() else sd[k] * (n / total)
            acc = t.clone() if acc is None else acc.add_(t)
        out[k] = acc
    return out


def uniform_average(states):
    return weighted_average([(1, s) for s in states])


def state_to_device(sd, device):
    return {k: v.to(device) for k, v in sd.items()}


def model_sparsity(sd):
    """Percent zeros over non-mask entries (``sailentgrads_api.py:68-83``)."""
    nz = tot = 0
    for k, v in sd.items():
        if "mask" in k:
            continue
        nz += int(torch.count_nonzero(v).item())
        tot += v.numel()
    return 100.0 * (tot - nz) / max(1, tot)


class Client:
    """Per-client wrapper around the shared trainer (``sailentgrads/client.py:14-119``)."""

    def __init__(self, client_idx, local_training_data, local_test_data, local_sample_number, args, device,
                 model_trainer, logger=None, local_val_data=None):
        self.client_idx = client_idx
        self.local_training_data = local_training_data
        self.local_test_data = local_test_data
        self.local_val_data = local_val_data
        self.local_sample_number = local_sample_number
        self.args = args
        self.device = device
        self.model_trainer = model_trainer
        self.logger = logger or log

    def update_local_dataset(self, client_idx, local_training_data, local_test_data, local_sample_number):
        self.client_idx = client_idx
        self.local_training_data = local_training_data
        self.local_test_data = local_test_data
        self.local_sample_number = local_sample_number

    def get_sample_number(self):
        return self.local_sample_number

    def train(self, w_global, round_idx=0, masks=None, **kw):
        comm = self.model_trainer.count_communication_params(w_global)
        self.model_trainer.set_model_params(w_global)
        self.model_trainer.set_id(self.client_idx)
        self.model_trainer.train(self.local_training_data, self.device, self.args, round_idx, masks, **kw)
        weights = self.model_trainer.get_model_params()
        flops = self.args.epochs * self.local_sample_number
        comm += self.model_trainer.count_communication_params(weights)
        self.logger.info("communication parameters for search %d", comm)
        return weights, flops, comm

    def local_test(self, w, b_use_test_dataset=True):
        data = self.local_test_data if b_use_test_dataset else self.local_training_data
        self.model_trainer.set_model_params(w)
        return self.model_trainer.test(data, self.device, self.args)

    def val_test(self, w):
        self.model_trainer.set_model_params(w)
        return self.model_trainer.test(self.local_val_data, self.device, self.args)


def summarize(metrics_list):
    acc = float(np.mean([m["test_correct"] / max(1, m["test_total"]) for m in metrics_list]))
    loss = float(np.mean([m["test_loss"] / max(1, m["test_total"]) for m in metrics_list]))
    return acc, loss


def init_stat_info(class_counts=None):
    return {
        "label_num": class_counts, "sum_comm_params": 0, "sum_training_flops": 0, "avg_inference_flops": 0,
        "old_mask_test_acc": [], "new_mask_test_acc": [], "final_masks": [], "mask_dis_matrix": [],
        "global_test_acc": [], "person_test_acc": [], "round_time_s": [],
    }


class APIBase:
    """Common constructor: unpacks the dataset 8/9-tuple and builds one Client per client.

    ``train()`` of every subclass first offers the run to the client-batched MI355X executor
    (``algorithms/hip_dispatch.py``: a GPU device, the built extension and a supported model / data layout); the
    eager, sequential-client loop of the subclass is the fallback and the test oracle (``args.engine = "torch"``
    or ``NIDT_API_ENGINE=torch`` forces it).  ``engine_used`` says which one ran."""

    engine_used = None

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if "train" not in cls.__dict__:
            return
        eager = cls.__dict__["train"]

        @functools.wraps(eager)
        def train(self, *a, **k):
            if not getattr(self, "_hip_offered", False):
                self._hip_offered = True
                from .hip_dispatch import try_train_on_hip
                if try_train_on_hip(self):
                    return None
                self.engine_used = "eager"
            return eager(self, *a, **k)

        cls.train = train

    def record_avg_inference_flops(self, w_global, mask_pers=None):
        """Mean over clients of the sparse-aware inference FLOPs of ``w_global`` (under each client's personal
        mask when given) — ``subavg_api.py:223-235``; counted with the trainer's forward-hook counter."""
        tr = self.model_trainer
        keep = tr.get_model_params()
        flops = []
        for c in range(self.args.client_num_in_total):
            if mask_pers is None:
                w = w_global
            else:
                w = {k: (v * mask_pers[c][k].to(v.device) if k in mask_pers[c] else v) for k, v in w_global.items()}
            flops.append(tr.count_inference_flops(w))
            if mask_pers is None:  # the same model for every client
                flops = flops * self.args.client_num_in_total
                break
        tr.set_model_params(keep)
        self.stat_info["avg_inference_flops"] = float(sum(flops) / len(flops))
        return self.stat_info["avg_inference_flops"]

    def __init__(self, dataset, device, args, model_trainer, logger=None):
        self.logger = logger or log
        self.device = device
        self.args = args
        if len(dataset) > 8:  # 9-tuple of the val loaders: (..., num, train, val, test, class_num)
            (self.train_data_num_in_total, self.test_data_num_in_total, self.train_global, self.test_global,
             self.train_data_local_num_dict, self.train_data_local_dict, self.val_data_local_dict,
             self.test_data_local_dict, self.class_counts) = dataset[:9]
        else:
            (self.train_data_num_in_total, self.test_data_num_in_total, self.train_global, self.test_global,
             self.train_data_local_num_dict, self.train_data_local_dict, self.test_data_local_dict,
             self.class_counts) = dataset[:8]
            self.val_data_local_dict = None
        self.model_trainer = model_trainer
        self.client_list = []
        self._setup_clients()
        self.stat_info = init_stat_info(self.class_counts)

    def _setup_clients(self):
        self.logger.info("############setup_clients (START)#############")
        for c in range(self.args.client_num_in_total):
            self.client_list.append(Client(
                c, self.train_data_local_dict[c], self.test_data_local_dict[c],
                self.train_data_local_num_dict[c], self.args, self.device, self.model_trainer, self.logger,
                None if self.val_data_local_dict is None else self.val_data_local_dict[c]))
        self.logger.info("############setup_clients (END)#############")

    def _client_sampling(self, round_idx, total, per_round):
        idx = client_sampling(round_idx, total, per_round)
        self.logger.info("client_indexes = %s", str(idx))
        return idx

    def _aggregate(self, w_locals):
        return weighted_average(w_locals)

    def _eval_clients(self, w_of_client, tag):
        ms = []
        for c in range(self.args.client_num_in_total):
            ms.append(self.client_list[c].local_test(w_of_client(c), True))
            if getattr(self.args, "ci", 0) == 1:
                break
        return summarize(ms)

    def _test_on_all_clients(self, w_global, w_per_mdls, round_idx):
        self.logger.info("################global_test_on_all_clients : %s", round_idx)
        g_acc, g_loss = self._eval_clients(lambda c: w_global, "global")
        p_acc, p_loss = self._eval_clients(lambda c: w_per_mdls[c], "person")
        self.stat_info["global_test_acc"].append(g_acc)
        self.stat_info["person_test_acc"].append(p_acc)
        self.logger.info({"global_test_acc": g_acc, "global_test_loss": g_loss})
        self.logger.info({"person_test_acc": p_acc, "person_test_loss": p_loss})
        return g_acc, p_acc

    def _local_test_on_all_clients(self, w_per_mdls, round_idx, key="old_mask_test_acc"):
        self.logger.info("################local_test_on_all_clients after local training in communication round: %s",
                         round_idx)
        acc, loss = self._eval_clients(lambda c: w_per_mdls[c], "local")
        self.stat_info[key].append(acc)
        self.logger.info({"test_acc": acc, "test_loss": loss})
        return acc


def deepcopy(x):
    return copy.deepcopy(x)
