"""Personalized / decentralised FL baselines of the reference harness, reference semantics (torch eager).

* :class:`DisPFLAPI`  — ``DisPFL/dispfl_api.py:46-301``, ``DisPFL/client.py:32-99``: per-client sparse masks (ERK or
  uniform), masked local training, cosine-annealed fire (smallest |w|) + regrow (top |g| or random), client
  dropout ``--active``, mask Hamming bookkeeping.  The reference has neighbour aggregation commented out
  (quirk Q10), so by default each client continues its own model; ``--dispfl_aggregate 1`` enables the
  DisPFL paper's masked neighbour averaging.
* :class:`SubAvgAPI`  — ``subavg/subavg_api.py:43-221``: gradient-masked training, ``fake_prune`` at the first and
  last epoch, prune when the mask moved (> ``dist_thresh``), density > ``dense_ratio`` and the pruned model's
  local accuracy > ``acc_thresh``; server averages each coordinate over the clients keeping it.
* :class:`DittoAPI`   — ``ditto/ditto_api.py:40-105``: FedAvg global model + personal models trained with a
  proximal pull ``w -= lr * lamda * (w - w_global)`` for ``local_epochs``; evaluation on personal models.
* :class:`DPSGDAPI`   — ``dpsgd/dpsgd_api.py:41-178``: every client averages its neighbours (ring/random/full) then
  trains; the global mean is used for evaluation.
* :class:`FedFomoAPI` — ``fedfomo/fedfomo_api.py:53-217``: validation-loss-improvement-per-distance neighbour
  weights, 50 % argmax-affinity / 50 % random neighbour choice.
* :class:`LocalAPI`   — ``local/local_api.py:51-84``: local-only training.
"""
from __future__ import annotations

import copy
import time

import numpy as np
import torch

from .common import APIBase, client_sampling, summarize, weighted_average, uniform_average
from . import sparse as SP


# ------------------------------------------------------------------------------------------------ DisPFL
class DisPFLAPI(APIBase):

    def _benefit_choose(self, round_idx, cur_clnt, total, per_round, dist_local=None, total_dist=None, cs=None,
                        active=None):
        if total == per_round:
            return np.array(list(range(total)))
        # the reference forces cs = "random" (dispfl_api.py:201) and draws from the (global) numpy stream
        k = min(per_round, total)
        idx = self.np_rng.choice(range(total), k, replace=False)
        while cur_clnt in idx:
            idx = self.np_rng.choice(range(total), k, replace=False)
        return idx

    def _aggregate_func(self, clnt, nei, w_per_mdls, masks):
        """Masked neighbour average (used only with ``dispfl_aggregate``)."""
        idx = list(nei) + [clnt]
        out = copy.deepcopy(w_per_mdls[clnt])
        for k in out:
            if k in masks[clnt]:
                num = sum(w_per_mdls[i][k] * masks[i][k].to(out[k].device) for i in idx)
                cnt = sum(masks[i][k].to(out[k].device) for i in idx)
                avg = num / cnt.clamp_min(1)
                out[k] = torch.where(cnt > 0, avg, out[k]) * masks[clnt][k].to(out[k].device)
            else:
                out[k] = sum(w_per_mdls[i][k].float() for i in idx) / len(idx)
        return out

    def train(self):
        a = self.args
        tr = self.model_trainer
        # masks cover every named parameter (get_trainable_params, DisPFL/my_model_trainer.py:125-129)
        params = {n: p.detach().cpu() for n, p in tr.model.named_parameters()}
        N = a.client_num_in_total
        self.np_rng = np.random.RandomState(getattr(a, "seed", 0))
        gen = torch.Generator().manual_seed(getattr(a, "seed", 0) + 17)  # mask init stream (same as the executor's DisPFLRunner)
        dense = [a.dense_ratio] * N
        dist = "uniform" if getattr(a, "uniform", False) else "ERK"
        eps = getattr(a, "erk_power_scale", 1.0)
        sp = SP.erk_sparsities(params, a.dense_ratio, erk_power_scale=eps, distribution=dist)
        if not getattr(a, "different_initial", False):
            base = SP.init_masks(params, sp, generator=gen)
            masks = [SP.copy_masks(base) for _ in range(N)]
        elif not getattr(a, "diff_spa", False):
            masks = [SP.init_masks(params, sp, generator=gen) for _ in range(N)]
        else:
            p_divide = [0.2, 0.4, 0.6, 0.8, 1.0]
            masks = []
            for i in range(N):
                dense[i] = p_divide[i % 5]
                masks.append(SP.init_masks(params, SP.erk_sparsities(params, dense[i], erk_power_scale=eps,
                                                                     distribution=dist), generator=gen))
        dev = next(tr.model.parameters()).device
        masks = [{k: v.to(dev) for k, v in m.items()} for m in masks]
        w_global = tr.get_model_params()
        w_per = []
        for c in range(N):
            w = copy.deepcopy(w_global)
            for n in masks[c]:
                w[n] = w_global[n] * masks[c][n].to(w_global[n].device)
            w_per.append(w)
        shared = [SP.copy_masks(m) for m in masks]
        dist_locals = np.zeros((N, N))
        agg = bool(getattr(a, "dispfl_aggregate", False))
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            active = self.np_rng.choice([0, 1], size=N, p=[1.0 - a.active, a.active])
            w_last = copy.deepcopy(w_per)
            shared_last = [SP.copy_masks(m) for m in shared]
            after, before = [], []
            for c in range(N):
                d, tot = SP.hamming_distance(shared_last[c], masks[c])
                dist_locals[c][c] = d
                nei = np.array([], dtype=int) if active[c] == 0 else self._benefit_choose(
                    round_idx, c, N, a.client_num_per_round, dist_locals[c], tot, a.cs, active)
                if N != a.client_num_per_round:
                    nei = np.append(nei, c)
                nei = np.sort(nei).astype(int)
                for j in nei:
                    if int(j) != c:
                        dist_locals[c][int(j)], _ = SP.hamming_distance(masks[c], shared_last[int(j)])
                w_local = self._aggregate_func(c, [int(j) for j in nei], w_last, shared_last) if (agg and len(nei)
                                                                                                  and active[c]) \
                    else copy.deepcopy(w_last[c])
                shared[c] = SP.copy_masks(masks[c])
                client = self.client_list[c]
                before.append(client.local_test(w_local, True))
                comm = tr.count_communication_params(w_local)
                tr.set_model_params(w_local)
                tr.set_id(c)
                tr.train(client.local_training_data, self.device, a, round_idx, masks[c], mask_mode="weight")
                w_new = tr.get_model_params()
                after.append(tr.test(client.local_test_data, self.device, a))
                update = {k: w_new[k] - w_local[k] for k in w_new}
                if not getattr(a, "static", False):
                    grad = None if getattr(a, "dis_gradient_check", False) else \
                        tr.screen_gradients(client.local_training_data, self.device)
                    if grad is not None:
                        grad = {k: v.to(dev) for k, v in grad.items()}
                    new_m, num_remove = SP.fire_mask(masks[c], w_new, round_idx, a.anneal_factor, a.comm_round)
                    masks[c] = SP.regrow_mask(new_m, num_remove, grad)
                w_per[c] = w_new
                self.stat_info["sum_comm_params"] += comm + tr.count_communication_params(update)
                self.stat_info["sum_training_flops"] += a.epochs * client.get_sample_number()
            acc, loss = summarize(after)
            acc0, loss0 = summarize(before)
            self.stat_info["new_mask_test_acc"].append(acc)
            self.stat_info["old_mask_test_acc"].append(acc0)
            self.logger.info({"test_acc": acc, "test_loss": loss})
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        for i in range(N):
            self.stat_info["mask_dis_matrix"].append([SP.hamming_distance(masks[i], masks[j])[0] for j in range(N)])
        if getattr(a, "save_masks", False):
            self.stat_info["final_masks"] = [{k: v.bool() for k, v in m.items()} for m in masks]
        self.masks, self.w_per_mdls = masks, w_per
        return w_per


# ------------------------------------------------------------------------------------------------ SubAvg
class SubAvgAPI(APIBase):

    def record_mask_diffrence(self, mask_pers):
        n = len(mask_pers)
        if n < 2:
            return
        d = np.mean([SP.dist_masks(mask_pers[i], mask_pers[j]) for i in range(n) for j in range(n) if i != j])
        self.stat_info.setdefault("mask_diff", []).append(float(d))

    def train(self):
        a = self.args
        tr = self.model_trainer
        masks = {n: torch.ones_like(p).detach() for n, p in tr.model.named_parameters()}  # every parameter (init_masks)
        N = a.client_num_in_total
        mask_pers = [SP.copy_masks(masks) for _ in range(N)]
        w_global = tr.get_model_params()
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            if getattr(a, "record_mask_diff", False):
                self.record_mask_diffrence(mask_pers)
            idx = self._client_sampling(round_idx, N, a.client_num_per_round)
            w_locals, next_masks = [], []
            for c in idx:
                client = self.client_list[c]
                m_c = SP.copy_masks(mask_pers[c])
                w_c = SP.real_prune(copy.deepcopy(w_global), m_c)
                comm = tr.count_communication_params(w_c)
                tr.set_model_params(w_c)
                tr.set_id(c)
                dense, _ = SP.print_pruning({k: v for k, v in w_c.items() if k in m_c})
                pm = {}

                def hook(ep, pm=pm, m_c=m_c):
                    if ep == 0:
                        pm["m1"] = SP.fake_prune(a.each_prune_ratio, tr.get_model_params(), m_c)
                    if ep == a.epochs - 1:
                        pm["m2"] = SP.fake_prune(a.each_prune_ratio, tr.get_model_params(), m_c)
                tr.train(client.local_training_data, self.device, a, round_idx, m_c, mask_mode="grad",
                         epoch_hook=hook)
                state = tr.get_model_params()
                final = m_c
                if SP.dist_masks(pm["m1"], pm["m2"]) > a.dist_thresh and dense > a.dense_ratio:
                    tr.set_model_params(SP.real_prune(state, pm["m2"]))
                    met = tr.test(client.local_training_data, self.device, a)
                    if met["test_correct"] / max(1, met["test_total"]) > a.acc_thresh:
                        state = SP.real_prune(state, pm["m2"])
                        final = pm["m2"]
                w_locals.append((SP.copy_masks(mask_pers[c]), copy.deepcopy(state)))
                next_masks.append((c, final))
                self.stat_info["sum_comm_params"] += comm + tr.count_communication_params(state)
                self.stat_info["sum_training_flops"] += a.epochs * client.get_sample_number()
            w_global = SP.masked_average(w_global, w_locals)
            if round_idx == a.comm_round - 1 or round_idx % max(1, a.frequency_of_the_test) == 0:
                ms = [self.client_list[c].local_test(SP.real_prune(w_global, mask_pers[c]), True) for c in range(N)]
                acc, loss = summarize(ms)
                self.stat_info["old_mask_test_acc"].append(acc)
                self.logger.info({"test_acc": acc, "test_loss": loss})
            for c, m in next_masks:
                mask_pers[c] = m
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self.mask_pers, self.w_global = mask_pers, w_global
        self.record_avg_inference_flops(w_global, mask_pers)  # subavg_api.py:91
        return w_global


# ------------------------------------------------------------------------------------------------ Ditto
class DittoAPI(APIBase):

    def train(self):
        a = self.args
        tr = self.model_trainer
        N = a.client_num_in_total
        w_global = tr.get_model_params()
        w_per = [copy.deepcopy(w_global) for _ in range(N)]
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            idx = self._client_sampling(round_idx, N, a.client_num_per_round)
            w_locals = []
            for c in idx:
                client = self.client_list[c]
                comm = tr.count_communication_params(w_global)  # ditto/client.py:43-49 (downlink + uplink)
                tr.set_model_params(w_global)
                tr.set_id(c)
                tr.train(client.local_training_data, self.device, a, round_idx)
                w_locals.append((client.get_sample_number(), tr.get_model_params()))
                self.stat_info["sum_comm_params"] += int(comm + tr.count_communication_params(w_locals[-1][1]))
                # personal model: proximal pull towards the round's global model (ditto/my_model_trainer.py:38-68)
                tr.set_model_params(w_per[c])
                tr.train(client.local_training_data, self.device, a, round_idx, prox_ref=w_global,
                         prox_lamda=a.lamda, epochs=getattr(a, "local_epochs", a.epochs))
                w_per[c] = tr.get_model_params()
            w_global = weighted_average(w_locals)
            if round_idx == a.comm_round - 1 or round_idx % max(1, a.frequency_of_the_test) == 0:
                self._local_test_on_all_clients(w_per, round_idx, key="person_test_acc")
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self.w_global, self.w_per_mdls = w_global, w_per
        self.record_avg_inference_flops(w_global)  # ditto_api.py:78
        return w_per


# ------------------------------------------------------------------------------------------------ D-PSGD
class DPSGDAPI(APIBase):

    def _benefit_choose(self, round_idx, cur_clnt, total, per_round, cs="ring"):
        """Neighbourhood incl. the client itself (``dpsgd_api.py:116-139`` + the append in ``train``)."""
        if total == per_round:
            return list(range(total))
        if cs == "random":
            np.random.seed(round_idx + cur_clnt)
            idx = np.random.choice(range(total), min(per_round, total), replace=False)
            while cur_clnt in idx:
                idx = np.random.choice(range(total), min(per_round, total), replace=False)
            nei = list(idx)
        elif cs == "ring":
            nei = [(cur_clnt - 1 + total) % total, (cur_clnt + 1) % total]
        elif cs == "full":
            nei = [j for j in range(total) if j != cur_clnt]
        else:
            raise ValueError(cs)
        return sorted(int(j) for j in nei + [cur_clnt])

    def train(self):
        a = self.args
        tr = self.model_trainer
        N = a.client_num_in_total
        w_global = tr.get_model_params()
        w_per = [copy.deepcopy(w_global) for _ in range(N)]
        cs = getattr(a, "cs", "ring")
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            last = copy.deepcopy(w_per)
            for c in range(N):
                nei = self._benefit_choose(round_idx, c, N, a.client_num_per_round, cs)
                w_local = uniform_average([last[j] for j in nei])
                client = self.client_list[c]
                tr.set_model_params(w_local)
                tr.set_id(c)
                tr.train(client.local_training_data, self.device, a, round_idx)
                w_per[c] = tr.get_model_params()
            w_global = uniform_average(w_per)
            self._test_on_all_clients(w_global, w_per, round_idx)
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self.w_global, self.w_per_mdls = w_global, w_per
        return w_global


# ------------------------------------------------------------------------------------------------ FedFomo
class FedFomoAPI(APIBase):
    """Reference ``fedfomo_api.py:53-217``: train from the last model, choose neighbours (argsort of the affinity
    ``p_choose`` half of the time, random otherwise), weigh them by validation-loss improvement per unit distance
    (the client's own freshly trained model stands in for itself), move to the weighted combination."""

    def _benefit_choose(self, round_idx, cur_clnt, total, per_round, p_choose):
        if total == per_round:
            return list(range(total))
        p_choose[cur_clnt] = 0
        if self.py_rng.random() >= 0.5:
            idx = np.argsort(p_choose)[-per_round:]
        else:
            idx = self.np_rng.choice(range(total), per_round, replace=False)
            while cur_clnt in idx:
                idx = self.np_rng.choice(range(total), per_round, replace=False)
        return sorted(int(j) for j in list(idx) + [cur_clnt])

    def _val(self, c, w):
        client = self.client_list[c]
        m = client.val_test(w) if client.local_val_data is not None else client.local_test(w, False)
        return m["test_loss"]

    def _updates_weight_local(self, c, nei, last, weight_local, w_new):
        loss_cur = self._val(c, last[c])
        for j in nei:
            src = w_new if j == c else last[j]
            lj = self._val(c, src)
            d = np.sqrt(max(SP.model_difference({k: v.float() for k, v in src.items()},
                                                {k: v.float() for k, v in last[c].items()}), 0.0))
            weight_local[j] = 0.0 if d == 0 else (loss_cur - lj) / d
        return weight_local

    def _aggregate_func(self, c, nei, last, weights, w_new):
        wpos = np.maximum(weights[nei], 0)
        tot = float(np.sum(wpos))
        if tot == 0.0:
            return copy.deepcopy(last[c])
        out = {}
        for k, v in last[c].items():
            acc = v.float().clone()
            for j, wj in zip(nei, wpos):
                src = w_new if j == c else last[j]
                acc += (src[k].float() - v.float()) * (wj / tot)
            out[k] = acc.to(v.dtype) if v.is_floating_point() else acc.round().to(v.dtype)  # fixes quirk Q12
        return out

    def train(self):
        import random
        a = self.args
        tr = self.model_trainer
        N = a.client_num_in_total
        self.np_rng = np.random.RandomState(getattr(a, "seed", 0))
        self.py_rng = random.Random(getattr(a, "seed", 0))
        w_global = tr.get_model_params()
        w_per = [copy.deepcopy(w_global) for _ in range(N)]
        weights_locals = np.full((N, N), 1.0 / N)
        p_choose = np.ones((N, N))
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            last = copy.deepcopy(w_per)
            after_train, after_agg = [], []
            for c in range(N):
                client = self.client_list[c]
                tr.set_model_params(last[c])
                tr.set_id(c)
                tr.train(client.local_training_data, self.device, a, round_idx)
                w_new = tr.get_model_params()
                after_train.append(tr.test(client.local_test_data, self.device, a))
                nei = self._benefit_choose(round_idx, c, N, a.client_num_per_round, p_choose[c])
                weights_locals[c] = self._updates_weight_local(c, nei, last, weights_locals[c].copy(), w_new)
                p_choose[c] = p_choose[c] + weights_locals[c]
                w_per[c] = self._aggregate_func(c, nei, last, weights_locals[c], w_new)
                after_agg.append(client.local_test(w_per[c], True))
            acc0, _ = summarize(after_train)
            acc, loss = summarize(after_agg)
            self.stat_info["old_mask_test_acc"].append(acc0)
            self.stat_info["person_test_acc"].append(acc)
            self.logger.info({"test_acc": acc, "test_loss": loss})
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self.w_per_mdls = w_per
        return w_per


# ------------------------------------------------------------------------------------------------ Local
class LocalAPI(APIBase):

    def train(self):
        a = self.args
        tr = self.model_trainer
        N = a.client_num_in_total
        w0 = tr.get_model_params()
        w_per = [copy.deepcopy(w0) for _ in range(N)]
        for round_idx in range(a.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            for c in range(N):
                client = self.client_list[c]
                tr.set_model_params(w_per[c])
                tr.set_id(c)
                tr.train(client.local_training_data, self.device, a, round_idx)
                w_per[c] = tr.get_model_params()
            if round_idx == a.comm_round - 1 or round_idx % max(1, a.frequency_of_the_test) == 0:
                # per-client accuracy = correct/total (the reference accumulates test_acc across batches, Q14)
                self._local_test_on_all_clients(w_per, round_idx, key="person_test_acc")
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self.w_per_mdls = w_per
        return w_per
