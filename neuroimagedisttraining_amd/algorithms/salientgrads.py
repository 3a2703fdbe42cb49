"""SalientGrads (reference ``fedml_api/standalone/sailentgrads/sailentgrads_api.py:18-348``).

1. every client computes SNIP saliency averaged over ``itersnip_iteration`` random mini-batches;
2. the server averages across clients, takes a global top-k at ``dense_ratio`` -> one mask;
3. per round, sampled clients train from ``w_global`` with the fixed mask (weights re-masked after
   each step), then sample-weighted FedAvg over all keys;
4. every round: global model and each client's last local ("personalized") model are evaluated
   on every client's test split.

This is the torch-eager, sequential-client implementation with reference semantics (and the
test oracle).  The production path — all clients of a GPU training in lockstep on HIP kernels,
RCCL aggregation across GPUs — is :class:`neuroimagedisttraining_amd.engine.runner.FLRunner`.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .common import APIBase, model_sparsity
from . import snip as S


def _dataset_tensors(ds):
    """(inputs, labels) tensors behind a TensorDataset / AugmentedTensorDataset (un-augmented); other datasets
    fall back to item access."""
    if hasattr(ds, "tensors"):
        return ds.tensors[0], ds.tensors[1]
    if hasattr(ds, "x") and hasattr(ds, "y"):
        return ds.x, ds.y
    items = [ds[i] for i in range(len(ds))]
    return (torch.stack([torch.as_tensor(a) for a, _ in items]),
            torch.as_tensor(np.asarray([np.asarray(b).reshape(-1)[0] for _, b in items])))


class SailentGradsAPI(APIBase):

    def generate_global_mask_snip(self):
        per_client = []
        for c in range(self.args.client_num_in_total):
            per_client.append(self.client_score(c))
        self.logger.info("@@@@@Aggregate the local masks@@@@@@@@@@@@@@@@@@@")
        avg = S.mean_scores(per_client)
        _, final = S.mask_from_scores(self.model_trainer.model, avg, self.args.dense_ratio)
        return final

    def client_score(self, c):
        """IterSNIP scores of client ``c`` (``sailentgrads/client.py:30-53``): the mean over
        ``itersnip_iteration`` mini-batches of ``|w * dL/dw|``.  Each iteration takes the first batch of a fresh
        shuffle, or with ``--stratified_sampling`` a label-stratified batch (:func:`snip.stratified_batch`, the
        same draw as the client-batched runner's, so both paths select the same global mask)."""
        client = self.client_list[c]
        loader = client.local_training_data
        iters = int(getattr(self.args, "itersnip_iteration", 1))
        stratified = bool(getattr(self.args, "stratified_sampling", False))
        scores = []
        for it in range(iters):
            if stratified:
                x, y = self._stratified_xy(c, loader, it)
            else:
                batch = next(iter(loader))
                x, y = self.model_trainer._xy(batch, loader, self.device)
            scores.append(S.snip_scores(self.model_trainer.model.to(self.device), x, y))
        return S.mean_scores(scores)

    def _stratified_xy(self, c, loader, it):
        """(x, y) of the stratified IterSNIP batch of client ``c`` at iteration ``it``."""
        rng = S.stratified_rng(getattr(self.args, "seed", 0), c, it)
        B = int(getattr(loader, "batch_size", None) or self.args.batch_size)
        store = getattr(loader, "store", None)
        if store is not None and hasattr(loader, "indices"):  # ABCD IndexLoader: subject indices into a store
            idx = S.stratified_batch(loader.indices, loader._y, B, rng)
            return store.fetch(torch.from_numpy(idx.astype(np.float32)), device=self.device)
        # generic DataLoader: stratify over the positions of its dataset.  Labels and images are read from the
        # dataset's tensors, not through ds[i]: an augmenting dataset would run (and draw RNG for) a crop/flip per
        # access, shifting later randomness and feeding SNIP an augmented batch the client-batched runner never sees
        ds = loader.dataset
        xt, yt = _dataset_tensors(ds)
        ys = np.asarray(yt.reshape(len(ds), -1)[:, 0], dtype=np.float64)
        pos = S.stratified_batch(np.arange(len(ds)), ys, B, rng)
        ix = torch.as_tensor(np.asarray(pos, dtype=np.int64))
        return xt[ix].to(self.device), torch.as_tensor(yt)[ix].reshape(len(ix), -1)[:, 0].to(self.device)

    def train(self):
        mask = self.generate_global_mask_snip()
        if not getattr(self.args, "snip_mask", True):
            mask = {k: torch.ones_like(v) for k, v in mask.items()}  # Q6 "no mask" branch
        w_global = self.model_trainer.get_model_params()
        w_per_mdls = [dict(w_global) for _ in range(self.args.client_num_in_total)]
        self.mask = mask
        for round_idx in range(self.args.comm_round):
            t0 = time.perf_counter()
            self.logger.info("################Communication round : %d", round_idx)
            idx = np.sort(self._client_sampling(round_idx, self.args.client_num_in_total,
                                                self.args.client_num_per_round))
            w_locals = []
            for c in idx:
                self.logger.info("@@@@@@@@@@@@@@@@ Training Client CM(%d): %d", round_idx, c)
                client = self.client_list[c]
                w_per, flops, comm = client.train(w_global, round_idx, mask)
                w_per_mdls[c] = w_per
                w_locals.append((client.get_sample_number(), w_per))
                self.stat_info["sum_training_flops"] += flops
                self.stat_info["sum_comm_params"] += comm
            w_global = self._aggregate(w_locals)
            self.stat_info["global_sparsity"] = model_sparsity(w_global)
            if getattr(self.args, "frequency_of_the_test", 1) and (round_idx % max(1, self.args.frequency_of_the_test) == 0):
                self._test_on_all_clients(w_global, w_per_mdls, round_idx)
            self.stat_info["round_time_s"].append(time.perf_counter() - t0)
        self._test_on_all_clients(w_global, w_per_mdls, -1)
        self.w_global = w_global
        return w_global
