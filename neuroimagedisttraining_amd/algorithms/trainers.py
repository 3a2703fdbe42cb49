"""Reference-semantics local trainers (torch eager; also the numerics oracle for the engine).

``VolumeTrainer`` reproduces ``sailentgrads/my_model_trainer.py:201-274`` /
``fedavg/my_model_trainer.py:85-183``:

* optimiser rebuilt every call: ``SGD(lr * lr_decay**round, momentum, weight_decay=wd)`` (Q4);
* ``BCEWithLogitsLoss`` on ``[B,1]`` logits, ``clip_grad_norm_(params, 10)`` every step;
* SalientGrads: after each ``optimizer.step()`` the *weights* are multiplied by the mask (Q2);
* eval: ``sigmoid`` then ``BCEWithLogitsLoss`` (double sigmoid, Q1 — ``args.fix_eval_loss``
  switches to the plain logit loss) and threshold 0.5; returns summed correct / loss·n / total.

Unlike the reference, batches are gathered from a device-resident :class:`VolumeStore` rather
than an HDF5 file re-opened per batch, the model never leaves the device between clients, masks
are kept on-device (no per-step H2D copy), and ``args.amp`` selects bf16 autocast.

``ClassificationTrainer`` is the 2D/tabular counterpart with ``CrossEntropyLoss`` used by the
CIFAR/Tiny-ImageNet baselines (SubAvg, Ditto, D-PSGD, FedFomo, Local) and the LR plumbing config.
"""
from __future__ import annotations

import copy
import logging

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..core.trainer import ModelTrainer

log = logging.getLogger(__name__)


def _amp_ctx(args, device):
    dt = getattr(args, "amp", None)
    if dt in (None, "", "none", "fp32", False):
        return torch.autocast(device_type="cpu", enabled=False)
    dtype = torch.bfloat16 if dt in ("bf16", True) else torch.float16
    dev = torch.device(device).type
    return torch.autocast(device_type=dev, dtype=dtype)


def unpack_batch(batch, device):
    """Turn a loader batch into ``(x, y)`` on ``device``.

    * volume loaders (``(index, y, site)`` with a VolumeStore) are resolved by the trainer,
    * plain ``(x, y)`` / ``(x, y, extra)`` tuples are moved to device."""
    x, y = batch[0], batch[1]
    return x.to(device, non_blocking=True), y.to(device, non_blocking=True)


class _TrainerBase(ModelTrainer):
    def __init__(self, model, args=None, logger=None):
        super().__init__(model, args)
        self.logger = logger or log
        self.offload = bool(getattr(args, "offload_params", False))

    # -- params -----------------------------------------------------------------------
    def get_model_params(self):
        sd = self.model.state_dict()
        if self.offload:
            return {k: v.detach().cpu().clone() for k, v in sd.items()}
        return {k: v.detach().clone() for k, v in sd.items()}

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def get_trainable_params(self):
        return {n: p for n, p in self.model.named_parameters()}

    def get_model_sps(self):
        """Percentage of zero entries among all parameters (``my_model_trainer.py:144-158``)."""
        nz = tot = 0
        for _, p in self.model.named_parameters():
            nz += int(torch.count_nonzero(p.detach()).item())
            tot += p.numel()
        return 100.0 * (tot - nz) / max(1, tot)

    def _xy(self, batch, loader, device):
        store = getattr(loader, "store", None)
        if store is not None:
            x, y = store.fetch(batch[0], device=device)
            return x, y
        return unpack_batch(batch, device)

    def _optimizer(self, args, round_idx):
        lr = args.lr * (args.lr_decay ** round_idx)
        params = [p for p in self.model.parameters() if p.requires_grad]
        if getattr(args, "client_optimizer", "sgd") == "sgd":
            return torch.optim.SGD(params, lr=lr, momentum=args.momentum, weight_decay=args.wd)
        return torch.optim.Adam(params, lr=lr, weight_decay=args.wd, amsgrad=True)


class VolumeTrainer(_TrainerBase):
    """Binary-logit (``class_num=1``) 3D-CNN trainer with optional SalientGrads mask."""

    def _loss_targets(self, logits, y):
        if logits.dim() == 2 and logits.shape[1] == 1:
            return logits, y.view(-1, 1).float()
        return logits, y.long()

    def _criterion(self, logits):
        return nn.BCEWithLogitsLoss() if (logits.dim() == 2 and logits.shape[1] == 1) else nn.CrossEntropyLoss()

    def train(self, train_data, device, args, round_idx=0, masks=None, prox_ref=None, mask_mode="weight",
              epoch_hook=None, epochs=None, prox_lamda=None):
        """``mask_mode``: "weight" multiplies weights by the mask after each step (SalientGrads / DisPFL),
        "grad" multiplies gradients before the step (SubAvg).  ``epoch_hook(epoch)`` runs after every epoch.
        ``prox_lamda`` + ``prox_ref``: Ditto's proximal pull w -= lr*lamda*(w - w_ref) after each step."""
        model = self.model
        model.to(device)
        model.train()
        opt = self._optimizer(args, round_idx)
        use_mask = masks is not None and (mask_mode != "weight" or bool(getattr(args, "snip_mask", True)))
        dev_masks = None
        if use_mask:
            dev_masks = {n: masks[n].to(device) for n, _ in model.named_parameters() if n in masks}
        mu = float(getattr(args, "fedprox_mu", 0.0) or 0.0)
        named = dict(model.named_parameters())
        epoch_losses = []
        lr_now = opt.param_groups[0]["lr"]
        for epoch in range(args.epochs if epochs is None else epochs):
            losses = []
            for batch in train_data:
                x, y = self._xy(batch, train_data, device)
                model.zero_grad(set_to_none=True)
                with _amp_ctx(args, device):
                    out = model(x)
                    out = out[0] if isinstance(out, (list, tuple)) else out
                logits, t = self._loss_targets(out.float(), y)
                loss = self._criterion(logits)(logits, t)
                if mu > 0 and prox_ref is not None:
                    # FedProx proximal term mu/2 ||w - w_global||^2 (new; absent in the reference)
                    prox = sum(((named[k] - prox_ref[k].to(device)) ** 2).sum() for k in named if k in prox_ref)
                    loss = loss + 0.5 * mu * prox
                loss.backward()
                if use_mask and mask_mode == "grad":
                    for n, p in named.items():
                        m = dev_masks.get(n)
                        if m is not None and p.grad is not None:
                            p.grad.mul_(m)
                torch.nn.utils.clip_grad_norm_(model.parameters(), 10)
                opt.step()
                losses.append(loss.detach())
                if prox_lamda is not None and prox_ref is not None:
                    with torch.no_grad():
                        for n, p in named.items():
                            if n in prox_ref:
                                p.sub_(lr_now * prox_lamda * (p - prox_ref[n].to(p.device)))
                if use_mask and mask_mode == "weight":
                    with torch.no_grad():
                        for n, p in named.items():
                            m = dev_masks.get(n)
                            if m is not None:
                                p.mul_(m)
            ep = torch.stack(losses).mean().item() if losses else float("nan")
            epoch_losses.append(ep)
            self.logger.info("Client Index = %s\tEpoch: %d\tLoss: %.6f", self.id, epoch, ep)
            if epoch_hook is not None:
                epoch_hook(epoch)
        return epoch_losses

    def screen_gradients(self, train_data, device):
        """Full (unmasked) gradient on one batch, model in eval mode (``DisPFL/my_model_trainer.py:166-189``)."""
        model = self.model
        model.to(device)
        model.eval()
        model.zero_grad()
        batch = next(iter(train_data))
        x, y = self._xy(batch, train_data, device)
        out = model(x)
        out = out[0] if isinstance(out, (list, tuple)) else out
        logits, t = self._loss_targets(out.float(), y)
        self._criterion(logits)(logits, t).backward()
        return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}

    @torch.no_grad()
    def test(self, test_data, device, args):
        model = self.model
        model.to(device)
        model.eval()
        correct = torch.zeros((), device=device)
        loss_sum = torch.zeros((), device=device)
        total = 0
        fix = bool(getattr(args, "fix_eval_loss", False))
        for batch in test_data:
            x, y = self._xy(batch, test_data, device)
            with _amp_ctx(args, device):
                out = model(x)
                out = out[0] if isinstance(out, (list, tuple)) else out
            out = out.float()
            if out.dim() == 2 and out.shape[1] == 1:
                prob = torch.sigmoid(out)
                loss = F.binary_cross_entropy_with_logits(out if fix else prob, y.view(-1, 1).float())
                pred = (prob >= 0.5).float().squeeze(1)
                correct += (pred == y.float()).float().sum()
            else:
                loss = F.cross_entropy(out, y.long())
                correct += (out.argmax(1) == y.long()).float().sum()
            loss_sum += loss * y.shape[0]
            total += int(y.shape[0])
        return {"test_correct": correct.item(), "test_loss": loss_sum.item(), "test_total": total,
                "test_acc": correct.item() / max(1, total)}


class ClassificationTrainer(VolumeTrainer):
    """CrossEntropy trainer for multi-class image / tabular data (same loop as VolumeTrainer;
    loss chosen from the logit width)."""

    def __init__(self, model, args=None, logger=None, grad_masks=False):
        super().__init__(model, args, logger)
        self.grad_masks = grad_masks


def clone_state(sd):
    return {k: v.detach().clone() for k, v in sd.items()}


def deepcopy_state(sd):
    return copy.deepcopy(sd)
