"""NAS training utilities (reference ``fedml_api/model/cv/darts/utils.py:1-100``)."""
from __future__ import annotations

import os
import shutil

import numpy as np
import torch


class AvgrageMeter:  # reference spelling kept for import compatibility
    def __init__(self):
        self.reset()

    def reset(self):
        self.avg = 0.0
        self.sum = 0.0
        self.cnt = 0

    def update(self, val, n=1):
        self.sum += float(val) * n
        self.cnt += n
        self.avg = self.sum / self.cnt


AverageMeter = AvgrageMeter


def accuracy(output, target, topk=(1,)):
    """Top-k accuracy in percent, one tensor per k."""
    maxk = max(topk)
    _, pred = output.topk(maxk, 1, True, True)
    hit = pred.t().eq(target.view(1, -1))
    return [hit[:k].reshape(-1).float().sum(0).mul_(100.0 / target.size(0)) for k in topk]


class Cutout:
    """Zero a random ``length x length`` square of a CHW image tensor (clipped at the border)."""

    def __init__(self, length, generator=None):
        self.length = length
        self.rng = generator or np.random

    def __call__(self, img):
        h, w = img.shape[-2:]
        y, x = self.rng.randint(h), self.rng.randint(w)
        y0, y1 = max(0, y - self.length // 2), min(h, y + self.length // 2)
        x0, x1 = max(0, x - self.length // 2), min(w, x + self.length // 2)
        img = img.clone()
        img[..., y0:y1, x0:x1] = 0
        return img


def count_parameters_in_MB(model):  # noqa: N802
    return sum(v.numel() for n, v in model.named_parameters() if "auxiliary" not in n) / 1e6


def save_checkpoint(state, is_best, save):
    os.makedirs(save, exist_ok=True)
    fn = os.path.join(save, "checkpoint.pth.tar")
    torch.save(state, fn)
    if is_best:
        shutil.copyfile(fn, os.path.join(save, "model_best.pth.tar"))


def save(model, model_path):
    torch.save(model.state_dict(), model_path)


def load(model, model_path):
    model.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True))


def drop_path(x, drop_prob, generator=None):
    """Per-sample path dropout (out of place, works on any device)."""
    if drop_prob <= 0.0:
        return x
    keep = 1.0 - drop_prob
    mask = torch.empty((x.size(0),) + (1,) * (x.dim() - 1), device=x.device, dtype=x.dtype)
    mask.bernoulli_(keep, generator=generator)
    return x * mask / keep


def create_exp_dir(path, scripts_to_save=None):
    os.makedirs(path, exist_ok=True)
    if scripts_to_save:
        d = os.path.join(path, "scripts")
        os.makedirs(d, exist_ok=True)
        for s in scripts_to_save:
            shutil.copyfile(s, os.path.join(d, os.path.basename(s)))
