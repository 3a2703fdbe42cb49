"""Client-batched engine for the remaining 2-D image models of the reference's entry points.

``main_subavg.py:143-158`` (and the other standalone mains) select ``lenet5``, ``cnn_cifar10``, ``cnn_cifar100`` and
``vgg11`` besides ``resnet18``.  ResNet-18-GN has its own hand-written kernel engine (``resnet2d_hip.py``); these
smaller models run here on the same :class:`~.runner.FLRunner` (every algorithm, lockstep rows, RCCL collectives)
with the forward/backward of all G clients of a lockstep step as ONE batched launch sequence: ``torch.func.vmap``
over the client axis of the parameter rows, so each conv / linear layer is a single grouped MIOpen / hipBLASLt call
for the whole group instead of G sequential per-client passes (``TorchEngine``).  The optimizer step and the SNIP
saliency accumulation are the fused HIP kernels of the other engines (``optim.hip``) on the GPU, their torch twins
on the CPU.

Inputs follow the reference image loaders (``cifar10/data_loader.py:46-52``): uint8 HWC images, train-time
RandomCrop(S, padding=4) + RandomHorizontalFlip drawn per (step seed, client id, batch position) with the same
counter-based hash as the ResNet engine's fused input stage (``img.hip``), computed on the device (no host sync per
step), then ``Normalize(mean, std)``.  Compute is bf16 autocast on the GPU (fp32 master rows), fp32 on the CPU.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import os

from .flat import ParamLayout
from .resnet2d_hip import AUG_PAD

_M64 = (1 << 64) - 1


def _s64(v):
    """uint64 constant as the int64 two's-complement value torch arithmetic wraps with."""
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


_K0, _K1, _K2 = _s64(0x9e3779b97f4a7c15), _s64(0xbf58476d1ce4e5b9), _s64(0x94d049bb133111eb)


def _lsr(z, s):
    """Logical right shift of int64 tensors holding uint64 bit patterns."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def mix64_t(seed, a, b):
    """Tensor twin of ``resnet2d_hip.mix64`` / ``img.hip`` (int64 tensors, uint64 semantics by wrap-around)."""
    z = seed ^ (_K0 * (((a & 0xffffffff) << 32) ^ b))
    z = (z ^ _lsr(z, 30)) * _K1
    z = (z ^ _lsr(z, 27)) * _K2
    return z ^ _lsr(z, 31)


def aug_draws_t(seed, cids, B, pad=AUG_PAD):
    """Device draws of :func:`~.resnet2d_hip.aug_draws`: ``seed`` an int64 scalar tensor, ``cids`` int64 [G];
    returns (oy, ox, flip) int64 [G * B]."""
    span = 2 * pad + 1
    j = torch.arange(B, device=cids.device, dtype=torch.int64)
    h = mix64_t(seed.view(1, 1), cids.view(-1, 1), j.view(1, -1)).reshape(-1)
    lo, hi = h & 0xffffffff, _lsr(h, 32)
    return lo % span, (lo // span) % span, hi & 1


def augment_batch(img, oy, ox, flip, pad=AUG_PAD):
    """RandomCrop(size, padding=pad, zero fill) + RandomHorizontalFlip of uint8 HWC images [N, H, W, C] with given
    per-sample draws, as one gather (the vectorised form of ``resnet2d_hip.augment_u8``)."""
    N, H, W, C = img.shape
    padded = F.pad(img.permute(0, 3, 1, 2), (pad, pad, pad, pad)).permute(0, 2, 3, 1)
    ar_h = torch.arange(H, device=img.device)
    ar_w = torch.arange(W, device=img.device)
    rows = oy.view(N, 1) + ar_h.view(1, H)
    cols_fwd = ar_w.view(1, W).expand(N, W)
    cols = torch.where(flip.view(N, 1).bool(), (W - 1) - cols_fwd, cols_fwd) + ox.view(N, 1)
    n = torch.arange(N, device=img.device).view(N, 1, 1)
    return padded[n, rows.view(N, H, 1), cols.view(N, 1, W)]


class BatchedModuleEngine:
    """Engine API of :class:`~.executor.HipEngine` (train_step / eval_logits / local_opt / saliency_acc) for a
    buffer-free 2-D image ``nn.Module`` on uint8 HWC images ``[N, S, S, 3]``, clients batched with vmap."""
    sample_fields = ("x8", "labels")
    supports_graphs = False

    def __init__(self, template_model, images_u8, labels, device, mean, std, augment=True, amp=None):
        self.device = torch.device(device)
        self.model = template_model.to(self.device)
        self.players = ParamLayout.from_tensors(list(self.model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(self.model.named_buffers()))
        if self.blayers.total:
            raise ValueError("BatchedModuleEngine: the model carries buffers (BatchNorm running statistics); "
                             "use the eager engine")
        self.x8 = images_u8.to(self.device)
        self.labels = labels.to(self.device)
        self.augment = bool(augment)
        self.amp = (self.device.type == "cuda") if amp is None else bool(amp)
        c = int(self.x8.shape[-1])
        self._scale = (1.0 / (255.0 * torch.tensor(std, dtype=torch.float32, device=self.device))).view(1, c, 1, 1)
        self._shift = (-torch.tensor(mean, dtype=torch.float32, device=self.device)
                       / torch.tensor(std, dtype=torch.float32, device=self.device)).view(1, c, 1, 1)
        self._opt = None
        # GPU: the hand-written grouped layers (conv2d_hip.py: conv2d_any.hip convolutions, batched GEMM linears,
        # grouped GroupNorm) over group-stacked tensors instead of vmapped library convolutions; NIDT_B2D_HIP=0 keeps
        # the vmap path (the CPU always uses it)
        self._grouped = None
        if self.device.type == "cuda" and os.environ.get("NIDT_B2D_HIP", "1") != "0":
            from . import conv2d_hip
            if conv2d_hip.supports(self.model):
                from .. import ops
                ops.ext()  # fail loudly without the extension
                self._grouped = conv2d_hip.grouped_model(self.model)

    @property
    def uses_hip_layers(self):
        return self._grouped is not None

    @property
    def input_shape(self):
        n, h, w, c = self.x8.shape
        return (c, h, w)

    # ---------------------------------------------------------------------------------------------- inputs
    def _input(self, idx, aug=None):
        img = self.x8.index_select(0, idx.long())
        if aug is not None:
            img = augment_batch(img, *aug)
        x = img.permute(0, 3, 1, 2).float()
        return x * self._scale + self._shift

    def _params(self, theta, G):
        return {n: theta[:G, o:o + self.players.numel(i)].view((G,) + tuple(self.players.shapes[i]))
                for i, (n, o) in enumerate(zip(self.players.names, self.players.offsets))}

    def _grouped_forward(self, theta, G, x):
        """Group-stacked forward through the grouped twins (``x`` [G*B, C, H, W]); the parameter views of theta's
        rows are leaves when ``theta`` requires no grad, returned for the caller's backward."""
        gm, grp = self._grouped
        grp.G = G
        grp.params = {n: theta[:G, o:o + self.players.numel(i)].view((G,) + tuple(self.players.shapes[i]))
                      for i, (n, o) in enumerate(zip(self.players.names, self.players.offsets))}
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
            out = gm(x.contiguous(memory_format=torch.channels_last))
        out = out[0] if isinstance(out, (list, tuple)) else out
        return out.float(), grp.params

    def _grouped_train(self, theta, grads, x, y, G, B, keep):
        gm, grp = self._grouped
        gm.train(True)
        if keep >= 1.0:
            for mod in gm.modules():
                if isinstance(mod, torch.nn.Dropout):
                    mod.eval()
        leaves = theta.detach()
        gm_params = {}
        for i, (n, o) in enumerate(zip(self.players.names, self.players.offsets)):
            gm_params[n] = leaves[:G, o:o + self.players.numel(i)].view((G,) + tuple(self.players.shapes[i])) \
                .requires_grad_(True)
        grp.G, grp.params = G, gm_params
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
            out = gm(x.reshape((G * B,) + self.input_shape).contiguous(memory_format=torch.channels_last))
        out = (out[0] if isinstance(out, (list, tuple)) else out).float().view(G, B, -1)
        if out.shape[-1] == 1:
            loss = F.binary_cross_entropy_with_logits(out.view(G, B), y.float(), reduction="none").mean(1)
        else:
            loss = F.cross_entropy(out.reshape(G * B, -1), y.long().reshape(-1), reduction="none").view(G, B).mean(1)
        names = list(gm_params)
        gs = torch.autograd.grad(loss.sum(), [gm_params[n] for n in names])
        with torch.no_grad():
            for n, gr in zip(names, gs):
                i = self.players.names.index(n)
                o, k = self.players.offsets[i], self.players.numel(i)
                grads[:G, o:o + k].copy_(gr.reshape(G, k))
        return loss.detach()

    def _forward_fn(self):
        from torch.func import functional_call
        model = self.model

        def fwd(p, x):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.amp):
                out = functional_call(model, p, (x,))
            return (out[0] if isinstance(out, (list, tuple)) else out).float()
        return fwd

    # ---------------------------------------------------------------------------------------------- engine API
    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True):
        from torch.func import grad_and_value, vmap
        aug = None
        if self.augment and seed_dev is not None:
            cl = torch.as_tensor([int(c) for c in (range(G) if cids is None else cids)], dtype=torch.int64,
                                 device=self.device)
            aug = aug_draws_t(seed_dev.to(torch.int64).view(()) + int(seed), cl, B)
        x = self._input(idx, aug).view((G, B) + self.input_shape)
        y = self.labels.index_select(0, idx.long()).view(G, B)
        if self._grouped is not None:
            return self._grouped_train(theta, grads, x, y, G, B, keep)
        fwd = self._forward_fn()
        self.model.train(True)
        if keep >= 1.0:
            for mod in self.model.modules():
                if isinstance(mod, torch.nn.Dropout):
                    mod.eval()

        def loss_fn(p, xb, yb):
            out = fwd(p, xb)
            if out.shape[-1] == 1:
                return F.binary_cross_entropy_with_logits(out.view(-1), yb.float().view(-1))
            return F.cross_entropy(out, yb.long())

        g, loss = vmap(grad_and_value(loss_fn), randomness="different")(self._params(theta.detach(), G), x, y)
        with torch.no_grad():
            for i, (n, o) in enumerate(zip(self.players.names, self.players.offsets)):
                k = self.players.numel(i)
                grads[:G, o:o + k].copy_(g[n].reshape(G, k))
        return loss.detach()

    def eval_logits(self, theta, bufs, idx, G, B):
        from torch.func import vmap
        if self._grouped is not None:
            self._grouped[0].eval()
            with torch.no_grad():
                out, _ = self._grouped_forward(theta, G, self._input(idx))
            return out.reshape(G * B, -1)
        self.model.eval()
        with torch.no_grad():
            x = self._input(idx).view((G, B) + self.input_shape)
            out = vmap(self._forward_fn())(self._params(theta, G), x)
        return out.reshape(G * B, -1)

    def _delegate(self):
        from .executor import HipEngine, TorchEngine
        if self._opt is None:
            if self.device.type == "cuda":
                from .. import ops
                self._opt = HipEngine.__new__(HipEngine)
                self._opt.m = ops.ext()  # fused optimizer kernels: fail loudly without the extension
            else:
                self._opt = TorchEngine.__new__(TorchEngine)
        return self._opt

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False):
        from .executor import HipEngine, TorchEngine
        cls = HipEngine if self.device.type == "cuda" else TorchEngine
        cls.local_opt(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=lr_dev,
                      keep_grad=keep_grad)

    def saliency_acc(self, theta, grads, score, alpha):
        from .executor import HipEngine, TorchEngine
        cls = HipEngine if self.device.type == "cuda" else TorchEngine
        cls.saliency_acc(self._delegate(), theta, grads, score, alpha)
