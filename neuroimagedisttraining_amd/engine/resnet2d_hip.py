"""Client-batched ResNet-18-GN (CIFAR) on the gfx950 conv kernels: G clients' local steps in one lockstep pass.

The reference trains its CIFAR baselines (SubAvg / DisPFL / D-PSGD / FedFomo with ``customized_resnet18``,
``fedml_api/model/cv/resnet.py:91-124``: CIFAR ResNet-18, GroupNorm(32) everywhere, avg_pool2d(4) head) one
client after another through cuDNN.  Here every client of a launch group is a row of the flat ``[C, P]``
parameter matrix and each layer runs ONCE for all of them:

* every convolution (3x3 stride 1/2, the 1x1 stride-2 projection shortcuts, the stem) is the client-grouped
  LDS-DMA implicit-GEMM kernel of ``conv3d.hip`` run on D = 1 volumes with 9 taps (``conv_fwd_g``); the stem's
  3 input channels are zero-padded to 64 (one more layer-1-sized GEMM instead of a separate kernel);
* the data gradient is the same kernel on tap-flipped transposed weights (stride 2: on the zero-upsampled
  gradient; 1x1 stride 2: scattered to the even pixels), the weight gradient is the position-table wgrad
  kernel writing PyTorch-layout fp32 straight into the client's gradient row (``conv_wgrad_g``);
* activations are bf16 channels-last ``[G*B, H, W, C]``; GroupNorm (+ the residual add and ReLU, fused) is the
  one-block-per-sample ``gn.hip`` kernel pair; the head and the loss are small fp32 torch ops over the whole group
  (one launch per op, not per client).  The backward is written out explicitly (no autograd graph) and every op
  is deterministic and workspace-free, so the step is hipGraph-capturable.

A CPU twin (``device.type == 'cpu'``) runs the same graph with fp32 torch convolutions (grouped by client); the
CPU tests compare it with per-client autograd through the reference-shaped ``nn.Module``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from .flat import ParamLayout

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)   # reference cifar10/data_loader.py normalisation
CIFAR_STD = (0.2470, 0.2435, 0.2616)
GN_GROUPS = 32
GN_EPS = 1e-5


def _stream():
    return torch.cuda.current_stream().cuda_stream


def conv_fwd(x_ptr, w_ptr, y_ptr, G, B, D, H, W, Cin, Cout, kt, st, pad, padd, device):
    """Client-grouped conv forward (``conv_fwd_g``), split over the reduction when the output grid is too small to
    fill the chip (``conv_fwd_g_ksplit``: deep layers at small spatial size, few clients per GPU)."""
    m = ops.ext()
    ks = m.conv_fwd_g_ksplit(G, B, D, H, W, Cin, Cout, kt, st, pad, padd)
    if ks <= 1:
        m.conv_fwd_g(x_ptr, w_ptr, y_ptr, G, B, D, H, W, Cin, Cout, kt, st, pad, padd, _stream())
        return
    kd, khw = (3 if kt == 27 else 1), (1 if kt == 1 else 3)
    Mg = B * ((D + 2 * padd - kd) // st + 1) * ((H + 2 * pad - khw) // st + 1) * ((W + 2 * pad - khw) // st + 1)
    part = torch.empty(ks * G * Mg * Cout, device=device, dtype=torch.float32)
    m.conv_fwd_gk(x_ptr, w_ptr, y_ptr, part.data_ptr(), ks, G, B, D, H, W, Cin, Cout, kt, st, pad, padd, _stream())


class GroupedConv:
    """One conv layer of the client-grouped network (weights = rows of theta at ``off``, PyTorch layout
    ``[Cout, cin, k, k]``).  ``cin_p`` = channels of the activation tensor (cin zero-padded to 64)."""

    def __init__(self, off, cout, cin, k, stride, pad, hip):
        self.off, self.cout, self.cin, self.k, self.stride, self.pad = off, cout, cin, k, stride, pad
        self.kt = k * k
        self.cin_p = cin if cin % 64 == 0 else (cin + 63) // 64 * 64
        self.hip = hip
        self.numel = cout * cin * k * k
        self.need_dgrad = self.cin_p == self.cin  # the (channel-padded) stem needs no input gradient
        self._packed = None

    def out_hw(self, h, w):
        return ((h + 2 * self.pad - self.k) // self.stride + 1, (w + 2 * self.pad - self.k) // self.stride + 1)

    # ---------------------------------------------------------------- weights
    def _wp(self, theta, G, transposed):
        m = ops.ext()
        wp = torch.empty(G, self.cout, self.kt, self.cin_p, device=theta.device, dtype=torch.bfloat16)
        wt = torch.empty(G, self.cin_p, self.kt, self.cout, device=theta.device, dtype=torch.bfloat16) \
            if transposed else None
        m.pack_conv_wk(theta.data_ptr(), theta.stride(0), self.off, G, self.cout, self.cin_p, self.kt, self.cin, 1.0,
                       wp.data_ptr(), wt.data_ptr() if transposed else 0, _stream())
        return wp, wt

    def _wtorch(self, theta, G):
        return theta[:, self.off:self.off + self.numel].reshape(G * self.cout, self.cin, self.k, self.k)

    # ---------------------------------------------------------------- forward
    def fwd(self, x, theta, G, train=False):
        """``train``: also pack the transposed (dgrad) weights now and keep both for :meth:`bwd` of this step
        (one packing pass per conv per step instead of re-packing in the backward)."""
        N, H, W, C = x.shape
        assert C == self.cin_p and N % G == 0, (x.shape, self.cin_p, G)
        Ho, Wo = self.out_hw(H, W)
        if not self.hip:
            return self._torch_fwd(x, self._wtorch(theta, G), G)
        wp, wt = self._wp(theta, G, train and self.need_dgrad)
        self._packed = (theta.data_ptr(), G, wt) if train else None
        y = torch.empty(N, Ho, Wo, self.cout, device=x.device, dtype=torch.bfloat16)
        conv_fwd(x.data_ptr(), wp.data_ptr(), y.data_ptr(), G, N // G, 1, H, W, self.cin_p, self.cout,
                 self.kt, self.stride, self.pad, 0, x.device)
        return y

    def _torch_fwd(self, x, w, G):
        N, H, W, C = x.shape
        B = N // G
        xc = x[..., :self.cin].reshape(G, B, H, W, self.cin).permute(1, 0, 4, 2, 3).reshape(B, G * self.cin, H, W)
        y = F.conv2d(xc, w, stride=self.stride, padding=self.pad, groups=G)
        Ho, Wo = y.shape[-2:]
        return y.view(B, G, self.cout, Ho, Wo).permute(1, 0, 3, 4, 2).reshape(N, Ho, Wo, self.cout)

    # ---------------------------------------------------------------- backward
    def bwd(self, dy, x, theta, grads, G, need_dx, scratch=None):
        """dW -> grads rows (PyTorch layout at ``off``); returns dX ``[N, H, W, cin_p]`` (or None)."""
        if not self.hip:
            return self._torch_bwd(dy, x, theta, grads, G, need_dx)
        m, st = ops.ext(), _stream()
        N, H, W, _ = x.shape
        B = N // G
        Ho, Wo = dy.shape[1:3]
        dy = dy.contiguous()
        ns = m.conv_wgrad_nsplit_g(G, B, 1, H, W, self.cin_p, self.cout, self.kt, self.stride, self.pad, 0)
        part = torch.empty(ns * G * self.cout * self.kt * self.cin_p, device=x.device, dtype=torch.float32)
        ptab = torch.empty(B * Ho * Wo, 2, device=x.device, dtype=torch.int32)
        m.conv_pos_table_g(ptab.data_ptr(), B, 1, H, W, self.kt, self.stride, self.pad, 0, st)
        if self.cin_p == self.cin:
            m.conv_wgrad_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grads.data_ptr(), grads.stride(0), self.off,
                           G, B, 1, H, W, self.cin_p, self.cout, self.kt, self.stride, self.pad, 0, ns, 1.0,
                           ptab.data_ptr(), st)
        else:  # channel-padded stem: full-width gradient, then the live input channels into the row
            full = torch.empty(G, self.cout * self.cin_p * self.kt, device=x.device, dtype=torch.float32)
            m.conv_wgrad_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), full.data_ptr(), full.stride(0), 0, G, B, 1,
                           H, W, self.cin_p, self.cout, self.kt, self.stride, self.pad, 0, ns, 1.0, ptab.data_ptr(), st)
            grads[:, self.off:self.off + self.numel].view(G, self.cout, self.cin, self.kt).copy_(
                full.view(G, self.cout, self.cin_p, self.kt)[:, :, :self.cin])
        if not need_dx:
            return None
        pk, self._packed = self._packed, None
        if pk is not None and pk[0] == theta.data_ptr() and pk[1] == G and pk[2] is not None:
            wt = pk[2]
        else:
            _, wt = self._wp(theta, G, True)
        dx = torch.empty(N, H, W, self.cin_p, device=x.device, dtype=torch.bfloat16)
        if self.stride == 1:
            conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, 1, Ho, Wo, self.cout, self.cin_p, self.kt,
                         1, self.k - 1 - self.pad, 0, x.device)
        elif self.k == 3:
            # stride 2: dX = conv(zero-upsampled dY, flipped W^T, pad k-1-pad) (H = 2 Ho for the even CIFAR maps)
            assert H == 2 * Ho and W == 2 * Wo and self.pad == 1, (H, W, Ho, Wo)
            up = torch.zeros(N, H, W, self.cout, device=x.device, dtype=torch.bfloat16)
            up[:, ::2, ::2] = dy
            conv_fwd(up.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, 1, H, W, self.cout, self.cin_p, self.kt,
                         1, 1, 0, x.device)
        else:
            # 1x1 stride 2: only the even pixels were read: dX there = W^T dY, zero elsewhere
            assert self.k == 1 and self.pad == 0 and (H + 1) // 2 == Ho and (W + 1) // 2 == Wo
            sub = torch.empty(N, Ho, Wo, self.cin_p, device=x.device, dtype=torch.bfloat16)
            conv_fwd(dy.data_ptr(), wt.data_ptr(), sub.data_ptr(), G, B, 1, Ho, Wo, self.cout, self.cin_p, 1, 1,
                         0, 0, x.device)
            dx.zero_()
            dx[:, ::2, ::2] = sub
        return dx

    def _torch_bwd(self, dy, x, theta, grads, G, need_dx):
        w = self._wtorch(theta, G).detach().clone().requires_grad_(True)
        xx = x.detach().clone().requires_grad_(need_dx)
        with torch.enable_grad():
            y = self._torch_fwd(xx, w, G)
            outs = torch.autograd.grad(y, [w, xx] if need_dx else [w], dy.to(y.dtype))
        grads[:, self.off:self.off + self.numel].copy_(outs[0].reshape(G, -1))
        return outs[1] if need_dx else None


class GroupNormG:
    """GroupNorm(32) over channels-last activations of G clients (per-client affine rows at off_w / off_b), with the
    block's residual add and ReLU fused into the forward and the ReLU mask into the backward.  HIP: ``gn.hip``
    (one block per sample, deterministic, graph-safe); CPU: the same math in fp32 torch ops."""

    def __init__(self, off_w, off_b, C, hip):
        self.off_w, self.off_b, self.C, self.hip = off_w, off_b, C, hip

    def _affine(self, theta):
        return theta[:, self.off_w:self.off_w + self.C], theta[:, self.off_b:self.off_b + self.C]

    def fwd(self, t, theta, G, res=None, relu=False):
        """t [N, H, W, C] -> (relu?(gn(t) + res) in t's dtype, saved statistics)."""
        N, H, W, C = t.shape
        if self.hip:
            t = t.contiguous()
            y = torch.empty_like(t)
            stats = torch.empty(N, GN_GROUPS, 2, device=t.device, dtype=torch.float32)
            r = res.contiguous() if res is not None else None
            ops.ext().gn_fwd(t.data_ptr(), r.data_ptr() if r is not None else 0, theta.data_ptr(), theta.stride(0),
                             self.off_w, self.off_b, y.data_ptr(), stats.data_ptr(), N, N // G, H * W, C, int(relu),
                             _stream())
            return y, stats
        B = N // G
        tf = t.float().view(N, H * W, GN_GROUPS, C // GN_GROUPS)
        mean = tf.mean(dim=(1, 3), keepdim=True)
        rstd = torch.rsqrt((tf - mean).square().mean(dim=(1, 3), keepdim=True) + GN_EPS)
        gw, gb = self._affine(theta)
        y = ((tf - mean) * rstd).view(G, B, H * W, C) * gw.view(G, 1, 1, C) + gb.view(G, 1, 1, C)
        y = y.view(N, H, W, C)
        if res is not None:
            y = y + res.float()
        if relu:
            y = torch.relu(y)
        return y.to(t.dtype), (mean, rstd)

    def bwd(self, dy, mask, t, saved, theta, grads, G):
        """dy [N, H, W, C] (fp32 or bf16), times (mask > 0) if a mask is given; writes the dgamma/dbeta rows,
        returns dt in t's dtype."""
        N, H, W, C = t.shape
        B = N // G
        if self.hip:
            dy = dy.contiguous()
            assert dy.dtype in (torch.float32, torch.bfloat16)
            dt = torch.empty_like(t)
            part = torch.empty(N, C, 2, device=t.device, dtype=torch.float32)
            m = mask.contiguous() if mask is not None else None
            ops.ext().gn_bwd(dy.data_ptr(), int(dy.dtype == torch.bfloat16), m.data_ptr() if m is not None else 0,
                             t.data_ptr(), saved.data_ptr(), theta.data_ptr(), theta.stride(0), self.off_w,
                             dt.data_ptr(), part.data_ptr(), N, B, H * W, C, _stream())
            ops.ext().gn_param_grads(part.data_ptr(), G, B, C, grads.data_ptr(), grads.stride(0), self.off_w,
                                     self.off_b, _stream())
            return dt
        mean, rstd = saved
        cg = C // GN_GROUPS
        dy = dy.float()
        if mask is not None:
            dy = dy * (mask > 0)
        xhat = (t.float().view(N, H * W, GN_GROUPS, cg) - mean) * rstd
        dyv = dy.reshape(N, H * W, GN_GROUPS, cg)
        grads[:, self.off_w:self.off_w + C].copy_((dyv * xhat).view(G, B * H * W, C).sum(1))
        grads[:, self.off_b:self.off_b + C].copy_(dy.reshape(G, B * H * W, C).sum(1))
        gw, _ = self._affine(theta)
        dxh = (dy.reshape(G, B, H * W, C) * gw.view(G, 1, 1, C)).view(N, H * W, GN_GROUPS, cg)
        m1 = dxh.mean(dim=(1, 3), keepdim=True)
        m2 = (dxh * xhat).mean(dim=(1, 3), keepdim=True)
        return ((dxh - m1 - xhat * m2) * rstd).view(N, H, W, C).to(t.dtype)


class GroupedResNet18GN:
    """The forward/backward graph of ``customized_resnet18`` for G clients at once (see module docstring)."""

    def __init__(self, players: ParamLayout, device, hip=None):
        self.device = torch.device(device)
        self.hip = (self.device.type == "cuda") if hip is None else hip
        self.act = torch.bfloat16 if self.hip else torch.float32
        L = players
        off = {n: o for n, o in zip(L.names, L.offsets)}
        shp = dict(zip(L.names, L.shapes))

        def conv(name, stride, pad):
            co, ci, k, _ = shp[name]
            return GroupedConv(off[name], co, ci, k, stride, pad, self.hip)

        def gn(prefix):
            return GroupNormG(off[prefix + ".weight"], off[prefix + ".bias"], shp[prefix + ".weight"][0], self.hip)

        self.stem = conv("conv1.weight", 1, 1)
        self.stem_gn = gn("bn1")
        self.blocks = []
        for li in range(1, 5):
            for bi in range(2):
                p = "layer%d.%d." % (li, bi)
                stride = 2 if (li > 1 and bi == 0) else 1
                blk = {"c1": conv(p + "conv1.weight", stride, 1), "n1": gn(p + "bn1"),
                       "c2": conv(p + "conv2.weight", 1, 1), "n2": gn(p + "bn2")}
                if p + "shortcut.0.weight" in off:
                    blk["cs"] = conv(p + "shortcut.0.weight", stride, 0)
                    blk["ns"] = gn(p + "shortcut.1")
                self.blocks.append(blk)
        self.lw_off, self.lb_off = off["linear.weight"], off["linear.bias"]
        self.ncls, self.feat = shp["linear.weight"]
        mean = torch.tensor(CIFAR_MEAN, dtype=torch.float32).view(1, 1, 1, 3)
        std = torch.tensor(CIFAR_STD, dtype=torch.float32).view(1, 1, 1, 3)
        self.norm_scale = (1.0 / (255.0 * std)).to(self.device)
        self.norm_shift = (-mean / std).to(self.device)

    # ------------------------------------------------------------------ input
    def input(self, x8):
        """uint8 [N, 32, 32, 3] -> normalised activation [N, 32, 32, cin_p] (channels zero-padded)."""
        x = x8.float() * self.norm_scale + self.norm_shift
        cp = self.stem.cin_p
        if cp != 3:
            x = F.pad(x, (0, cp - 3))
        return x.to(self.act).contiguous()

    # ------------------------------------------------------------------ forward
    def forward(self, x, theta, G, train=False):
        saved = []
        t = self.stem.fwd(x, theta, G, train)
        a, st = self.stem_gn.fwd(t, theta, G, relu=True)
        saved.append((x, t, st, a))
        for blk in self.blocks:
            xin = a
            t1 = blk["c1"].fwd(xin, theta, G, train)
            h1, s1 = blk["n1"].fwd(t1, theta, G, relu=True)
            t2 = blk["c2"].fwd(h1, theta, G, train)
            if "cs" in blk:
                ts = blk["cs"].fwd(xin, theta, G, train)
                ysc, ss = blk["ns"].fwd(ts, theta, G)
            else:
                ts, ss, ysc = None, None, xin
            a, s2 = blk["n2"].fwd(t2, theta, G, res=ysc, relu=True)
            saved.append((xin, t1, s1, h1, t2, s2, ts, ss, a))
        N, H, W, C = a.shape
        pooled = a.float().view(N, H * W, C).mean(1)  # avg_pool2d(4) on the 4x4 map
        B = N // G
        lw = theta[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat)
        lb = theta[:, self.lb_off:self.lb_off + self.ncls]
        # the 512 -> 10 head as broadcast multiply-reduce, not bmm: BLAS calls keep library workspaces that a
        # replayed hipGraph would share with eager work
        logits = (pooled.view(G, B, 1, C) * lw.view(G, 1, self.ncls, C)).sum(-1) + lb.view(G, 1, self.ncls)
        return logits.view(N, self.ncls), pooled, saved

    # ------------------------------------------------------------------ train step
    def train_step(self, theta, grads, x, y, G, B):
        logits, pooled, saved = self.forward(x, theta, G, train=True)
        lg = logits.view(G, B, self.ncls)
        logp = torch.log_softmax(lg, dim=-1)
        yl = y.long().view(G, B)
        losses = -logp.gather(2, yl.unsqueeze(2)).squeeze(2).mean(1)
        # softmax - onehot (scatter, not F.one_hot: its range check syncs the host, which a graph capture forbids)
        dlog = logp.exp().scatter_add(2, yl.unsqueeze(2), torch.full_like(logp[..., :1], -1.0)) / B  # [G, B, K]
        lw = theta[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat)
        grads[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat).copy_(
            (dlog.view(G, B, self.ncls, 1) * pooled.view(G, B, 1, self.feat)).sum(1))
        grads[:, self.lb_off:self.lb_off + self.ncls].copy_(dlog.sum(1))
        dpool = (dlog.view(G, B, self.ncls, 1) * lw.view(G, 1, self.ncls, self.feat)).sum(2).view(G * B, 1, self.feat)
        a = saved[-1][-1]
        N, H, W, C = a.shape
        da = (dpool / float(H * W)).expand(N, H * W, C).reshape(N, H, W, C).contiguous()
        for blk, sv in zip(reversed(self.blocks), reversed(saved[1:])):
            xin, t1, s1, h1, t2, s2, ts, ss, a = sv
            dt2 = blk["n2"].bwd(da, a, t2, s2, theta, grads, G)
            dh1 = blk["c2"].bwd(dt2, h1, theta, grads, G, True)
            dt1 = blk["n1"].bwd(dh1, h1, t1, s1, theta, grads, G)
            dx1 = blk["c1"].bwd(dt1, xin, theta, grads, G, True)
            dx2 = None
            if "cs" in blk:
                dts = blk["ns"].bwd(da, a, ts, ss, theta, grads, G)
                dx2 = blk["cs"].bwd(dts, xin, theta, grads, G, True)
            if self.hip:
                out = torch.empty(dx1.shape, device=dx1.device, dtype=torch.float32)
                ops.ext().res_grad(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr() if dx2 is not None else 0,
                                   0 if dx2 is not None else da.data_ptr(), 0 if dx2 is not None else a.data_ptr(),
                                   out.numel(), _stream())
                da = out
            else:
                da = dx1.float() + (dx2.float() if dx2 is not None else da * (a > 0))
        x0, t0, st0, a0 = saved[0]
        dt0 = self.stem_gn.bwd(da, a0, t0, st0, theta, grads, G)
        self.stem.bwd(dt0, x0, theta, grads, G, False)
        return losses.detach()

    def eval_logits(self, theta, x, G):
        logits, _, _ = self.forward(x, theta, G)
        return logits


class ResNetHipEngine:
    """Engine API of :class:`~.executor.HipEngine` (train_step / eval_logits / local_opt / saliency_acc) for the
    client-batched ResNet-18-GN on CIFAR-shape uint8 images ``[N, 32, 32, 3]``."""

    def __init__(self, template_model, images_u8, labels, device, hip=None):
        self.device = torch.device(device)
        self.players = ParamLayout.from_tensors(list(template_model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(template_model.named_buffers()))
        assert self.blayers.total == 0, "GroupNorm ResNet carries no buffers"
        self.net = GroupedResNet18GN(self.players, self.device, hip=hip)
        self.x8 = images_u8.to(self.device)
        self.labels = labels.to(self.device)
        if self.net.hip:
            ops.ext()  # fail loudly on a GPU box without the extension
        self.supports_graphs = self.device.type == "cuda"
        self.graph_cache_limit = 24  # each captured step holds its own activation pool
        self._opt = None

    def _batch(self, idx):
        ix = idx.long()
        return self.net.input(self.x8.index_select(0, ix)), self.labels.index_select(0, ix)

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True):
        x, y = self._batch(idx)
        return self.net.train_step(theta, grads, x, y, G, B)

    def eval_logits(self, theta, bufs, idx, G, B):
        with torch.no_grad():
            x, _ = self._batch(idx)
            return self.net.eval_logits(theta, x, G).float()

    def _delegate(self):
        if self._opt is None:
            from .executor import HipEngine, TorchEngine
            self._opt = HipEngine.__new__(HipEngine) if self.net.hip else TorchEngine.__new__(TorchEngine)
            if self.net.hip:
                self._opt.m = ops.ext()
        return self._opt

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False):
        from .executor import HipEngine, TorchEngine
        cls = HipEngine if self.net.hip else TorchEngine
        cls.local_opt(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=lr_dev,
                      keep_grad=keep_grad)

    def saliency_acc(self, theta, grads, score, alpha):
        from .executor import HipEngine, TorchEngine
        cls = HipEngine if self.net.hip else TorchEngine
        cls.saliency_acc(self._delegate(), theta, grads, score, alpha)


def synthetic_cifar(n, n_classes=10, seed=0, signal=0.3):
    """CIFAR-10-shape synthetic images (uint8 [n, 32, 32, 3]) with a weak class-dependent colour/texture signal
    and labels; the reference's data files are not available offline."""
    g = np.random.default_rng(seed)
    labels = g.integers(0, n_classes, size=n)
    base = g.integers(0, 256, size=(n, 32, 32, 3)).astype(np.float32)
    proto = g.integers(0, 256, size=(n_classes, 32, 32, 3)).astype(np.float32)
    img = (1 - signal) * base + signal * proto[labels]
    return torch.from_numpy(np.clip(img, 0, 255).astype(np.uint8)), torch.from_numpy(labels.astype(np.int64))
