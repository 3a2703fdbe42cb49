"""Client-batched ResNet-18-GN (CIFAR-10/100, Tiny-ImageNet) on the gfx950 conv kernels: G clients' local steps in
one lockstep pass.

The reference trains its image baselines (SubAvg / DisPFL / D-PSGD / FedFomo / Ditto / Local with
``customized_resnet18`` on CIFAR, ``fedml_api/model/cv/resnet.py:91-124``, and ``tiny_resnet18`` on Tiny-ImageNet,
``resnet.py:134-214``: ResNet-18 with GroupNorm(32) everywhere) one client after another through cuDNN.  Here every
client of a launch group is a row of the flat ``[C, P]`` parameter matrix and each layer runs ONCE for all of them:

* input: one fused kernel (``img.hip``) gathers the batch's uint8 images, applies the reference's train-time
  RandomCrop(pad 4) + RandomHorizontalFlip with per-(step, client, sample) draws made on device, normalises and
  zero-pads the channels (``data_loader.py:46-52`` of the cifar10 / cifar100 / tiny loaders);
* weights: every layer's bf16 MFMA images (forward, and the data-gradient image in its tap-slot order) are packed
  in two launches per step (``pack.hip``);
* every convolution (3x3 stride 1/2, the 1x1 stride-2 projection shortcuts, the stem) is the client-grouped
  LDS-DMA implicit-GEMM kernel of ``conv3d.hip`` run on D = 1 volumes with 9 taps (``conv_fwd_g``); the stem's
  3x3 window is folded into the input channels by the input stage (27 live of 64), so it runs as a 1x1 conv
  ([STEM-FOLD]: 9x fewer MACs than nine channel-padded taps, forward and weight gradient);
* data gradients: stride 1 = the same kernel on tap-flipped transposed weights; stride 2 (3x3) = four sub-pixel
  phase convs over the dy grid with 1/2/2/4 taps written straight into the interleaved dX positions
  (``conv_dgrad_s2_g``: 4x fewer MACs than a conv over the zero-upsampled gradient, no memset); 1x1 stride 2 = the
  half-resolution W^T dY that ``res_grad_s2`` adds at the even pixels.  The weight gradient is the position-table
  wgrad kernel writing PyTorch-layout fp32 straight into the client's gradient row (``conv_wgrad_g``);
* activations are bf16 channels-last ``[G*B, H, W, C]``; GroupNorm (+ the residual add and ReLU, fused) is the
  one-block-per-sample ``gn.hip`` kernel pair (streaming variant for the 64x64 Tiny maps); the head and the loss are
  small fp32 torch ops over the whole group (one launch per op, not per client).  The backward is written out
  explicitly (no autograd graph) and every op is deterministic and workspace-free, so the step is
  hipGraph-capturable.

A CPU twin (``device.type == 'cpu'``) runs the same graph with fp32 torch convolutions (grouped by client) and the
same augmentation draws; the CPU tests compare it with per-client autograd through the reference-shaped
``nn.Module``.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from .flat import ParamLayout

CIFAR_MEAN = (0.49139968, 0.48215827, 0.44653124)   # reference cifar10/data_loader.py:43-44 normalisation
CIFAR_STD = (0.24703233, 0.24348505, 0.26158768)
TINY_MEAN = (0.5, 0.5, 0.5)                          # reference tiny_imagenet/data_loader.py:49-50
TINY_STD = (0.5, 0.5, 0.5)
AUG_PAD = 4                                          # RandomCrop(S, padding=4) of every image loader
GN_GROUPS = 32
GN_EPS = 1e-5


_stream = ops.stream
_EXT = {}


def _external(ptr):
    """torch stream object of a raw handle (cached): for the few torch ops a side branch issues."""
    s = _EXT.get(ptr)
    if s is None:
        s = _EXT[ptr] = torch.cuda.ExternalStream(ptr)
    return s


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


# ------------------------------------------------------------------------------------------------ augmentation
_M64 = (1 << 64) - 1


def mix64(seed, a, b):
    """The splitmix64 finaliser of ``img.hip`` (exact twin, Python ints)."""
    z = (int(seed) ^ ((0x9e3779b97f4a7c15 * (((int(a) & 0xffffffff) << 32) ^ int(b))) & _M64)) & _M64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & _M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & _M64
    return z ^ (z >> 31)


def aug_draws(seed, cids, B, pad=AUG_PAD):
    """Per-sample (crop y offset, crop x offset, flip) of a lockstep step: sample j of client cids[g] draws from
    mix64(step seed, client id, j) — offsets uniform in [0, 2 pad] (torchvision RandomCrop(padding=pad)), flip with
    p = 1/2 (RandomHorizontalFlip).  Returns int64 arrays [len(cids) * B]."""
    span = 2 * pad + 1
    oy, ox, fl = [], [], []
    for c in cids:
        for j in range(B):
            h = mix64(seed, c, j)
            lo, hi = h & 0xffffffff, h >> 32
            oy.append(lo % span)
            ox.append((lo // span) % span)
            fl.append(hi & 1)
    return np.array(oy), np.array(ox), np.array(fl)


def augment_u8(img, oy, ox, flip, pad=AUG_PAD):
    """torchvision RandomCrop(size, padding=pad) + RandomHorizontalFlip of uint8 HWC images [N, H, W, 3] with given
    draws (the CPU twin of the fused HIP input stage; padded pixels are 0)."""
    N, H, W, _ = img.shape
    padded = torch.zeros(N, H + 2 * pad, W + 2 * pad, 3, dtype=img.dtype, device=img.device)
    padded[:, pad:pad + H, pad:pad + W] = img
    out = torch.empty_like(img)
    for n in range(N):
        crop = padded[n, int(oy[n]):int(oy[n]) + H, int(ox[n]):int(ox[n]) + W]
        out[n] = crop.flip(1) if int(flip[n]) else crop
    return out


def fold_window(x, cin=3, cp=None):
    """The [STEM-FOLD] input from a channel-padded image [N, H, W, C] (channels < cin live): channel 3 t + c of pixel
    (y, x) = channel c of pixel (y + kh - 1, x + kw - 1), t = 3 kh + kw, zero outside (twin of img.hip k_img_fold)."""
    N, H, W, C = x.shape
    cp = C if cp is None else cp
    xp = F.pad(x[..., :cin].float(), (0, 0, 1, 1, 1, 1))
    out = torch.zeros(N, H, W, cp, dtype=torch.float32, device=x.device)
    for t in range(9):
        kh, kw = divmod(t, 3)
        out[..., cin * t:cin * (t + 1)] = xp[:, kh:kh + H, kw:kw + W]
    return out.to(x.dtype)


# ------------------------------------------------------------------------------------------------ convolutions
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


_SLAB_TABS = {}


def slab_conv2d(x_ptr, w_ptr, y_ptr, G, B, H, W, Cin, Cout, device, stats=None):
    """3x3 stride-1 pad-1 conv through the kd-slab union kernel (``conv2d_fwd_slab``: one input union per 64-channel
    chunk serves all nine taps) when the shape and grid qualify (``conv2d_fwd_slab_pick``; ``NIDT_2D_SLAB=0`` keeps
    the per-tap kernels); returns False otherwise.  The union table depends on the shape only and is built once per
    (B, H, W).  ``stats`` = (zero-bias ptr, partials ptr): [GN-EPI] the 256-position slab form also writes the
    per-block channel statistics (returns 2 then; the depth-batched form has blocks spanning samples and writes none)."""
    m = ops.ext()
    if not m.conv2d_fwd_slab_pick(G, B, H, W, Cin, Cout):
        if not m.conv2d_fwd_slab_bd_pick(G, B, H, W, Cin, Cout):
            return False
        # [SLAB-BD] maps whose blocks span several samples: the samples as the depth planes of one volume
        key = ("bd", str(device), B, H, W, Cin, Cout)  # the block size (256 / 128 positions) depends on the channels
        tab = _SLAB_TABS.get(key)
        if tab is None:
            tab = torch.empty(m.conv2d_fwd_slab_bd_table_size(B, H, W, Cin, Cout), device=device, dtype=torch.int32)
            m.conv2d_fwd_slab_bd_table(tab.data_ptr(), B, H, W, Cin, Cout, _stream())
            if not torch.cuda.is_current_stream_capturing():
                torch.cuda.current_stream().synchronize()
                _SLAB_TABS[key] = tab
        m.conv2d_fwd_slab_bd(x_ptr, w_ptr, y_ptr, G, B, H, W, Cin, Cout, tab.data_ptr(), _stream())
        return True
    key = (str(device), B, H, W)
    tab = _SLAB_TABS.get(key)
    if tab is None:
        tab = torch.empty(m.conv3d_fwd_slab_table_size(B, 1, H, W, 1), device=device, dtype=torch.int32)
        m.conv3d_fwd_slab_table(tab.data_ptr(), B, 1, H, W, 1, _stream())
        if not torch.cuda.is_current_stream_capturing():  # built inside a capture: that graph's memory, not cached
            # the cached table is read by launches on other streams (side lanes): complete it before sharing it
            torch.cuda.current_stream().synchronize()
            _SLAB_TABS[key] = tab
    if stats is not None:
        m.conv2d_fwd_slab_stats(x_ptr, w_ptr, stats[0], y_ptr, stats[1], G, B, H, W, Cin, Cout, tab.data_ptr(),
                                _stream())
        return 2
    m.conv2d_fwd_slab(x_ptr, w_ptr, y_ptr, G, B, H, W, Cin, Cout, tab.data_ptr(), _stream())
    return True


def tap_slots(kt, stride):
    """Tap order of a layer's data-gradient weight image (``conv_tap_slots`` in conv3d.hip): stride 1 -> flipped,
    stride 2 (3x3) -> sub-pixel phase order, 1x1 -> identity."""
    if torch.cuda.is_available():
        try:
            return list(ops.ext().conv_tap_slots(kt, stride))
        except Exception:  # noqa: BLE001 - CPU twin without the extension
            pass
    if kt == 1:
        return [0]
    if stride == 1:
        return [kt - 1 - t for t in range(kt)]
    # 2-D sub-pixel phases (conv_s2_phase_plan): per dim phase 0 <- k=1, phase 1 <- k=0, k=2
    lists = {0: [1], 1: [0, 2]}
    out, slot = [0] * kt, 0
    for ah in (0, 1):
        for aw in (0, 1):
            for kh in lists[ah]:
                for kw in lists[aw]:
                    out[kh * 3 + kw] = slot
                    slot += 1
    return out


class GroupedConv:
    """One conv layer of the client-grouped network (weights = rows of theta at ``off``, PyTorch layout
    ``[Cout, cin, k, k]``).  ``cin_p`` = channels of the activation tensor (cin zero-padded to 64)."""

    _keep = []  # tensors read by the weight-gradient branch of the step in flight (released at its join)

    def __init__(self, off, cout, cin, k, stride, pad, hip):
        self.off, self.cout, self.cin, self.k, self.stride, self.pad = off, cout, cin, k, stride, pad
        self.kt = k * k
        self.cin_p = cin if cin % 64 == 0 else (cin + 63) // 64 * 64
        self.hip = hip
        self.numel = cout * cin * k * k
        self.need_dgrad = self.cin_p == self.cin  # the (channel-padded) stem needs no input gradient
        self.slots = tap_slots(self.kt, stride)
        self.wp = self.wt = None  # packed images of the current step (WeightPacker.pack)
        self._ptabs = {}  # wgrad output-position tables per (B, H, W)
        # [STEM-FOLD] (set by the network for its 3-channel stem, HIP only): the input arrives with the 3x3 window
        # folded into its channels (img.hip k_img_fold, channel 3 t + c), so the layer runs as a 1x1 conv over
        # K = 27 (padded to cin_p) with the folded weight image [Cout][27 -> cin_p]
        self.fold = False
        # folded weight image per packed-image buffer (persistent: its zero tail is written once).  Keyed by the
        # buffer, not by G: launches of different shapes with the same G (a partial-batch step on a side lane beside
        # a full-batch step, concurrent evaluation lanes) must not share one
        self._wf = {}
        self._zb = {}  # [GN-EPI] zero bias per G (the statistics epilogue runs on the bias path)
        self.gn_part = None

    def geometry(self):
        """(taps, stride, pad) of the launches: the folded stem is a 1x1 stride-1 conv."""
        return (1, 1, 0) if self.fold else (self.kt, self.stride, self.pad)

    def _fold_w(self, wp, G):
        """[G, Cout, 1, cin_p] folded image from the step's 9-tap image wp [G, Cout, 9, cin_p] (channels < 3 live):
        wf[g, co, 3 t + c] = wp[g, co, t, c] (one strided copy; the 27 .. cin_p-1 tail stays zero)."""
        key = (wp.data_ptr(), G)
        wf = self._wf.get(key)
        if wf is None:
            wf = self._wf[key] = torch.zeros(G, self.cout, 1, self.cin_p, device=wp.device, dtype=torch.bfloat16)
        wf.view(G, self.cout, self.cin_p)[:, :, :self.kt * self.cin].view(G, self.cout, self.kt, self.cin).copy_(
            wp.view(G, self.cout, self.kt, self.cin_p)[..., :self.cin])
        return wf

    def out_hw(self, h, w):
        return ((h + 2 * self.pad - self.k) // self.stride + 1, (w + 2 * self.pad - self.k) // self.stride + 1)

    # ---------------------------------------------------------------- weights
    def _wp(self, theta, G, transposed):
        """Standalone per-layer packing (kernel tests); the network packs every layer at once (WeightPacker)."""
        m = ops.ext()
        wp = torch.empty(G, self.cout, self.kt, self.cin_p, device=theta.device, dtype=torch.bfloat16)
        wt = torch.empty(G, self.cin_p, self.kt, self.cout, device=theta.device, dtype=torch.bfloat16) \
            if transposed else None
        WeightPacker([self], theta.device).pack_into(theta, G, wp, wt)
        return wp, wt

    def _wtorch(self, theta, G):
        return theta[:, self.off:self.off + self.numel].reshape(G * self.cout, self.cin, self.k, self.k)

    # ---------------------------------------------------------------- forward
    def fwd(self, x, theta, G, train=False, packed=False, gn_stats=False):
        """``packed``: the network's WeightPacker has packed this step's images (``self.wp`` / ``self.wt``);
        otherwise (standalone layer) the layer packs its own, incl. the dgrad image when ``train``.  ``gn_stats``
        ([GN-EPI]): when the layer runs on the 256-position slab kernel, its epilogue also writes the per-block channel
        statistics of the output for the GroupNorm that follows (``self.gn_part`` = (partials, blocks per sample,
        positions per block), else None)."""
        self.gn_part = None
        N, H, W, C = x.shape
        assert C == self.cin_p and N % G == 0, (x.shape, self.cin_p, G)
        Ho, Wo = self.out_hw(H, W)
        if not self.hip:
            return self._torch_fwd(x, self._wtorch(theta, G), G)
        if not packed:
            wp, wt = self._wp(theta, G, train and self.need_dgrad)
            self.wp = (wp, G, theta.data_ptr())
            self.wt = (wt, G, theta.data_ptr()) if wt is not None else None
        wp = self.wp[0]
        y = torch.empty(N, Ho, Wo, self.cout, device=x.device, dtype=torch.bfloat16)
        if self.fold:
            conv_fwd(x.data_ptr(), self._fold_w(wp, G).data_ptr(), y.data_ptr(), G, N // G, 1, H, W, self.cin_p,
                     self.cout, 1, 1, 0, 0, x.device)
            return y
        if self.kt == 9 and self.stride == 1 and self.pad == 1:
            st = None
            if gn_stats and (H * W) % 256 == 0:
                zb = self._zb.get(G)
                if zb is None:
                    zb = self._zb[G] = torch.zeros(G, self.cout, device=x.device, dtype=torch.float32)
                part = torch.empty(N * (H * W // 256) * self.cout * 2, device=x.device, dtype=torch.float32)
                st = (zb.data_ptr(), part.data_ptr())
            r = slab_conv2d(x.data_ptr(), wp.data_ptr(), y.data_ptr(), G, N // G, H, W, self.cin_p, self.cout,
                            x.device, stats=st)
            if r == 2:
                self.gn_part = (part, H * W // 256, 256)
            if r:
                return y
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
    def bwd(self, dy, x, theta, grads, G, need_dx, scratch=None, ws=None, defer=None):
        """dW -> grads rows (PyTorch layout at ``off``); returns dX ``[N, H, W, cin_p]`` (or None).  For the 1x1
        stride-2 projection the returned gradient is the half-resolution one of the even pixels (``res_grad_s2``
        adds it into the residual stream).  ``ws``: raw handle of the step's weight-gradient branch stream — the wgrad is
        forked onto it (the caller joins it before the optimizer) and only the data gradient stays on the chain.
        ``defer`` (a list, with ``ws``): the wgrad launch is appended to it instead, for the caller to issue on ws
        after ONE fork for several layers ([FORK-GROUP])."""
        if not self.hip:
            return self._torch_bwd(dy, x, theta, grads, G, need_dx)
        m = ops.ext()
        N, H, W, _ = x.shape
        B = N // G
        Ho, Wo = dy.shape[1:3]
        dy = dy.contiguous()
        kt, st_, pd = self.geometry()
        ns = m.conv_wgrad_nsplit_g(G, B, 1, H, W, self.cin_p, self.cout, kt, st_, pd, 0)
        ptab = self._pos_table(B, H, W, Ho, Wo, x.device)
        if ws is None:  # no branch: the whole backward on the current stream
            self._wgrad(m, x, dy, grads, G, B, H, W, ns, ptab, _stream())
        else:
            # the branch (raw stream ws) reads x / dy / ptab: they stay referenced until the caller joins it (no
            # record_stream: its deferred frees are not capturable and pile up on large steps)
            self._keep.extend((x, dy, ptab))
            if defer is not None:
                defer.append(lambda: self._wgrad(m, x, dy, grads, G, B, H, W, ns, ptab, ws))
            else:
                m.stream_fork(_stream(), ws)
                self._wgrad(m, x, dy, grads, G, B, H, W, ns, ptab, ws)
        st = _stream()
        if not need_dx:
            return None
        wt = self.wt
        if wt is None or wt[1] != G or wt[2] != theta.data_ptr():  # backward without a training forward
            wt = (self._wp(theta, G, True)[1], G, theta.data_ptr())
        wt = wt[0]
        self.wt = None
        if self.stride == 1:
            dx = torch.empty(N, H, W, self.cin_p, device=x.device, dtype=torch.bfloat16)
            if self.kt == 9 and self.pad == 1 and slab_conv2d(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, Ho,
                                                              Wo, self.cout, self.cin_p, x.device):
                return dx
            conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, 1, Ho, Wo, self.cout, self.cin_p, self.kt,
                     1, self.k - 1 - self.pad, 0, x.device)
            return dx
        if self.k == 3:
            # sub-pixel phases: 4 stride-1 convs over the dy grid with 1/2/2/4 taps, written straight into the
            # interleaved positions of dX (no zero-upsampled copy of dy: 4x fewer MACs, no memset / scatter)
            assert self.pad == 1 and H in (2 * Ho, 2 * Ho - 1) and W in (2 * Wo, 2 * Wo - 1), (H, W, Ho, Wo)
            dx = torch.empty(N, H, W, self.cin_p, device=x.device, dtype=torch.bfloat16)
            m.conv_dgrad_s2_g(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, 1, Ho, Wo, self.cout, self.cin_p,
                              self.kt, 1, H, W, st)
            return dx
        # 1x1 stride 2: only the even pixels were read -> half-resolution gradient W^T dY (res_grad_s2 scatters)
        assert self.k == 1 and self.pad == 0 and (H + 1) // 2 == Ho and (W + 1) // 2 == Wo
        sub = torch.empty(N, Ho, Wo, self.cin_p, device=x.device, dtype=torch.bfloat16)
        conv_fwd(dy.data_ptr(), wt.data_ptr(), sub.data_ptr(), G, B, 1, Ho, Wo, self.cout, self.cin_p, 1, 1,
                 0, 0, x.device)
        return sub

    def _wgrad(self, m, x, dy, grads, G, B, H, W, ns, ptab, st):
        branch = st != _stream()
        kt, st_, pd = self.geometry()
        part = torch.empty(ns * G * self.cout * kt * self.cin_p, device=x.device, dtype=torch.float32)
        if branch:  # allocated on the main stream's pool, used on the branch: held until the join
            self._keep.append(part)
        if self.cin_p == self.cin:
            m.conv_wgrad_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grads.data_ptr(), grads.stride(0),
                           self.off, G, B, 1, H, W, self.cin_p, self.cout, kt, st_, pd, 0, ns,
                           1.0, ptab.data_ptr(), st)
        else:  # channel-padded stem: full-width gradient, then the live input channels into the row
            full = torch.empty(G, self.cout * self.cin_p * kt, device=x.device, dtype=torch.float32)
            m.conv_wgrad_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), full.data_ptr(), full.stride(0), 0, G, B,
                           1, H, W, self.cin_p, self.cout, kt, st_, pd, 0, ns, 1.0,
                           ptab.data_ptr(), st)
            if branch:
                self._keep.append(full)
            with torch.cuda.stream(_external(st)) if branch else _nullctx():
                dst = grads[:, self.off:self.off + self.numel].view(G, self.cout, self.cin, self.kt)
                if self.fold:  # folded column 3 t + c -> PyTorch [co][c][t]
                    dst.copy_(full.view(G, self.cout, self.cin_p)[:, :, :self.kt * self.cin]
                              .view(G, self.cout, self.kt, self.cin).transpose(2, 3))
                else:
                    dst.copy_(full.view(G, self.cout, self.cin_p, self.kt)[:, :, :self.cin])

    def _pos_table(self, B, H, W, Ho, Wo, device):
        """Output-position table of the wgrad kernel: a function of the shape only, built once per (B, H, W) outside
        graph capture (inside a capture it is rebuilt by the captured launch, as before)."""
        key = (B, H, W)
        tab = self._ptabs.get(key)
        if tab is None:
            kt, st_, pd = self.geometry()
            tab = torch.empty(B * Ho * Wo, 2, device=device, dtype=torch.int32)
            ops.ext().conv_pos_table_g(tab.data_ptr(), B, 1, H, W, kt, st_, pd, 0, _stream())
            if not torch.cuda.is_current_stream_capturing():
                torch.cuda.current_stream().synchronize()  # shared with launches on other streams from now on
                self._ptabs[key] = tab
        return tab

    def _torch_bwd(self, dy, x, theta, grads, G, need_dx):
        w = self._wtorch(theta, G).detach().clone().requires_grad_(True)
        xx = x.detach().clone().requires_grad_(need_dx)
        with torch.enable_grad():
            y = self._torch_fwd(xx, w, G)
            outs = torch.autograd.grad(y, [w, xx] if need_dx else [w], dy.to(y.dtype))
        grads[:, self.off:self.off + self.numel].copy_(outs[0].reshape(G, -1))
        if not need_dx:
            return None
        dx = outs[1]
        if self.stride == 2 and self.k == 1:  # same contract as the HIP path: the even pixels only
            dx = dx[:, ::2, ::2].contiguous()
        return dx


# descriptor of pack.hip (PackDesc): int64 src_off, wp_off, wt_off; int32 cout, cin_p, cin_src, kt, blk_plain, blk_t,
# blk_plain1, slot[27]; 160 bytes with the struct's 8-B alignment
_PACK_DTYPE = np.dtype({"names": ["src_off", "wp_off", "wt_off", "cout", "cin_p", "cin_src", "kt", "blk_plain",
                                  "blk_t", "blk_plain1", "slot"],
                        "formats": ["<i8", "<i8", "<i8", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4", "<i4",
                                    ("<i4", 27)],
                        "offsets": [0, 8, 16, 24, 28, 32, 36, 40, 44, 48, 52], "itemsize": 160})
# 1x1 layers on the no-LDS row-batched pack (pack.hip k_pack_plain1; config 5 12.48 -> 12.24 s/round,
# profiles/r4_ab_pack1.txt); NIDT_PACK1=0: the per-row kernel (A/B)
_PACK1 = os.environ.get("NIDT_PACK1", "1") != "0"
# NIDT_PACK_FUSE=0: the optimizer never writes the forward images (k_pack_plain every step; A/B)
_PACK_FUSE = os.environ.get("NIDT_PACK_FUSE", "1") != "0"
# [PACK-WT] NIDT_PACK_WT=1: the optimizer also writes the next step's data-gradient images (optim.hip
# k_local_step_pack_wt over 64 x 64-channel tiles, bit-identical), so the step runs no k_pack_trans.  Off by default:
# slower than k_pack_trans overlapped on the weight-gradient side stream (CIFAR SubAvg -2.4 %, DisPFL -4.5 %; with
# 16-channel tiles -0.3 / -2.8 %; profiles/r6_pack_wt.txt) — the optimizer is on the critical path, the transposes are not
_PACK_WT = os.environ.get("NIDT_PACK_WT", "0") == "1"
# [FORK-GROUP] NIDT_FORK_GROUP=1: one fork of the weight-gradient branch per residual block (its wgrads and GroupNorm
# parameter sums issued together after the block's data-gradient chain) instead of one per layer (A/B)
_FORK_GROUP = os.environ.get("NIDT_FORK_GROUP", "1") == "1"
# [GN-RMASK] the GroupNorm+ReLU backward of each block's first norm recomputes its ReLU mask from t (no mask read);
# [OMASK] the residual-gradient pass applies the previous block's output ReLU mask, so the block's second norm and
# shortcut norm backward read none either.  NIDT_GN_RMASK=0 / NIDT_OMASK2D=0: the mask tensors (A/B)
_GN_RMASK = os.environ.get("NIDT_GN_RMASK", "1") != "0"
_OMASK2D = os.environ.get("NIDT_OMASK2D", "1") != "0"
# [GN-EPI] NIDT_GN_EPI=1: GroupNorm statistics from the epilogue of the slab conv that produces its input (layers whose
# 256-position conv blocks lie inside one sample: the 32x32 / 16x16 CIFAR maps, 64x64 / 32x32 Tiny), then a streaming
# apply pass (gn.hip k_gn_apply, 4.7-6.2 TB/s) instead of the one-block-per-sample k_gn_fwd.  Off by default: the
# statistics epilogue adds more to the conv (64-channel slab blocks 261 -> 331 us at DisPFL's 100 clients) than the
# apply pass saves (CIFAR SubAvg -1.7 %, DisPFL -1.8 %; profiles/r6_gn_epi.txt)
_GN_EPI = os.environ.get("NIDT_GN_EPI", "0") == "1"
# [STEM-FOLD] the 3-channel stem as a 1x1 conv over the window-folded input (img.hip k_img_fold); NIDT_STEM_FOLD=0:
# the channel-padded 9-tap conv (A/B)
_STEM_FOLD = os.environ.get("NIDT_STEM_FOLD", "1") != "0"


class WeightPacker:
    """Per-step bf16 MFMA images of every conv layer of G clients in two launches (``pack.hip`` ``pack_convs``): the
    forward image of each layer and, for training steps, the data-gradient image (taps in the layer's slot order).
    Buffers are persistent per launch shape, so a captured step's graph writes and reads the same memory."""

    def __init__(self, convs, device):
        self.convs, self.device = list(convs), torch.device(device)
        self._plans = {}
        self._descs = {}
        self.last = None   # (key, theta data_ptr, row stride) of the last pack() call
        # key -> (theta data_ptr, theta._version, wt) whose forward images (and with wt the data-gradient images too)
        # the optimizer wrote
        self.fresh = {}
        # keys own their buffers (the 3-D engine's per-row-group training keys): an image stays fresh across other
        # keys' packs; otherwise only the very next pack may reuse one
        self.keep_other_fresh = False
        self.fresh_hits = 0  # packs that reused optimizer-written forward images

    def _plan(self, G, train, key=None):
        key = (G, train) if key is None else key
        if key in self._plans:
            return self._plans[key]
        if ops.ext().pack_desc_bytes() != _PACK_DTYPE.itemsize:
            raise RuntimeError("pack.hip PackDesc layout changed")
        desc = np.zeros(len(self.convs), dtype=_PACK_DTYPE)
        off = nplain = nplain1 = ntrans = 0
        views = []
        m = ops.ext()
        for i, c in enumerate(self.convs):
            d = desc[i]
            d["src_off"], d["cout"], d["cin_p"], d["cin_src"], d["kt"] = c.off, c.cout, c.cin_p, c.cin, c.kt
            d["blk_plain"], d["blk_t"], d["blk_plain1"] = nplain, ntrans, nplain1
            if _PACK1 and c.kt == 1 and c.cin_p % 8 == 0:
                rows = m.pack1_rows_host(c.cin_p)
                nplain1 += (c.cout + rows - 1) // rows
            else:
                nplain += c.cout * m.pack_plain_chunks(c.cin_p, c.kt)
            n_img = G * c.cout * c.kt * c.cin_p
            d["wp_off"] = off
            vp = (off, (G, c.cout, c.kt, c.cin_p))
            off += n_img
            vt = None
            if train and c.need_dgrad:
                assert c.cin_p % 8 == 0 and c.cout % 8 == 0, "pack.hip k_pack_trans: 16-B channel pieces"
                d["wt_off"] = off
                vt = (off, (G, c.cin_p, c.kt, c.cout))
                off += n_img
                ntrans += ((c.cin_p + 63) // 64) * ((c.cout + 63) // 64) * c.kt
            else:
                d["wt_off"] = -1
            d["slot"][:c.kt] = c.slots
            views.append((vp, vt))
        lds = max([m.pack_plain_lds(c.cin_p, c.kt) for c in self.convs
                   if not (_PACK1 and c.kt == 1 and c.cin_p % 8 == 0)] + [4])
        buf = torch.empty(max(1, off), dtype=torch.bfloat16, device=self.device)
        tab = torch.from_numpy(desc.view(np.uint8).copy()).to(self.device)
        plan = (tab, (nplain, nplain1), ntrans, lds, buf, views)
        self._plans[key] = plan
        self._descs[key] = desc
        return plan

    def wt_ok(self):
        """[PACK-WT] applies: every layer's channels fit the tiled step's 16-B runs and its LDS tile."""
        return _PACK_WT and all(c.cout % 16 == 0 and c.cin_p % 8 == 0 and c.kt <= 9 for c in self.convs)

    def fused_plan(self, key, P, wt=False):
        """Plan of the optimizer step that writes ``key``'s forward images itself (``optim.hip`` ``local_opt_pack``):
        (descriptor table with plain-grid prefixes over every conv layer, its length, conv blocks, {start, length}
        table of the other parameter ranges of a P-wide row, its length, LDS bytes, the image buffer).  ``wt``: the
        tiled grid of ``local_opt_pack_wt`` (16 output x 64 input channels x all taps per block), which also writes
        the data-gradient images of ``key``'s layers."""
        fk = ("fused", key, int(P), bool(wt))
        plan = self._plans.get(fk)
        if plan is not None:
            return plan
        m = ops.ext()
        desc = self._descs[key].copy()
        nconv, spans = 0, []
        for i, c in enumerate(self.convs):
            desc[i]["blk_plain"] = nconv
            nconv += m.wt_tiles(c.cout, c.cin_p) if wt else c.cout * m.pack_plain_chunks(c.cin_p, c.kt)
            spans.append((c.off, c.off + c.numel))
        rest, pos = [], 0
        for a, b in sorted(spans) + [(int(P), int(P))]:
            while pos < a:  # the parameters between conv layers, 4096 per block
                n = min(4096, a - pos)
                rest.append((pos, n))
                pos += n
            pos = max(pos, b)
        lds = max((m.wt_tile_lds(c.kt) if wt else m.pack_plain_lds(c.cin_p, c.kt)) for c in self.convs)
        tab = torch.from_numpy(desc.view(np.uint8).copy()).to(self.device)
        rt = torch.tensor(rest if rest else [(0, 0)], dtype=torch.int64).to(self.device)
        plan = (tab, len(self.convs), nconv, rt, len(rest), lds, self._plans[key][4])
        self._plans[fk] = plan
        return plan

    def pack(self, theta, G, train, key=None, side=None):
        """Pack every layer for this step and hand each conv its views (``conv.wp`` / ``conv.wt``).  When the previous
        optimizer step wrote this key's forward images from these rows (``fresh``, see :meth:`fused_plan`; the rows
        unchanged since by torch ops: same ``_version``), only the dgrad transposes run."""
        key = (G, train) if key is None else key
        tab, (nplain, nplain1), ntrans, lds, buf, views = self._plan(G, train, key)
        f = self.fresh.pop(key, None)
        if (f is not None and f[:2] == (theta.data_ptr(), theta._version)
                and not torch.cuda.is_current_stream_capturing()):
            nplain = nplain1 = 0
            if len(f) > 2 and f[2]:  # [PACK-WT] the data-gradient images too
                ntrans = 0
            self.fresh_hits += 1
        if not self.keep_other_fresh:
            self.fresh.clear()  # an image is only ever reused by the very next pack
        self.last = (key, theta.data_ptr(), theta.stride(0)) if train else None
        if side is not None and ntrans:  # forward images here, dgrad transposes on the side stream (caller joins)
            if nplain or nplain1:
                ops.ext().pack_convs(tab.data_ptr(), len(self.convs), nplain, nplain1, 0, lds, theta.data_ptr(),
                                     theta.stride(0), G, buf.data_ptr(), _stream())
            ops.ext().stream_fork(_stream(), side)
            ops.ext().pack_convs(tab.data_ptr(), len(self.convs), 0, 0, ntrans, lds, theta.data_ptr(),
                                 theta.stride(0), G, buf.data_ptr(), side)
        elif nplain or nplain1 or ntrans:
            ops.ext().pack_convs(tab.data_ptr(), len(self.convs), nplain, nplain1, ntrans, lds, theta.data_ptr(),
                                 theta.stride(0), G, buf.data_ptr(), _stream())
        for c, (vp, vt) in zip(self.convs, views):
            c.wp = (buf[vp[0]:vp[0] + int(np.prod(vp[1]))].view(vp[1]), G, theta.data_ptr())
            c.wt = (buf[vt[0]:vt[0] + int(np.prod(vt[1]))].view(vt[1]), G, theta.data_ptr()) if vt else None

    def pack_into(self, theta, G, wp, wt):
        """Single-layer packing into caller-provided tensors (tests, standalone layers)."""
        tab, (nplain, nplain1), ntrans, lds, buf, views = self._plan(G, wt is not None, key=("one", G, wt is not None))
        ops.ext().pack_convs(tab.data_ptr(), 1, nplain, nplain1, ntrans, lds, theta.data_ptr(), theta.stride(0), G,
                             buf.data_ptr(), _stream())
        (vp, vt), = views
        wp.copy_(buf[vp[0]:vp[0] + wp.numel()].view(wp.shape))
        if wt is not None:
            wt.copy_(buf[vt[0]:vt[0] + wt.numel()].view(wt.shape))


class GroupNormG:
    """GroupNorm(32) over channels-last activations of G clients (per-client affine rows at off_w / off_b), with the
    block's residual add and ReLU fused into the forward and the ReLU mask into the backward.  HIP: ``gn.hip``
    (one block per sample, deterministic, graph-safe); CPU: the same math in fp32 torch ops."""

    def __init__(self, off_w, off_b, C, hip):
        self.off_w, self.off_b, self.C, self.hip = off_w, off_b, C, hip

    def _affine(self, theta):
        return theta[:, self.off_w:self.off_w + self.C], theta[:, self.off_b:self.off_b + self.C]

    def fwd(self, t, theta, G, res=None, relu=False, part=None):
        """t [N, H, W, C] -> (relu?(gn(t) + res) in t's dtype, saved statistics).  ``part`` ([GN-EPI]): the producing
        conv's per-block statistics (``GroupedConv.gn_part``): a streaming apply pass instead of the per-sample kernel."""
        N, H, W, C = t.shape
        if self.hip:
            t = t.contiguous()
            y = torch.empty_like(t)
            stats = torch.empty(N, GN_GROUPS, 2, device=t.device, dtype=torch.float32)
            r = res.contiguous() if res is not None else None
            if part is not None:
                pt, nb, bp = part
                ops.ext().gn_apply(t.data_ptr(), r.data_ptr() if r is not None else 0, pt.data_ptr(), nb, bp,
                                   theta.data_ptr(), theta.stride(0), self.off_w, self.off_b, y.data_ptr(),
                                   stats.data_ptr(), N, N // G, H * W, C, int(relu), _stream())
                return y, stats
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

    def bwd(self, dy, mask, t, saved, theta, grads, G, ws=None, defer=None, rmask=False):
        """dy [N, H, W, C] (fp32 or bf16), times (mask > 0) if a mask is given; writes the dgamma/dbeta rows,
        returns dt in t's dtype.  ``ws``: raw handle of the weight-gradient branch stream — the per-client dgamma/dbeta sum
        (off the data-gradient chain) is forked onto it.  ``rmask``: ``mask`` is this GroupNorm's own ReLU output
        (no residual), so the HIP kernel recomputes it from t and the statistics instead of reading it ([GN-RMASK])."""
        N, H, W, C = t.shape
        B = N // G
        if self.hip:
            dy = dy.contiguous()
            assert dy.dtype in (torch.float32, torch.bfloat16)
            dt = torch.empty_like(t)
            part = torch.empty(N, C, 2, device=t.device, dtype=torch.float32)
            if rmask and mask is not None and _GN_RMASK and ops.ext().gn_rm_ok(H * W, C):
                ops.ext().gn_bwd_rm(dy.data_ptr(), int(dy.dtype == torch.bfloat16), t.data_ptr(), saved.data_ptr(),
                                    theta.data_ptr(), theta.stride(0), self.off_w, self.off_b, dt.data_ptr(),
                                    part.data_ptr(), N, B, H * W, C, _stream())
            else:
                m = mask.contiguous() if mask is not None else None
                ops.ext().gn_bwd(dy.data_ptr(), int(dy.dtype == torch.bfloat16), m.data_ptr() if m is not None else 0,
                                 t.data_ptr(), saved.data_ptr(), theta.data_ptr(), theta.stride(0), self.off_w,
                                 dt.data_ptr(), part.data_ptr(), N, B, H * W, C, _stream())
            if ws is None:
                ops.ext().gn_param_grads(part.data_ptr(), G, B, C, grads.data_ptr(), grads.stride(0), self.off_w,
                                         self.off_b, _stream())
                return dt
            GroupedConv._keep.append(part)

            def side():
                ops.ext().gn_param_grads(part.data_ptr(), G, B, C, grads.data_ptr(), grads.stride(0), self.off_w,
                                         self.off_b, ws)
            if defer is not None:  # [FORK-GROUP] issued by the caller after its one fork
                defer.append(side)
            else:
                ops.ext().stream_fork(_stream(), ws)
                side()
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
    """The forward/backward graph of ``customized_resnet18`` (32x32 CIFAR, avg_pool2d(4) over the final 4x4 map) and
    ``tiny_resnet18`` (64x64 Tiny-ImageNet, AdaptiveAvgPool2d over the final 8x8 map) for G clients at once — the two
    share every parameter and differ only in input size and pooling window, which is the whole final map in both
    (see module docstring).  ``mean``/``std``: the dataset's Normalize constants."""

    def __init__(self, players: ParamLayout, device, hip=None, mean=CIFAR_MEAN, std=CIFAR_STD):
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
        self.stem.fold = (self.hip and _STEM_FOLD and self.stem.k == 3 and self.stem.stride == 1 and self.stem.pad == 1
                          and self.stem.cin * self.stem.kt <= self.stem.cin_p)
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
        self.mean, self.std = tuple(float(v) for v in mean), tuple(float(v) for v in std)
        m_ = torch.tensor(self.mean, dtype=torch.float32).view(1, 1, 1, 3)
        s_ = torch.tensor(self.std, dtype=torch.float32).view(1, 1, 1, 3)
        self.norm_scale = (1.0 / (255.0 * s_)).to(self.device)
        self.norm_shift = (-m_ / s_).to(self.device)
        convs = [self.stem] + [b[k] for b in self.blocks for k in ("c1", "c2", "cs") if k in b]
        self.packer = WeightPacker(convs, self.device) if self.hip else None

    # ------------------------------------------------------------------ input
    def input(self, x8, idx, aug=None):
        """Gather + (train-time augmentation) + normalise + channel-pad the uint8 HWC images ``x8[idx]`` into the
        stem's activation [N, H, W, cin_p].  ``aug`` = (seed_dev, seed_base, cids_dev, cids, B) or None; the HIP path
        is one fused kernel (``img.hip``), the CPU twin draws the same crops/flips (:func:`aug_draws`)."""
        N = idx.numel()
        H, W = int(x8.shape[1]), int(x8.shape[2])
        cp = self.stem.cin_p
        if self.hip:
            out = torch.empty(N, H, W, cp, device=self.device, dtype=torch.bfloat16)
            idx32 = idx if idx.dtype == torch.int32 else idx.int()
            fn = ops.ext().img_input_fold if self.stem.fold else ops.ext().img_input  # [STEM-FOLD]
            if aug is not None:
                seed_dev, seed_base, cids_dev, _, B = aug
                fn(x8.data_ptr(), idx32.data_ptr(), out.data_ptr(), N, H, W, cp, *self.mean, *self.std, 1, AUG_PAD,
                   seed_dev.data_ptr(), int(seed_base), cids_dev.data_ptr(), B, _stream())
            else:
                fn(x8.data_ptr(), idx32.data_ptr(), out.data_ptr(), N, H, W, cp, *self.mean, *self.std, 0, AUG_PAD, 0,
                   0, 0, 1, _stream())
            return out
        img = x8.index_select(0, idx.long().to(x8.device))
        if aug is not None:
            seed_dev, seed_base, _, cids, B = aug
            oy, ox, fl = aug_draws(int(seed_base) + int(seed_dev.reshape(-1)[0]), cids, B)
            img = augment_u8(img, oy, ox, fl)
        x = img.float() * self.norm_scale.to(img.device) + self.norm_shift.to(img.device)
        if cp != 3:
            x = F.pad(x, (0, cp - 3))
        return x.to(self.act).contiguous()

    # ------------------------------------------------------------------ forward
    def forward(self, x, theta, G, train=False):
        a, saved = self.features(x, theta, G, train)
        N, H, W, C = a.shape
        pooled = a.float().view(N, H * W, C).mean(1)  # avg_pool2d(4) on 4x4 (CIFAR) / adaptive 1x1 on 8x8 (Tiny)
        B = N // G
        lw = theta[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat)
        lb = theta[:, self.lb_off:self.lb_off + self.ncls]
        # the 512 -> K head as broadcast multiply-reduce, not bmm: BLAS calls keep library workspaces that a
        # replayed hipGraph would share with eager work
        logits = (pooled.view(G, B, 1, C) * lw.view(G, 1, self.ncls, C)).sum(-1) + lb.view(G, 1, self.ncls)
        return logits.view(N, self.ncls), pooled, saved

    def features(self, x, theta, G, train=False, side=None):
        """Stem + the four stages: the final activation map [N, H, W, 512] and the saved tensors of the backward."""
        saved = []
        packed = self.packer is not None
        if packed:
            self.packer.pack(theta, G, train, key=(G, x.shape[0] // G, train), side=side)
        t = self.stem.fwd(x, theta, G, train, packed)
        a, st = self.stem_gn.fwd(t, theta, G, relu=True)
        if train:  # evaluation keeps no activations alive (only the backward reads them)
            saved.append((x, t, st, a))
        for blk in self.blocks:
            xin = a
            t1 = blk["c1"].fwd(xin, theta, G, train, packed, gn_stats=_GN_EPI)
            h1, s1 = blk["n1"].fwd(t1, theta, G, relu=True, part=blk["c1"].gn_part)
            t2 = blk["c2"].fwd(h1, theta, G, train, packed, gn_stats=_GN_EPI)
            if "cs" in blk:
                ts = blk["cs"].fwd(xin, theta, G, train, packed)
                ysc, ss = blk["ns"].fwd(ts, theta, G)
            else:
                ts, ss, ysc = None, None, xin
            a, s2 = blk["n2"].fwd(t2, theta, G, res=ysc, relu=True, part=blk["c2"].gn_part)
            if train:
                saved.append((xin, t1, s1, h1, t2, s2, ts, ss, a))
        return a, saved

    def _fused_head(self, theta):
        return (self.hip and self.lw_off % 2 == 0 and theta.stride(0) % 2 == 0 and self.ncls <= 256
                and self.feat <= 512 and os.environ.get("NIDT_CLS_HEAD", "1") != "0")

    def _head_train(self, a, theta, grads, y, G, B):
        """Classifier head + CrossEntropy forward/backward: per-client mean losses [G], the head's gradient rows,
        and the bf16 input gradient of the final map.  HIP: two launches (``head.hip`` ``cls_head_train``)."""
        N, H, W, C = a.shape
        if self._fused_head(theta):
            dev = a.device
            pooled = torch.empty(N, C, device=dev, dtype=torch.float32)
            dlog = torch.empty(N, self.ncls, device=dev, dtype=torch.float32)
            lossn = torch.empty(N, device=dev, dtype=torch.float32)
            losses = torch.empty(G, device=dev, dtype=torch.float32)
            da = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
            yl = y if y.dtype == torch.int64 else y.long()
            ops.ext().cls_head_train(a.contiguous().data_ptr(), theta.data_ptr(), theta.stride(0), self.lw_off,
                                     self.lb_off, yl.contiguous().data_ptr(), G, B, H * W, C, self.ncls,
                                     pooled.data_ptr(), dlog.data_ptr(), lossn.data_ptr(), losses.data_ptr(),
                                     grads.data_ptr(), grads.stride(0), da.data_ptr(), _stream())
            return losses, da
        pooled = a.float().view(N, H * W, C).mean(1)
        lw = theta[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat)
        lb = theta[:, self.lb_off:self.lb_off + self.ncls]
        logits = (pooled.view(G, B, 1, C) * lw.view(G, 1, self.ncls, C)).sum(-1) + lb.view(G, 1, self.ncls)
        logp = torch.log_softmax(logits, dim=-1)
        yl = y.long().view(G, B)
        losses = -logp.gather(2, yl.unsqueeze(2)).squeeze(2).mean(1)
        # softmax - onehot (scatter, not F.one_hot: its range check syncs the host, which a graph capture forbids)
        dlog = logp.exp().scatter_add(2, yl.unsqueeze(2), torch.full_like(logp[..., :1], -1.0)) / B  # [G, B, K]
        grads[:, self.lw_off:self.lw_off + self.ncls * self.feat].view(G, self.ncls, self.feat).copy_(
            (dlog.view(G, B, self.ncls, 1) * pooled.view(G, B, 1, self.feat)).sum(1))
        grads[:, self.lb_off:self.lb_off + self.ncls].copy_(dlog.sum(1))
        dpool = (dlog.view(G, B, self.ncls, 1) * lw.view(G, 1, self.ncls, self.feat)).sum(2).view(G * B, 1, self.feat)
        # bf16 residual-gradient stream on the HIP path (res_grad writes bf16; re-read by every GroupNorm backward)
        da = (dpool / float(H * W)).expand(N, H * W, C).reshape(N, H, W, C).to(self.act).contiguous()
        return losses, da

    # ------------------------------------------------------------------ train step
    def train_step(self, theta, grads, x, y, G, B):
        # the branch stream (see _wgrad_stream) also takes the dgrad-image transposes, overlapped with the forward
        ws = self._wgrad_stream(G, B, x.shape[1] * x.shape[2])
        a, saved = self.features(x, theta, G, train=True, side=ws)
        losses, da = self._head_train(a, theta, grads, y, G, B)
        if ws is not None:
            ops.ext().stream_fork(ws, _stream())  # the dgrad images (pack_trans on the branch)
        # [OMASK] dm: da is already multiplied by this block's output ReLU mask (a > 0) — the previous residual-gradient
        # pass applied it — so the block's n2 / shortcut GroupNorm backward read no mask tensor
        dm = False
        for blk, sv in zip(reversed(self.blocks), reversed(saved[1:])):
            xin, t1, s1, h1, t2, s2, ts, ss, a = sv
            am = None if dm else a
            dfr = [] if (ws is not None and _FORK_GROUP) else None
            dt2 = blk["n2"].bwd(da, am, t2, s2, theta, grads, G, ws=ws, defer=dfr)
            dh1 = blk["c2"].bwd(dt2, h1, theta, grads, G, True, ws=ws, defer=dfr)
            dt1 = blk["n1"].bwd(dh1, h1, t1, s1, theta, grads, G, ws=ws, defer=dfr, rmask=True)
            dx1 = blk["c1"].bwd(dt1, xin, theta, grads, G, True, ws=ws, defer=dfr)
            dx2 = None
            if "cs" in blk:
                dts = blk["ns"].bwd(da, am, ts, ss, theta, grads, G, ws=ws, defer=dfr)
                dx2 = blk["cs"].bwd(dts, xin, theta, grads, G, True, ws=ws, defer=dfr)
            if dfr:  # [FORK-GROUP] the block's weight-gradient work: one fork, then every launch on the branch
                ops.ext().stream_fork(_stream(), ws)
                for f in dfr:
                    f()
            half = dx2 is not None and blk["cs"].stride == 2  # 1x1 stride-2 projection: even-pixel gradient
            if self.hip:
                out = torch.empty(dx1.shape, device=dx1.device, dtype=torch.bfloat16)
                om = xin.data_ptr() if _OMASK2D else 0  # [OMASK] the previous block's (or the stem's) ReLU output
                if half:
                    Nn, Hh, Ww, Cc = dx1.shape
                    ops.ext().res_grad_s2_om(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr(), om, Nn, 1, Hh, Ww, Cc, 1,
                                             _stream())
                else:
                    ops.ext().res_grad_om(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr() if dx2 is not None else 0,
                                          0 if dx2 is not None else da.data_ptr(),
                                          0 if (dx2 is not None or dm) else a.data_ptr(), om, out.numel(),
                                          1 | (2 if da.dtype == torch.bfloat16 else 0), _stream())
                da = out
                dm = bool(om)
            elif half:
                da = dx1.float().clone()
                da[:, ::2, ::2] += dx2.float()
            else:
                da = dx1.float() + (dx2.float() if dx2 is not None else da * (a > 0))
        x0, t0, st0, a0 = saved[0]
        dt0 = self.stem_gn.bwd(da, None if dm else a0, t0, st0, theta, grads, G, ws=ws)
        self.stem.bwd(dt0, x0, theta, grads, G, False, ws=ws)
        if ws is not None:
            ops.ext().stream_fork(ws, _stream())  # join: the optimizer reads every weight gradient
            GroupedConv._keep.clear()  # later reuse of their memory on this stream is ordered after the branch
        return losses.detach()

    def _wgrad_stream(self, G, B, HW):
        """Weight-gradient branch stream of one launch shape, or None (CPU; NIDT_WGRAD_STREAM=0; graph capture).
        The branch takes the weight gradients, the GroupNorm parameter sums and the dgrad-image transposes (those
        overlapped with the forward), i.e. everything off the data-gradient chain.

        Measured (profiles/r5_wgrad_stream.txt): CIFAR SubAvg 0.749 -> 0.714 s/round, CIFAR DisPFL 3.785 -> 3.59,
        Tiny SubAvg 2.544 -> 2.435, Tiny DisPFL 18.6 -> 18.4.  (A first version pinned the branch's inputs with
        record_stream: Tiny DisPFL went to 26-28 s as the deferred frees piled up; the branch now holds plain
        references until its join.)"""
        if not self.hip or os.environ.get("NIDT_WGRAD_STREAM", "1") == "0":
            return None
        if torch.cuda.is_current_stream_capturing():  # captured steps: one stream
            return None
        if not hasattr(self, "_ws"):
            self._ws = {}
        if (G, B) not in self._ws:
            self._ws[(G, B)] = torch.cuda.Stream(device=self.device)
        return self._ws[(G, B)].cuda_stream  # raw handle: forks / joins through ops.stream_fork

    def eval_logits(self, theta, x, G):
        logits, _, _ = self.forward(x, theta, G)
        return logits


class ResNetHipEngine:
    """Engine API of :class:`~.executor.HipEngine` (train_step / eval_logits / local_opt / saliency_acc) for the
    client-batched ResNet-18-GN on uint8 HWC images: CIFAR-10/100 ``[N, 32, 32, 3]`` (``customized_resnet18``) or
    Tiny-ImageNet ``[N, 64, 64, 3]`` (``tiny_resnet18``).  ``augment``: the reference's train-time RandomCrop(pad 4)
    + RandomHorizontalFlip, drawn on device per (step, client, sample) and fused into the input stage."""
    sample_fields = ("x8", "labels")

    @property
    def input_shape(self):
        n, h, w, c = self.x8.shape  # NHWC uint8 store
        return (c, h, w)

    def __init__(self, template_model, images_u8, labels, device, hip=None, mean=None, std=None, augment=True):
        self.device = torch.device(device)
        self.players = ParamLayout.from_tensors(list(template_model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(template_model.named_buffers()))
        assert self.blayers.total == 0, "GroupNorm ResNet carries no buffers"
        hw = int(images_u8.shape[1])
        if mean is None:
            mean, std = (TINY_MEAN, TINY_STD) if hw == 64 else (CIFAR_MEAN, CIFAR_STD)
        self.net = GroupedResNet18GN(self.players, self.device, hip=hip, mean=mean, std=std)
        self.x8 = images_u8.to(self.device)
        self.labels = labels.to(self.device)
        self.augment = bool(augment)
        if self.net.hip:
            ops.ext()  # fail loudly on a GPU box without the extension
        self.supports_graphs = self.device.type == "cuda"
        # replaying captured steps measured ~3 % slower than eager launches for this engine (CIFAR SubAvg 0.810 vs
        # 0.786 s/round with the graphs reused across rounds, Tiny 1.969 vs 1.965 s; profiles/r4_graphs_ab.txt):
        # eager unless FLConfig.hip_graphs=True
        self.graphs_default = False
        self.graph_cache_limit = 24  # each captured step holds its own activation pool
        self._opt = None
        self._cid_cache = {}

    def _cids_dev(self, cids):
        key = tuple(int(c) for c in cids)
        ct = self._cid_cache.get(key)
        if ct is None:  # one upload per client group (in the eager first step of a shape, before any capture)
            ct = torch.tensor(key, dtype=torch.int32, device=self.device)
            self._cid_cache[key] = ct
        return ct

    accepts_cids_dev = True  # see HipEngine.train_step

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True,
                   cids_dev=None):
        aug = None
        if self.augment and seed_dev is not None:
            cids = list(range(G)) if cids is None else [int(c) for c in cids]
            aug = (seed_dev, int(seed), cids_dev if cids_dev is not None else self._cids_dev(cids), cids, B)
        x = self.net.input(self.x8, idx, aug)
        y = self.labels.index_select(0, idx.long())
        return self.net.train_step(theta, grads, x, y, G, B)

    def eval_logits(self, theta, bufs, idx, G, B):
        with torch.no_grad():
            if self.net.packer is not None:
                self.net.packer.fresh.clear()
            x = self.net.input(self.x8, idx)
            return self.net.eval_logits(theta, x, G).float()

    def _delegate(self):
        if self._opt is None:
            from .executor import HipEngine, TorchEngine
            self._opt = HipEngine.__new__(HipEngine) if self.net.hip else TorchEngine.__new__(TorchEngine)
            if self.net.hip:
                self._opt.m = ops.ext()
        return self._opt

    # [PACK-FUSE] the runner may ask the optimizer step to write the next step's forward images (pack_next: the same
    # rows train again right after, with nothing else touching them in between)
    fused_pack = True

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False,
                  pack_next=False):
        from .executor import HipEngine, TorchEngine
        pk = self.net.packer
        if (pack_next and pk is not None and pk.last is not None and _PACK_FUSE
                and pk.last[1:] == (theta.data_ptr(), theta.stride(0)) and pk.last[0][0] == theta.shape[0]
                and not torch.cuda.is_current_stream_capturing()):
            key = pk.last[0]
            wt = pk.wt_ok()
            HipEngine.local_opt_pack(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm,
                                     pk.fused_plan(key, theta.shape[1], wt=wt), lr_dev=lr_dev, keep_grad=keep_grad,
                                     wt=wt)
            pk.fresh = {key: (theta.data_ptr(), theta._version, wt)}
            return
        if pk is not None:
            pk.fresh.clear()
        cls = HipEngine if self.net.hip else TorchEngine
        cls.local_opt(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=lr_dev,
                      keep_grad=keep_grad)

    def saliency_acc(self, theta, grads, score, alpha):
        from .executor import HipEngine, TorchEngine
        if self.net.packer is not None:
            self.net.packer.fresh.clear()
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
