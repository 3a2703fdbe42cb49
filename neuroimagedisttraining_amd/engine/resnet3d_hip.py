"""Client-batched 3D ResNet (BASELINE config 5: Bottleneck ResNet-50 on full-resolution 1x121x145x121 volumes) on the
gfx950 kernels: G clients' local steps in one lockstep pass over rows of the flat ``[C, P]`` parameter matrix.

* every bottleneck convolution — 1x1x1 (the GEMM path: ``conv_fwd_g`` with one tap; batched library GEMMs opt-in,
  :func:`gemm_1x1`), 3x3x3 at stride 1 and 2, the 1x1x1 stride-2 projections — runs on the client-grouped LDS-DMA
  implicit-GEMM kernels of ``conv3d.hip``, with
  every layer's bf16 MFMA images packed in two launches per step (``pack.hip``); data gradients: stride 1 = the
  same kernels on tap-flipped transposed weights, 3x3x3 stride 2 = eight sub-pixel phase convs over the dy grid
  written straight into dX (``conv_dgrad_s2_g``: 8x fewer MACs than the zero-upsampled form, no memset or crop),
  1x1x1 stride 2 = the half-resolution gradient of the even voxels added by ``res_grad_s2``; weight gradients the
  position-table wgrad kernel straight into the client's gradient row;
* BatchNorm3d (train and eval mode, per-client statistics / affine / running stats) is ``bnr.hip``, with the
  residual add and ReLU fused into the apply and the ReLU mask into the backward;
* the stem (7x7x7 stride-2 conv with ONE input channel, BN, ReLU, 3x3x3 max-pool) is ``stem.hip``: the uint8
  volume in polyphase form turns the stride-2 7^3 conv into a stride-1 4^3 conv over 8 phase channels (512 MFMA
  k-slots), fused with the per-block BN statistics (merged by ``bn.hip``'s finalize), a BN+ReLU+pool kernel that
  keeps a uint8 argmax, and the backward (unpool + ReLU mask + BN sums, the BN coefficients, an MFMA weight
  gradient over x-shifted phase rows); the CPU twin (``hip=False``) is the same graph in PyTorch;
* the head (global average pool, fc -> 1, BCE) is a few batched torch ops.

Reference model: ``fedml_api/model/cv/salient_models.py:8-139`` (3D ResNet blocks); the 4-stage ResNet-50 is this
framework's config-5 model (``models/resnet3d.py``).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import ops
from .flat import ParamLayout

BN_EPS = 1e-5
BN_MOM = 0.1


_stream = ops.stream

_BRANCH_KEEP = []  # tensors read by the weight-gradient branch of the step in flight (released at its join)


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
# 1x1x1 stride-1 convs (forward and data gradient) are plain per-client GEMMs [M, Cin] x [Cin, Cout] on channels-last
# rows; NIDT_R3D_BLAS=1 runs them as batched library GEMMs (torch.bmm) instead of the general LDS-DMA conv kernel
# (which spends ~7 VALU per MFMA on per-tap addressing, 14 % MFMA busy, profiles/r4_pmc_config5.txt).  OFF by
# default: at config-5 scale (32 clients x 142 k positions x 256 channels, > 2^31 elements per batched operand) the
# run hung with the GPU left in a memory-fault state (profiles/r4_blas_1x1_fault.txt); the engine tests at small
# shapes pass.  Operands below 2^31 bytes only, even when enabled.
_BLAS_1X1 = os.environ.get("NIDT_R3D_BLAS", "0") == "1"


# 1x1x1 stride-1 convs (forward, data gradient, and the stride-2 projection's half-resolution data gradient) on the
# streaming per-client GEMM kernel gemm1x1.hip (K <= 512); NIDT_R3D_G1=0 keeps them on the general conv kernel (A/B)
_G1 = os.environ.get("NIDT_R3D_G1", "1") != "0"


# NIDT_R3D_G1STATS=0: the following BatchNorm reads its training statistics in a pass of its own (k_bnr_partial)
# instead of from the GEMM epilogue (A/B)
_G1STATS = os.environ.get("NIDT_R3D_G1STATS", "1") != "0"


def g1_gemm(x, w, out, G, K, N, stats=False):
    """out[g] = x[g] @ w[g]^T on channels-last rows with the hand-written streaming GEMM (``gemm1x1.hip``); False
    (nothing launched) when the shape has no kernel (K >= 1024) or the switch is off.  ``stats``: also the BatchNorm
    chunk partials of ``out`` (returned as ``(part, nchunk)`` instead of True)."""
    m = ops.ext()
    if not _G1 or not m.gemm1x1_ok(K, N):
        return False
    Mg = x.numel() // (G * K)
    assert x.numel() == G * Mg * K and out.numel() == G * Mg * N and x.is_contiguous() and out.is_contiguous()
    part = None
    if stats and _G1STATS:
        nch = m.gemm1x1_chunks(G, Mg, K, N)
        part = (torch.empty(nch, G, N, 2, device=x.device, dtype=torch.float32), nch)
    m.gemm1x1_g(x.data_ptr(), w.data_ptr(), out.data_ptr(), G, Mg, K, N, part[0].data_ptr() if part else 0,
                _stream())
    return part if part else True


def gemm_1x1(x, w, out, G):
    """out[g] = x[g] @ w[g]^T for channels-last x [G*B, D, H, W, K] and a packed image w [G, N, 1, K] (bf16, fp32
    accumulation), written into out [G*B, D, H, W, N].  False (nothing launched) when an operand reaches 2^31 bytes."""
    K, N = x.shape[-1], out.shape[-1]
    if max(x.numel(), out.numel()) * 2 >= (1 << 31):
        return False
    torch.bmm(x.view(G, -1, K), w.view(G, N, K).transpose(1, 2), out=out.view(G, -1, N))
    return True


def slab_conv(x_ptr, w_ptr, y_ptr, G, B, D, H, W, Cin, Cout, pad, device, bias=0, stats=0):
    """3x3x3 stride-1 conv through the kd-slab union kernel (``k_conv_fwd_slab``) when the shape is eligible (its
    band unions fit the kernel's LDS); returns False otherwise.  The union table is a function of the shape only and
    is built once per (B, D, H, W, pad).  ``stats``: [G, nPB, Cout, 2] per-256-position-block BatchNorm statistics
    of the output from the epilogue (needs a ``bias`` [G, Cout], zeros for the bias-free ResNet convs)."""
    m = ops.ext()
    if not m.conv3d_fwd_slab_pick(G, B, D, H, W, Cin, Cout, pad):
        return False
    key = (str(device), B, D, H, W, pad)
    tab = _SLAB_TABS.get(key)
    if tab is None:
        tab = torch.empty(m.conv3d_fwd_slab_table_size(B, D, H, W, pad), device=device, dtype=torch.int32)
        m.conv3d_fwd_slab_table(tab.data_ptr(), B, D, H, W, pad, _stream())
        if torch.cuda.is_current_stream_capturing():  # built inside a capture: that graph's memory, not cached
            m.conv3d_fwd_slab(x_ptr, w_ptr, bias, 0, y_ptr, stats, G, B, D, H, W, Cin, Cout, pad, tab.data_ptr(),
                              _stream())
            return True
        torch.cuda.current_stream().synchronize()  # shared with launches on other streams from now on
        _SLAB_TABS[key] = tab
    m.conv3d_fwd_slab(x_ptr, w_ptr, bias, 0, y_ptr, stats, G, B, D, H, W, Cin, Cout, pad, tab.data_ptr(), _stream())
    return True


# [SLAB-STATS] the BatchNorm after a slab-kernel 3x3x3 conv takes its training statistics from the conv epilogue
# (per-block mean / M2, merged by bn.hip's finalize) instead of a k_bnr_partial pass; NIDT_R3D_SLAB_STATS=0: A/B
_SLAB_STATS = os.environ.get("NIDT_R3D_SLAB_STATS", "1") != "0"
_ZERO_BIAS = {}


def _zero_bias(G, C, device):
    key = (G, C, str(device))
    z = _ZERO_BIAS.get(key)
    if z is None:
        z = _ZERO_BIAS[key] = torch.zeros(G, C, device=device, dtype=torch.float32)
    return z


# 3x3x3 stride-1 weight gradients with the union-staged B operand of the AlexNet3D conv2-5 kernels (k_conv_wgrad_slab:
# one kd-slab union per 64 channels, or k_conv_wgrad_tri: one three-tap union per (kd, kh)) where the shape is eligible;
# NIDT_R3D_WG_UNION=0 keeps every layer on the position-table kernel k_conv_wgrad_dma (A/B)
_WG_UNION = os.environ.get("NIDT_R3D_WG_UNION", "1") != "0"
_WG_TABS = {}


def union_wgrad(x, dy, grads, off, G, B, D, H, W, cin, cout, pad):
    """dW of a 3x3x3 stride-1 conv into the gradient rows through k_conv_wgrad_slab / k_conv_wgrad_tri; False
    (nothing launched) when neither applies."""
    m = ops.ext()
    if not _WG_UNION:
        return False
    if m.conv3d_wgrad_slab_pick(G, B, D, H, W, cin, cout, pad):
        kind, ns = "slab", m.conv3d_wgrad_slab_nsplit(G, B, D, H, W, cin, cout, pad)
    elif m.conv3d_wgrad_tri_pick(G, B, D, H, W, cin, cout, pad):
        kind, ns = "tri", m.conv3d_wgrad_tri_nsplit(G, B, D, H, W, cin, cout, pad)
    else:
        return False
    key = (kind, str(x.device), B, D, H, W, pad)
    tab = _WG_TABS.get(key)
    if tab is None:
        size = (m.conv3d_wgrad_slab_table_size if kind == "slab" else m.conv3d_wgrad_tri_table_size)(B, D, H, W, pad)
        tab = torch.empty(size, device=x.device, dtype=torch.int32)
        (m.conv3d_wgrad_slab_table if kind == "slab" else m.conv3d_wgrad_tri_table)(tab.data_ptr(), B, D, H, W, pad,
                                                                                     _stream())
        if not torch.cuda.is_current_stream_capturing():
            torch.cuda.current_stream().synchronize()  # shared with launches on other streams from now on
            _WG_TABS[key] = tab
        else:
            _BRANCH_KEEP.append(tab)
    part = torch.empty(ns * G * cout * 27 * cin, device=x.device, dtype=torch.float32)
    fn = m.conv3d_wgrad_slab if kind == "slab" else m.conv3d_wgrad_tri
    fn(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grads.data_ptr(), grads.stride(0), off, G, B, D, H, W, cin, cout,
       pad, ns, 1.0, tab.data_ptr(), _stream())
    return True


class GConv3:
    """Client-grouped Conv3d (k = 1 or 3, stride 1/2, no bias) on channels-last ``[N, D, H, W, C]`` bf16.  Weight
    images come from the network's :class:`~.resnet2d_hip.WeightPacker` (two launches per step for all layers;
    the dgrad image in this layer's tap-slot order)."""

    def __init__(self, off, cout, cin, k, stride, pad, hip=True):
        assert k in (1, 3) and cin % 64 == 0 and cout % 64 == 0, (k, cin, cout)
        self.off, self.cout, self.cin, self.k, self.stride, self.pad = off, cout, cin, k, stride, pad
        self.hip = hip
        self.kt = 27 if k == 3 else 1
        self.cin_p = cin
        self.need_dgrad = True
        self.numel = cout * cin * self.kt
        self.slots = list(ops.ext().conv_tap_slots(self.kt, stride)) if hip else None
        self.wp = self.wt = None
        self._ptabs = {}
        self._part = None  # BatchNorm partials of the last forward output (fwd(stats=True) on the GEMM path)
        self._bstats = None  # ... on the slab path: (per-block stats, nPB, block size, positions per client)

    def take_bstats(self):
        """The per-block BatchNorm statistics of the last ``fwd(stats=True)`` output on the slab path, or None."""
        p, self._bstats = self._bstats, None
        return p

    def take_part(self):
        """The BatchNorm chunk partials of the last ``fwd(stats=True)`` output, or None (then the BN computes its
        own); cleared by the call."""
        p, self._part = self._part, None
        return p

    def out_dims(self, d, h, w):
        f = lambda n: (n + 2 * self.pad - self.k) // self.stride + 1  # noqa: E731
        return f(d), f(h), f(w)

    def _wp(self, theta, G, transposed):
        """Standalone packing of this layer (tests); the network packs every layer at once."""
        from .resnet2d_hip import WeightPacker
        wp = torch.empty(G, self.cout, self.kt, self.cin, device=theta.device, dtype=torch.bfloat16)
        wt = torch.empty(G, self.cin, self.kt, self.cout, device=theta.device, dtype=torch.bfloat16) \
            if transposed else None
        WeightPacker([self], theta.device).pack_into(theta, G, wp, wt)
        return wp, wt

    def _torch_fwd(self, x, w, G):
        N, D, H, W, C = x.shape
        B = N // G
        xc = x.reshape(G, B, D, H, W, C).permute(1, 0, 5, 2, 3, 4).reshape(B, G * C, D, H, W)
        y = F.conv3d(xc, w.reshape(G * self.cout, self.cin, self.k, self.k, self.k), stride=self.stride,
                     padding=self.pad, groups=G)
        return y.view(B, G, self.cout, *y.shape[2:]).permute(1, 0, 3, 4, 5, 2).reshape(N, *y.shape[2:], self.cout)

    def fwd(self, x, theta, G, train=False, packed=False, stats=False):
        self._part = None
        self._bstats = None
        N, D, H, W, C = x.shape
        if not self.hip:  # CPU twin (its BN output may be a permuted view)
            return self._torch_fwd(x, theta[:, self.off:self.off + self.numel], G)
        assert C == self.cin and N % G == 0 and x.is_contiguous()
        Do, Ho, Wo = self.out_dims(D, H, W)
        if not packed:
            wp, wt = self._wp(theta, G, train)
            self.wp = (wp, G, theta.data_ptr())
            self.wt = (wt, G, theta.data_ptr()) if wt is not None else None
        wp = self.wp[0]
        y = torch.empty(N, Do, Ho, Wo, self.cout, device=x.device, dtype=torch.bfloat16)
        if self.kt == 1 and self.stride == 1:
            r = g1_gemm(x, wp, y, G, self.cin, self.cout, stats=stats)
            if r is not False:
                self._part = r if isinstance(r, tuple) else None
                return y
        if self.kt == 1 and self.stride == 1 and _BLAS_1X1 and gemm_1x1(x, wp, y, G):
            return y
        if self.kt == 27 and self.stride == 1:
            bst, bias = None, 0
            if stats and _SLAB_STATS:
                Mg = (N // G) * Do * Ho * Wo
                npb = (Mg + 255) // 256
                bst = (torch.empty(G, npb, self.cout, 2, device=x.device, dtype=torch.float32), npb, 256, Mg)
                bias = _zero_bias(G, self.cout, x.device).data_ptr()
            if slab_conv(x.data_ptr(), wp.data_ptr(), y.data_ptr(), G, N // G, D, H, W, self.cin, self.cout, self.pad,
                         x.device, bias=bias, stats=bst[0].data_ptr() if bst is not None else 0):
                self._bstats = bst
                return y
        conv_fwd(x.data_ptr(), wp.data_ptr(), y.data_ptr(), G, N // G, D, H, W, self.cin, self.cout,
                 self.kt, self.stride, self.pad, self.pad if self.kt == 27 else 0, x.device)
        return y

    def bwd(self, dy, x, theta, grads, G, need_dx=True, ws=None):
        """dW -> grads rows; returns dX (None without ``need_dx``).  ``ws``: stream of the step's weight-gradient
        branch (the wgrad is forked onto it; the caller joins it before the optimizer)."""
        if not self.hip:
            w = theta[:, self.off:self.off + self.numel].detach().clone().requires_grad_(True)
            xx = x.detach().clone().requires_grad_(need_dx)
            with torch.enable_grad():
                y = self._torch_fwd(xx, w, G)
                outs = torch.autograd.grad(y, [w, xx] if need_dx else [w], dy.to(y.dtype))
            grads[:, self.off:self.off + self.numel].copy_(outs[0])
            if not need_dx:
                return None
            if self.k == 1 and self.stride == 2:  # same contract as the HIP path: the even voxels only
                return outs[1][:, ::2, ::2, ::2].contiguous()
            return outs[1]
        m, st = ops.ext(), _stream()
        N, D, H, W, _ = x.shape
        B = N // G
        Do, Ho, Wo = dy.shape[1:4]
        dy = dy.contiguous()
        padd = self.pad if self.kt == 27 else 0
        ns = m.conv_wgrad_nsplit_g(G, B, D, H, W, self.cin, self.cout, self.kt, self.stride, self.pad, padd)
        key = (B, D, H, W)
        ptab = self._ptabs.get(key)
        if ptab is None:  # a function of the shape only: built once per (B, D, H, W)
            ptab = torch.empty(B * Do * Ho * Wo, 2, device=x.device, dtype=torch.int32)
            m.conv_pos_table_g(ptab.data_ptr(), B, D, H, W, self.kt, self.stride, self.pad, padd, st)
            if not torch.cuda.is_current_stream_capturing():
                torch.cuda.current_stream().synchronize()  # shared with launches on other streams from now on
                self._ptabs[key] = ptab
        cur = torch.cuda.current_stream()
        if ws is not None:
            ws.wait_stream(cur)
            _BRANCH_KEEP.extend((x, dy, ptab))  # referenced until the branch joins (no record_stream)
        with torch.cuda.stream(ws if ws is not None else cur):
            union = self.kt == 27 and self.stride == 1 and union_wgrad(x, dy, grads, self.off, G, B, D, H, W,
                                                                       self.cin, self.cout, self.pad)
            if not union:
                part = torch.empty(ns * G * self.cout * self.kt * self.cin, device=x.device, dtype=torch.float32)
                m.conv_wgrad_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grads.data_ptr(), grads.stride(0),
                               self.off, G, B, D, H, W, self.cin, self.cout, self.kt, self.stride, self.pad, padd, ns,
                               1.0, ptab.data_ptr(), _stream())
        if not need_dx:
            return None
        pk, self.wt = self.wt, None
        wt = pk[0] if (pk is not None and pk[2] == theta.data_ptr() and pk[1] == G) else self._wp(theta, G, True)[1]
        if self.stride == 1:
            dx = torch.empty(N, D, H, W, self.cin, device=x.device, dtype=torch.bfloat16)
            p2 = self.k - 1 - self.pad
            if self.kt == 1 and g1_gemm(dy, wt, dx, G, self.cout, self.cin):
                return dx
            if self.kt == 1 and _BLAS_1X1 and gemm_1x1(dy, wt, dx, G):
                return dx
            if self.kt == 27 and slab_conv(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, Do, Ho, Wo, self.cout,
                                           self.cin, p2, x.device):
                return dx
            conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, Do, Ho, Wo, self.cout, self.cin, self.kt,
                         1, p2, p2 if self.kt == 27 else 0, x.device)
            return dx
        if self.k == 3:
            # stride 2, pad 1: 8 sub-pixel phase convs over the dy grid (1..8 taps each, 27 in all) written straight
            # into the interleaved voxels of dX — 8x fewer MACs than a conv over the zero-upsampled dy, no memset,
            # no crop copy (conv_dgrad_s2_g; odd extents: the last odd-phase plane has no dy plane beyond it)
            dx = torch.empty(N, D, H, W, self.cin, device=x.device, dtype=torch.bfloat16)
            ops.ext().conv_dgrad_s2_g(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, Do, Ho, Wo, self.cout,
                                      self.cin, 27, D, H, W, st)
            return dx
        # 1x1 stride 2: the half-resolution W^T dY of the even voxels (res_grad_s2 adds it into the residual stream)
        sub = torch.empty(N, Do, Ho, Wo, self.cin, device=x.device, dtype=torch.bfloat16)
        if g1_gemm(dy, wt, sub, G, self.cout, self.cin):
            return sub
        if _BLAS_1X1 and gemm_1x1(dy, wt, sub, G):
            return sub
        conv_fwd(dy.data_ptr(), wt.data_ptr(), sub.data_ptr(), G, B, Do, Ho, Wo, self.cout, self.cin, 1, 1, 0, 0,
                 x.device)
        return sub


class GBN3:
    """Client-grouped BatchNorm3d on ``[G*B, D, H, W, C]`` (``bnr.hip``); affine rows in theta, running stats in
    the buffer rows."""

    def __init__(self, off_w, off_b, C, off_rm, off_rv, off_nbt, hip=True):
        self.off_w, self.off_b, self.C = off_w, off_b, C
        self.off_rm, self.off_rv, self.off_nbt = off_rm, off_rv, off_nbt
        self.hip = hip

    def _torch_fwd(self, t, theta, bufs, G, train, res, relu):
        C = self.C
        tf = t.float().reshape(G, -1, C)
        M = tf.shape[1]
        if train:
            mean = tf.mean(1)
            var = (tf - mean[:, None]).square().mean(1)
            rm = bufs[:, self.off_rm:self.off_rm + C]
            rv = bufs[:, self.off_rv:self.off_rv + C]
            rm.copy_((1 - BN_MOM) * rm + BN_MOM * mean)
            rv.copy_((1 - BN_MOM) * rv + BN_MOM * var * (M / max(1, M - 1)))
            if self.off_nbt >= 0:
                bufs[:, self.off_nbt] += 1
        else:
            mean = bufs[:, self.off_rm:self.off_rm + C].clone()
            var = bufs[:, self.off_rv:self.off_rv + C].clone()
        rstd = torch.rsqrt(var + BN_EPS)
        y = (tf - mean[:, None]) * (rstd * theta[:, self.off_w:self.off_w + C])[:, None] + \
            theta[:, self.off_b:self.off_b + C][:, None]
        y = y.reshape(t.shape)
        if res is not None:
            y = y + res.float()
        if relu:
            y = torch.relu(y)
        return y.to(t.dtype), torch.stack([mean, rstd], -1)

    def fwd(self, t, theta, bufs, G, train, res=None, relu=False, part=None, bstats=None):
        """``part``: (chunk partials [n][G][C][2], n) of ``t`` computed by the producing GEMM's epilogue (training
        mode): only the finalize runs, no statistics pass over ``t``."""
        if not self.hip:
            return self._torch_fwd(t, theta, bufs, G, train, res, relu)
        m, st = ops.ext(), _stream()
        N = t.shape[0]
        M = t.numel() // (self.C * G)
        stats = torch.empty(G, self.C, 2, device=t.device, dtype=torch.float32)
        if train and bstats is not None and bufs is not None and self.off_nbt >= 0:
            # [SLAB-STATS] per-block (mean, M2) of the conv epilogue, merged with the running-stat update
            bst, npb, bp, Mg = bstats
            assert Mg == M
            co = torch.empty(4, G * self.C, device=t.device, dtype=torch.float32)  # scale, shift, mean, invstd
            m.bn_finalize(bst.data_ptr(), npb, bp, Mg, G, self.C, theta.data_ptr(), theta.stride(0), self.off_w,
                          self.off_b, bufs.data_ptr(), bufs.stride(0), self.off_rm, self.off_rv, self.off_nbt, BN_MOM,
                          BN_EPS, co[0].data_ptr(), co[1].data_ptr(), co[2].data_ptr(), co[3].data_ptr(), 1, st)
            stats.copy_(co[2:4].t().reshape(G, self.C, 2))
        elif train and part is not None:
            m.bnr_finalize_part(part[0].data_ptr(), part[1], G, M, self.C, BN_EPS, BN_MOM, stats.data_ptr(),
                                bufs.data_ptr() if bufs is not None else 0, bufs.stride(0) if bufs is not None else 0,
                                self.off_rm, self.off_rv, self.off_nbt, st)
        elif train:
            ws = torch.empty(m.bnr_workspace(G, M, self.C), device=t.device, dtype=torch.float32)
            m.bnr_stats(t.data_ptr(), G, M, self.C, BN_EPS, BN_MOM, ws.data_ptr(), stats.data_ptr(),
                        bufs.data_ptr() if bufs is not None else 0, bufs.stride(0) if bufs is not None else 0,
                        self.off_rm, self.off_rv, self.off_nbt, st)
        else:
            m.bnr_eval_stats(G, self.C, BN_EPS, bufs.data_ptr(), bufs.stride(0), self.off_rm, self.off_rv,
                             stats.data_ptr(), st)
        y = torch.empty_like(t)
        r = res.contiguous() if res is not None else None
        m.bnr_apply(t.data_ptr(), r.data_ptr() if r is not None else 0, stats.data_ptr(), theta.data_ptr(),
                    theta.stride(0), self.off_w, self.off_b, y.data_ptr(), G, M, self.C, int(relu), st)
        assert N % G == 0
        return y, stats

    def bwd(self, dy, mask, t, stats, theta, grads, G, eval_mode=False, tmask=False, part=None):
        """``tmask`` (HIP): the forward was ``fwd(relu=True)`` without residual and ``mask`` is its output; the kernels
        recompute that ReLU mask from ``t`` bit-exactly instead of reading the mask tensor ([TMASK], ``bnr.hip``)."""
        if not self.hip:
            C = self.C
            d = dy.float().reshape(G, -1, C)
            if mask is not None:
                d = d * (mask.reshape(G, -1, C) > 0)
            mean, rstd = stats[..., 0], stats[..., 1]
            xh = (t.float().reshape(G, -1, C) - mean[:, None]) * rstd[:, None]
            A, Bs = d.sum(1), (d * xh).sum(1)
            grads[:, self.off_w:self.off_w + C].copy_(Bs)
            grads[:, self.off_b:self.off_b + C].copy_(A)
            M = d.shape[1]
            g = theta[:, self.off_w:self.off_w + C]
            if eval_mode:
                dt = (rstd * g)[:, None] * d
            else:
                dt = (rstd * g)[:, None] * (d - (A / M)[:, None] - xh * (Bs / M)[:, None])
            return dt.reshape(t.shape).to(t.dtype)
        m, st = ops.ext(), _stream()
        M = t.numel() // (self.C * G)
        dy = dy.contiguous()
        coef = torch.empty(G, self.C, 2, device=t.device, dtype=torch.float32)
        dt = torch.empty_like(t)
        if part is not None:  # [RESBN] statistics from the residual-gradient pass that produced dy
            assert mask is None and not eval_mode and dy.dtype == torch.bfloat16
            m.bnr_bwd_part(t.data_ptr(), dy.data_ptr(), stats.data_ptr(), theta.data_ptr(), theta.stride(0),
                           self.off_w, self.off_b, grads.data_ptr(), grads.stride(0), part.data_ptr(), coef.data_ptr(),
                           dt.data_ptr(), G, M, self.C, st)
            return dt
        ws = torch.empty(m.bnr_workspace(G, M, self.C), device=t.device, dtype=torch.float32)
        tm = bool(tmask) and mask is not None and dy.dtype == torch.bfloat16
        m.bnr_bwd_tm(t.data_ptr(), dy.data_ptr(), int(dy.dtype == torch.bfloat16),
                     mask.data_ptr() if (mask is not None and not tm) else 0, stats.data_ptr(), theta.data_ptr(),
                     theta.stride(0), self.off_w, self.off_b, grads.data_ptr(), grads.stride(0), ws.data_ptr(),
                     coef.data_ptr(), dt.data_ptr(), G, M, self.C, int(eval_mode), int(tm), st)
        return dt


class GroupedResNet3D:
    """Forward/backward graph of ``models.resnet3d.ResNet3D`` (Bottleneck) for G clients at once."""

    def __init__(self, players: ParamLayout, blayers: ParamLayout, device, hip=None):
        self.device = torch.device(device)
        self.hip = (self.device.type == "cuda") if hip is None else hip
        self.act = torch.bfloat16 if self.hip else torch.float32
        off = {n: o for n, o in zip(players.names, players.offsets)}
        shp = dict(zip(players.names, players.shapes))
        boff = {n: o for n, o in zip(blayers.names, blayers.offsets)}
        self.off, self.shp, self.boff = off, shp, boff

        def conv(name, stride):
            co, ci, k = shp[name][0], shp[name][1], shp[name][2]
            return GConv3(off[name], co, ci, k, stride, (k - 1) // 2, self.hip)

        def bn(prefix):
            return GBN3(off[prefix + ".weight"], off[prefix + ".bias"], shp[prefix + ".weight"][0],
                        boff[prefix + ".running_mean"], boff[prefix + ".running_var"],
                        boff.get(prefix + ".num_batches_tracked", -1), self.hip)

        self.blocks = []
        li = 1
        while ("layer%d.0.conv1.weight" % li) in off:
            bi = 0
            while ("layer%d.%d.conv1.weight" % (li, bi)) in off:
                p = "layer%d.%d." % (li, bi)
                stride = 2 if (li > 1 and bi == 0) else 1
                blk = {"c1": conv(p + "conv1.weight", 1), "n1": bn(p + "bn1"),
                       "c2": conv(p + "conv2.weight", stride), "n2": bn(p + "bn2"),
                       "c3": conv(p + "conv3.weight", 1), "n3": bn(p + "bn3")}
                if p + "downsample.0.weight" in off:
                    blk["cd"] = conv(p + "downsample.0.weight", stride)
                    blk["nd"] = bn(p + "downsample.1")
                self.blocks.append(blk)
                bi += 1
            li += 1
        self.fc_w, self.fc_b = off["fc.weight"], off["fc.bias"]
        self.ncls, self.feat = shp["fc.weight"]
        self.stem_c = shp["conv1.weight"][0]
        if self.hip:
            from .resnet2d_hip import WeightPacker
            self.packer = WeightPacker([b[k] for b in self.blocks for k in ("c1", "c2", "c3", "cd") if k in b],
                                       self.device)
            self.packer.keep_other_fresh = _PACK_FUSE_G
        else:
            self.packer = None

    # ------------------------------------------------------------------ stem
    def _stem(self, x8, theta, bufs, G, train, idx=None):
        """uint8 volumes -> pooled stem activation [N, 31, 37, 31, C] (+ what the backward needs).  HIP: ``x8`` is
        the volume store and ``idx`` the samples of this step (None: all of ``x8``, in order)."""
        if self.hip:
            return self._stem_hip(x8, idx, theta, bufs, G, train)
        return self._stem_torch(x8, theta, bufs, G, train)

    def _stem_hip(self, x8, idx, theta, bufs, G, train):
        m, st = ops.ext(), _stream()
        dev = theta.device
        assert x8.dim() == 4 and x8.dtype == torch.uint8 and x8.device == dev and x8.is_contiguous(), \
            "stem.hip reads contiguous uint8 [N, D, H, W] volumes on the compute device"
        D, H, W = x8.shape[1:]
        assert self.stem_c == 64 and W <= 128, "stem.hip: 64 channels, output rows of at most 64 voxels"
        Od, Oh, Ow = (D - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
        Qd, Qh, Qw = (Od - 1) // 2 + 1, (Oh - 1) // 2 + 1, (Ow - 1) // 2 + 1
        if idx is None:
            idx = torch.arange(x8.shape[0], device=dev, dtype=torch.int32)
        idx = idx.to(device=dev, dtype=torch.int32).contiguous()
        N = idx.numel()
        assert N % G == 0
        B = N // G
        C, o, bo = self.stem_c, self.off, self.boff
        sz = m.stem_sizes(N, D, H, W)
        xp = torch.empty(sz[0], device=dev, dtype=torch.uint8)
        xq = torch.empty(sz[0], device=dev, dtype=torch.uint8) if train else None
        m.stem_polyphase(x8.data_ptr(), idx.data_ptr(), N, D, H, W, xp.data_ptr(), xq.data_ptr() if train else 0, st)
        y = torch.empty(N, Od, Oh, Ow, C, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(sz[3], device=dev, dtype=torch.float32)
        wk = torch.empty(G * sz[5], device=dev, dtype=torch.bfloat16)
        m.stem_fwd(xp.data_ptr(), theta.data_ptr(), theta.stride(0), o["conv1.weight"], N, B, D, H, W, wk.data_ptr(),
                   y.data_ptr(), stats.data_ptr(), st)
        del xp
        coef = torch.empty(4, G * C, device=dev, dtype=torch.float32)  # scale, shift, mean, invstd
        ptrs = [coef[i].data_ptr() for i in range(4)]
        nbt = bo.get("bn1.num_batches_tracked", -1)
        if train:
            upd = bufs is not None and nbt >= 0
            m.bn_finalize(stats.data_ptr(), B * Od, Oh * Ow, B * Od * Oh * Ow, G, C, theta.data_ptr(),
                          theta.stride(0), o["bn1.weight"], o["bn1.bias"], bufs.data_ptr() if upd else 0,
                          bufs.stride(0) if upd else 0, bo["bn1.running_mean"], bo["bn1.running_var"], nbt, BN_MOM,
                          BN_EPS, *ptrs, int(upd), st)
        else:
            m.bn_eval(G, C, theta.data_ptr(), theta.stride(0), o["bn1.weight"], o["bn1.bias"], bufs.data_ptr(),
                      bufs.stride(0), bo["bn1.running_mean"], bo["bn1.running_var"], BN_EPS, *ptrs, st)
        out = torch.empty(N, Qd, Qh, Qw, C, device=dev, dtype=torch.bfloat16)
        amax = torch.empty(N, Qd, Qh, Qw, C, device=dev, dtype=torch.uint8)
        m.stem_pool(y.data_ptr(), ptrs[0], ptrs[1], N, B, D, H, W, out.data_ptr(), amax.data_ptr(), st)
        return out, ((y, xq, amax, coef, N, B, (D, H, W)) if train else None)

    def _stem_hip_bwd(self, saved, da, theta, grads, G):
        y, xq, amax, coef, N, B, (D, H, W) = saved
        m, st = ops.ext(), _stream()
        dev = theta.device
        sz = m.stem_sizes(N, D, H, W)
        o = self.off
        da = da.to(torch.bfloat16).contiguous()  # the bf16 residual gradient stream (a no-op in train_step)
        dz = torch.empty_like(y)
        part = torch.empty(sz[3], device=dev, dtype=torch.float32)
        bcoef = torch.empty(G * self.stem_c * 3, device=dev, dtype=torch.float32)
        slab = torch.empty(sz[4], device=dev, dtype=torch.float32)
        m.stem_bwd(da.data_ptr(), amax.data_ptr(), y.data_ptr(), xq.data_ptr(), coef[0].data_ptr(),
                   coef[1].data_ptr(), coef[2].data_ptr(), coef[3].data_ptr(), N, B, D, H, W, theta.data_ptr(),
                   theta.stride(0), o["bn1.weight"], grads.data_ptr(), grads.stride(0), o["conv1.weight"],
                   o["bn1.weight"], o["bn1.bias"], dz.data_ptr(), part.data_ptr(), bcoef.data_ptr(), slab.data_ptr(),
                   st)

    def _stem_torch(self, x8, theta, bufs, G, train):
        N = x8.shape[0]
        B = N // G
        C = self.stem_c
        o = self.off
        w = theta[:, o["conv1.weight"]:o["conv1.weight"] + C * 343].reshape(G * C, 1, 7, 7, 7)
        gam = theta[:, o["bn1.weight"]:o["bn1.weight"] + C].reshape(G * C)
        bet = theta[:, o["bn1.bias"]:o["bn1.bias"] + C].reshape(G * C)
        leaf = [w.detach().clone().requires_grad_(train), gam.detach().clone().requires_grad_(train),
                bet.detach().clone().requires_grad_(train)]
        rm = bufs[:, self.boff["bn1.running_mean"]:self.boff["bn1.running_mean"] + C].reshape(G * C).clone()
        rv = bufs[:, self.boff["bn1.running_var"]:self.boff["bn1.running_var"] + C].reshape(G * C).clone()
        xin = (x8.to(self.act) / 255.0).view(G, B, *x8.shape[1:]).transpose(0, 1)  # [B, G, D, H, W]
        with torch.set_grad_enabled(train):
            s = F.conv3d(xin, leaf[0].to(self.act), stride=2, padding=3, groups=G)          # [B, G*C, ...]
            s = F.batch_norm(s.float(), rm, rv, leaf[1], leaf[2], training=train, momentum=BN_MOM, eps=BN_EPS)
            s = F.max_pool3d(torch.relu(s), 3, 2, 1)
            d, h, ww = s.shape[2:]
            out = s.view(B, G, C, d, h, ww).permute(1, 0, 3, 4, 5, 2).reshape(N, d, h, ww, C)
        if train:
            bufs[:, self.boff["bn1.running_mean"]:self.boff["bn1.running_mean"] + C].copy_(rm.view(G, C))
            bufs[:, self.boff["bn1.running_var"]:self.boff["bn1.running_var"] + C].copy_(rv.view(G, C))
            if "bn1.num_batches_tracked" in self.boff:
                bufs[:, self.boff["bn1.num_batches_tracked"]] += 1
        # downstream layers get a detached activation (the stem's own backward is autograd.grad(out, leaf, da))
        return out.detach().to(self.act).contiguous(), (out, leaf)

    # ------------------------------------------------------------------ forward
    def forward(self, x8, theta, bufs, G, train, idx=None):
        packed = self.packer is not None
        N = x8.shape[0] if idx is None else idx.numel()
        if packed:  # every bottleneck layer's MFMA images for this step, two launches
            # [PACK-FUSE-G] training images per row group (keyed by the rows' address): the runner's step-major plan
            # interleaves the row groups, and the optimizer of a group writes that group's next-step images
            key = (G, N // G, train, theta.data_ptr()) if (train and _PACK_FUSE_G) else (G, N // G, train)
            self.packer.pack(theta, G, train, key=key)
        a, stem = self._stem(x8, theta, bufs, G, train, idx)
        saved = []
        for blk in self.blocks:
            xin = a
            # the 1x1x1 GEMMs hand their outputs' BatchNorm partials to the next BN (training mode)
            t1 = blk["c1"].fwd(xin, theta, G, train, packed, stats=train)
            h1, s1 = blk["n1"].fwd(t1, theta, bufs, G, train, relu=True, part=blk["c1"].take_part())
            t2 = blk["c2"].fwd(h1, theta, G, train, packed, stats=train)
            h2, s2 = blk["n2"].fwd(t2, theta, bufs, G, train, relu=True, bstats=blk["c2"].take_bstats())
            t3 = blk["c3"].fwd(h2, theta, G, train, packed, stats=train)
            p3 = blk["c3"].take_part()
            if "cd" in blk:
                td = blk["cd"].fwd(xin, theta, G, train, packed, stats=train)
                yd, sd = blk["nd"].fwd(td, theta, bufs, G, train, part=blk["cd"].take_part())
            else:
                td, sd, yd = None, None, xin
            a, s3 = blk["n3"].fwd(t3, theta, bufs, G, train, res=yd, relu=True, part=p3)
            if train:
                saved.append((xin, t1, s1, h1, t2, s2, h2, t3, s3, td, sd, a))
        N = a.shape[0]
        C = a.shape[-1]
        pooled = a.float().view(N, -1, C).mean(1)
        fw = theta[:, self.fc_w:self.fc_w + self.ncls * self.feat].view(G, self.ncls, self.feat)
        fb = theta[:, self.fc_b:self.fc_b + self.ncls]
        B = N // G
        logits = (pooled.view(G, B, 1, C) * fw.view(G, 1, self.ncls, C)).sum(-1) + fb.view(G, 1, self.ncls)
        return logits.reshape(N, self.ncls), pooled, saved, stem

    def train_step(self, theta, bufs, grads, x8, y, G, B, bn_train=True, idx=None):
        logits, pooled, saved, stem = self.forward(x8, theta, bufs, G, True, idx)
        lg = logits.view(G, B)
        yt = y.float().view(G, B)
        losses = F.binary_cross_entropy_with_logits(lg, yt, reduction="none").mean(1)
        dlog = (torch.sigmoid(lg) - yt) / B                                           # [G, B]
        fw = theta[:, self.fc_w:self.fc_w + self.feat].view(G, self.feat)
        grads[:, self.fc_w:self.fc_w + self.feat].copy_((dlog.unsqueeze(2) * pooled.view(G, B, self.feat)).sum(1))
        grads[:, self.fc_b:self.fc_b + 1].copy_(dlog.sum(1, keepdim=True))
        a = saved[-1][-1]
        N = a.shape[0]
        S = a[0].numel() // a.shape[-1]
        dpool = (dlog.unsqueeze(2) * fw.unsqueeze(1)).reshape(N, 1, self.feat) / float(S)
        # the residual-stream gradient is kept in bf16 on the HIP path (res_grad writes bf16): it is re-read by the
        # BatchNorm backward of every block, where fp32 doubled the bytes
        da = dpool.expand(N, S, self.feat).reshape(a.shape).to(self.act).contiguous()
        # NIDT_WGRAD_STREAM=1: weight gradients on a branch forked from the data-gradient chain (joined after the stem
        # backward); off by default, as in the 2-D engine (profiles/r3_ab_wgrad_stream.txt)
        ws = None
        if self.hip and os.environ.get("NIDT_WGRAD_STREAM", "0") == "1" and not torch.cuda.is_current_stream_capturing():
            if getattr(self, "_ws", None) is None:
                self._ws = torch.cuda.Stream(device=self.device)
            ws = self._ws
        # [OMASK] HIP: the residual-gradient kernel of a block also applies the ReLU mask of the previous block's
        # output (its input xin), so that block's BN3 / downsample-BN backward and identity shortcut take the stream
        # pre-masked (no mask reads); NIDT_R3D_OMASK=0 keeps the masks in the BN backward (A/B)
        omask_on = self.hip and os.environ.get("NIDT_R3D_OMASK", "1") != "0"
        # [TMASK] bn1 / bn2 backward recompute their ReLU mask from t (no h1 / h2 reads); NIDT_R3D_TMASK=0: A/B
        tm = self.hip and os.environ.get("NIDT_R3D_TMASK", "1") != "0"
        # [RESBN] with [OMASK], the residual-gradient pass also reduces the backward statistics of the previous block's
        # bn3 (and downsample BN): their backward skips its own pass over (t, dy); NIDT_R3D_RESBN=0: A/B
        resbn = omask_on and os.environ.get("NIDT_R3D_RESBN", "1") != "0"
        pre3 = pred = None
        da_masked = False
        for bi, (blk, sv) in enumerate(zip(reversed(self.blocks), reversed(saved))):
            xin, t1, s1, h1, t2, s2, h2, t3, s3, td, sd, a = sv
            amask = None if da_masked else a
            dt3 = blk["n3"].bwd(da, amask, t3, s3, theta, grads, G, part=pre3)
            dh2 = blk["c3"].bwd(dt3, h2, theta, grads, G, ws=ws)
            dt2 = blk["n2"].bwd(dh2, h2, t2, s2, theta, grads, G, tmask=tm)
            dh1 = blk["c2"].bwd(dt2, h1, theta, grads, G, ws=ws)
            dt1 = blk["n1"].bwd(dh1, h1, t1, s1, theta, grads, G, tmask=tm)
            dx1 = blk["c1"].bwd(dt1, xin, theta, grads, G, ws=ws)
            dx2 = None
            if "cd" in blk:
                dtd = blk["nd"].bwd(da, amask, td, sd, theta, grads, G, part=pred)
                dx2 = blk["cd"].bwd(dtd, xin, theta, grads, G, ws=ws)
            half = dx2 is not None and blk["cd"].stride == 2  # 1x1x1 stride-2 projection: even-voxel gradient
            if self.hip:
                out = torch.empty(dx1.shape, device=dx1.device, dtype=torch.bfloat16)
                # the input of the network's first block is the stem output (its backward applies its own masks)
                om = xin if (omask_on and bi + 1 < len(self.blocks)) else None
                omp = om.data_ptr() if om is not None else 0
                pre3 = pred = None
                if resbn and om is not None and not half:
                    psv = saved[len(saved) - 2 - bi]  # the previous block (next in this backward walk)
                    t3p, s3p, tdp, sdp = psv[7], psv[8], psv[9], psv[10]
                    Cc = out.shape[-1]
                    Mm = out.numel() // (Cc * G)
                    mm = ops.ext()
                    pre3 = torch.empty(mm.bnr_workspace(G, Mm, Cc), device=out.device, dtype=torch.float32)
                    pred = torch.empty_like(pre3) if tdp is not None else None
                    mm.bnr_res_partial(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr() if dx2 is not None else 0,
                                       0 if dx2 is not None else da.data_ptr(),
                                       0 if (dx2 is not None or amask is None) else amask.data_ptr(), omp,
                                       t3p.data_ptr(), s3p.data_ptr(), pre3.data_ptr(),
                                       tdp.data_ptr() if tdp is not None else 0,
                                       sdp.data_ptr() if tdp is not None else 0,
                                       pred.data_ptr() if pred is not None else 0, G, Mm, Cc, _stream())
                elif half:
                    Nn, Dd, Hh, Ww, Cc = dx1.shape
                    ops.ext().res_grad_s2_om(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr(), omp, Nn, Dd, Hh, Ww, Cc,
                                             1, _stream())
                else:
                    ops.ext().res_grad_om(out.data_ptr(), dx1.data_ptr(), dx2.data_ptr() if dx2 is not None else 0,
                                          0 if dx2 is not None else da.data_ptr(),
                                          0 if (dx2 is not None or amask is None) else amask.data_ptr(), omp,
                                          out.numel(), 1 | (2 if da.dtype == torch.bfloat16 else 0), _stream())
                da = out
                da_masked = om is not None
            elif half:
                da = dx1.float().clone()
                da[:, ::2, ::2, ::2] += dx2.float()
            else:
                da = dx1.float() + (dx2.float() if dx2 is not None else da * (a > 0))
        if self.hip:
            self._stem_hip_bwd(stem, da, theta, grads, G)
            if ws is not None:
                torch.cuda.current_stream().wait_stream(ws)  # join: the optimizer reads every weight gradient
                _BRANCH_KEEP.clear()
            return losses.detach()
        out, leaf = stem
        gw, gg, gb = torch.autograd.grad(out, leaf, da.to(out.dtype))
        C = self.stem_c
        o = self.off
        grads[:, o["conv1.weight"]:o["conv1.weight"] + C * 343].copy_(gw.reshape(G, -1))
        grads[:, o["bn1.weight"]:o["bn1.weight"] + C].copy_(gg.view(G, C))
        grads[:, o["bn1.bias"]:o["bn1.bias"] + C].copy_(gb.view(G, C))
        return losses.detach()


# [PACK-FUSE-G] the optimizer step writes the next step's forward weight images (``optim.hip`` ``local_opt_pack``,
# the 2-D engine's fusion) with one image buffer per training row group (8 x 5.9 GB at config 5: the HBM is sized
# for it); NIDT_R3D_PACK_FUSE=0: every step packs from theta (A/B)
_PACK_FUSE_G = os.environ.get("NIDT_R3D_PACK_FUSE", "1") != "0"


class ResNet3DHipEngine:
    """Engine API (train_step / eval_logits / local_opt / saliency_acc) of the client-batched 3D ResNet on uint8
    ABCD-shape volumes ``[N, D, H, W]`` (labels {0, 1}, BCE head with one logit)."""
    sample_fields = ("x8", "labels")

    supports_graphs = False  # launches here are few and large (seconds per step at config-5 shapes)
    fused_pack = _PACK_FUSE_G   # runner: local_opt(pack_next=True) where the same rows train next at this shape
    images_per_group = True     # ... also when several row groups share the launch shape (separate image buffers)

    @property
    def input_shape(self):
        return (1,) + tuple(self.x8.shape[1:])

    def __init__(self, template_model, volumes_u8, labels, device, hip=None):
        self.device = torch.device(device)
        self.players = ParamLayout.from_tensors(list(template_model.named_parameters()))
        self.blayers = ParamLayout.from_tensors(list(template_model.named_buffers()))
        self.net = GroupedResNet3D(self.players, self.blayers, self.device, hip=hip)
        self.x8 = volumes_u8
        self.labels = labels.to(self.device)
        if self.net.hip:
            ops.ext()  # fail loudly without the extension
        self._opt = None

    def _src(self, idx):
        """(volumes, sample index) for the network: a device-resident store is read in place by the HIP stem's
        polyphase gather; otherwise the step's samples are gathered to the device first."""
        if self.net.hip and self.x8.device == self.device:
            return self.x8, idx
        return self._x(idx), None

    def _x(self, idx):
        return self.x8.index_select(0, idx.long().to(self.x8.device)).to(self.device, non_blocking=True)

    def train_step(self, theta, bufs, grads, idx, G, B, keep, seed, cids=None, seed_dev=None, bn_train=True):
        y = self.labels.index_select(0, idx.long())
        x, sel = self._src(idx)
        return self.net.train_step(theta, bufs, grads, x, y, G, B, bn_train, idx=sel)

    def eval_logits(self, theta, bufs, idx, G, B):
        with torch.no_grad():
            x, sel = self._src(idx)
            logits, _, _, _ = self.net.forward(x, theta, bufs, G, False, idx=sel)
        return logits.float()

    def _opt_cls(self):
        from .executor import HipEngine, TorchEngine
        return HipEngine if theta_on_gpu(self) else TorchEngine  # fused HIP optimizer, or its torch twin on CPU

    def _delegate(self):
        if self._opt is None:
            cls = self._opt_cls()
            self._opt = cls.__new__(cls)
            if theta_on_gpu(self):
                self._opt.m = ops.ext()
        return self._opt

    def local_opt(self, theta, grads, mom_buf, spec, lr, wd, momentum, max_norm, lr_dev=None, keep_grad=False,
                  pack_next=False):
        pk = self.net.packer
        if (pack_next and _PACK_FUSE_G and pk is not None and pk.last is not None
                and pk.last[1:] == (theta.data_ptr(), theta.stride(0)) and pk.last[0][0] == theta.shape[0]):
            from .executor import HipEngine
            key = pk.last[0]
            HipEngine.local_opt_pack(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm,
                                     pk.fused_plan(key, theta.shape[1]), lr_dev=lr_dev, keep_grad=keep_grad)
            pk.fresh[key] = (theta.data_ptr(), theta._version)
            return
        if pk is not None and pk.last is not None:  # these rows change without their images
            pk.fresh.pop(pk.last[0], None)
        self._opt_cls().local_opt(self._delegate(), theta, grads, mom_buf, spec, lr, wd, momentum, max_norm,
                                  lr_dev=lr_dev, keep_grad=keep_grad)

    def saliency_acc(self, theta, grads, score, alpha):
        self._opt_cls().saliency_acc(self._delegate(), theta, grads, score, alpha)


def theta_on_gpu(engine):
    return torch.device(engine.device).type == "cuda"
