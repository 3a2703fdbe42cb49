"""Client-batched AlexNet3D_Dropout train/eval step on the gfx950 HIP kernels.

One call trains G virtual clients in lockstep: every client has its own fp32 master row in ``theta [G, P]``
(reference param order, so state_dict keys / masks / SNIP scores line up with
``fedml_api/model/cv/salient_models.py:142-191``), its own BN running stats row in ``bufs [G, Q]``, and its own
batch of B volumes.  The forward/backward is an explicit launch sequence (no autograd, no MIOpen):

  conv1+BN1+ReLU+pool1 (fused, BN1 stats from patch moments)  ->  conv2 (MFMA, BN-stat epilogue)
  -> BN2+ReLU+pool2 -> conv3 -> conv4 (BN3+ReLU fused into its loader) -> conv5 (BN4 fused) -> BN5+ReLU+pool5
  -> head (dropout MLP + BCEWithLogits, fwd+bwd) -> BN5/conv5 bwd -> ... -> conv1 sparse wgrad + closed form.

Gradients are written (not accumulated) straight into ``grads [G, P]`` at the reference parameter offsets;
the fused clip+SGD+mask optimizer then updates ``theta`` in place.
"""
from __future__ import annotations

import os

import torch

from .. import ops

BN_EPS = 1e-5
BN_MOM = 0.1
# (conv idx, bn idx, Cin, Cout, pad, in spatial)
L2 = (4, 5, 64, 128, 0, (19, 23, 19))
L3 = (8, 9, 128, 192, 1, (5, 7, 5))
L4 = (11, 12, 192, 192, 1, (5, 7, 5))
L5 = (14, 15, 192, 128, 1, (5, 7, 5))
NM = 125 + 125 * 125
# [EAGER-BRANCH] weight gradients on a forked branch of the step (see train_step).  Captured steps run without it
# (64 clients: no faster, profiles/r3_ab_wgrad_stream.txt; 8 clients captured with the branch -1.0 %).  Launches of
# <= NIDT_AX_EAGER_MAXG clients (default 32: the per-GPU loads of the 2-, 4- and 8-GPU strong-scaling bench) run
# EAGER steps with the branch instead: 8 / 16 / 32 clients +1.7 / +2.9 / +2.0 % over captured steps without it,
# 64 clients -4.2 % (stays captured) (profiles/r6_eager_branch.txt).  HipEngine.graphs_default_for picks the mode
# per trained row set; NIDT_AX_WGRAD_STREAM=0 / 1 forces the branch off / on for every launch.
# [WG2-EARLY] with the branch, the conv2 wgrad is forked before the conv2 dgrad (beside it) for launches of <= 8
# clients, after it (beside the conv1 wgrad) above: 8 clients +0.9 %, 16 / 32 clients -2.1 / -1.6 %
# (profiles/r6_eager_branch.txt); NIDT_WG2_EARLY=0 / 1 forces it.
_WS_ENV = os.environ.get("NIDT_AX_WGRAD_STREAM")
_WG2_EARLY_ENV = os.environ.get("NIDT_WG2_EARLY")
_EAGER_MAXG = int(os.environ.get("NIDT_AX_EAGER_MAXG", "32"))


def eager_branch(G):
    """Launches of G clients train in eager steps with the weight-gradient branch ([EAGER-BRANCH])."""
    return G <= _EAGER_MAXG


def _wg2_early(G):
    return _WG2_EARLY_ENV == "1" if _WG2_EARLY_ENV is not None else G <= 8


def _wgrad_branch(G):
    if _WS_ENV is not None:
        return _WS_ENV == "1"
    return eager_branch(G) and not torch.cuda.is_current_stream_capturing()
# conv2-5 weight packs batched into two pack.hip launches per step instead of eight: 8 clients per GPU +0.3%,
# 64 within noise (profiles/r4_ab_alexnet_bpack.txt); NIDT_AX_BPACK=0: the per-layer packs (A/B)
_BPACK = os.environ.get("NIDT_AX_BPACK", "1") != "0"


def _p(t):
    return t.data_ptr() if t is not None else 0


class HipAlexNet3D:
    """Owns scratch buffers for a (G, B) shape and runs fused train / eval steps."""

    def __init__(self, players, blayers, device):
        self.m = ops.ext()
        self.pl, self.bl = players, blayers
        self.dev = torch.device(device)
        self.P, self.Q = players.total, blayers.total
        self._cache = {}
        self.o = {n: off for n, off in zip(players.names, players.offsets)}
        self.ob = {n: off for n, off in zip(blayers.names, blayers.offsets)}

    # ---------------------------------------------------------------------------------------------
    def _bufs(self, G, B, train):
        key = (G, B, train)
        if key in self._cache:
            return self._cache[key]
        d, bf, f32, u8 = self.dev, torch.bfloat16, torch.float32, torch.uint8
        NB = G * B
        e = lambda *s, dt=bf: torch.empty(s, dtype=dt, device=d)  # noqa: E731
        b = dict(
            w1p=e(G, 64, 224), w125=e(G, 64, 125, dt=f32),
            s1=e(G, 64, dt=f32), t1=e(G, 64, dt=f32), m1=e(G, 64, dt=f32), i1=e(G, 64, dt=f32),
            Mb=e(G, NM, dt=torch.float64), mu=e(G, 125, dt=f32), covw=e(G, 64, 125, dt=f32),
            p1=e(NB, 19, 23, 19, 64), a1=e(NB, 19, 23, 19, 64, dt=u8),
            y2=e(NB, 17, 21, 17, 128), p2=e(NB, 5, 7, 5, 128), a2=e(NB, 5, 7, 5, 128, dt=u8),
            y3=e(NB, 5, 7, 5, 192), y4=e(NB, 5, 7, 5, 192), y5=e(NB, 5, 7, 5, 128),
            h3=e(NB, 5, 7, 5, 192), h4=e(NB, 5, 7, 5, 192),
            p5=e(NB, 1, 2, 1, 128), a5=e(NB, 1, 2, 1, 128, dt=u8),
            logits=e(NB, dt=f32), loss=e(G, dt=f32),
        )
        for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
            b["w%dp" % ci] = e(G, cout, 27, cin)
            b["bias%d" % ci] = e(G, cout, dt=f32)
            for k in ("s", "t", "m", "i"):
                b["%s%d" % (k, ci)] = e(G, cout, dt=f32)
            mg = B * (sp[0] + 2 * pad - 2) * (sp[1] + 2 * pad - 2) * (sp[2] + 2 * pad - 2)
            bp = self.m.conv3d_fwd_bp(cin, cout, 0, G, mg)
            npb = self.m.conv3d_fwd_nblocks(B, sp[0], sp[1], sp[2], pad, bp)
            if self.m.conv3d_fwd_vol_pick(G, B, *sp, cin, cout, pad):  # k_conv_fwd_vol: statistics per sample
                bp, npb = mg // B, B
            b["st%d" % ci] = e(G, npb, cout, 2, dt=f32)
            b["npb%d" % ci] = npb
            b["bp%d" % ci] = bp
        # split-K for the forward/dgrad convs whose grids would not fill the chip (few clients per GPU)
        fp_sz = 0
        for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
            out = tuple(d + 2 * pad - 2 for d in sp)
            for tag, (c_in, c_out, vol, pd) in (("f", (cin, cout, sp, pad)), ("d", (cout, cin, out, 2 - pad))):
                mg = B * (vol[0] + 2 * pd - 2) * (vol[1] + 2 * pd - 2) * (vol[2] + 2 * pd - 2)
                ks = self.m.conv3d_fwd_ksplit(c_in, c_out, G, mg)
                b["ks%s%d" % (tag, ci)] = ks
                if (tag == "f" or train) and self.m.conv3d_fwd_vol_pick(G, B, *vol, c_in, c_out, pd):
                    # whole-sample union staging (k_conv_fwd_vol): the 5x7x5 conv3-5 forward / data gradient
                    b["fv%s%d" % (tag, ci)] = True
                if ks > 1:
                    fp_sz = max(fp_sz, ks * G * mg * c_out)
        b["fpart"] = e(max(fp_sz, 1), dt=f32)
        # forward / dgrad convs with the three-tap union B staging (k_conv_fwd_tri) and their union tables
        st0 = ops.stream()
        for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
            out = tuple(d + 2 * pad - 2 for d in sp)
            for tag, (c_in, c_out, vol, pd) in (("f", (cin, cout, sp, pad)), ("d", (cout, cin, out, 2 - pad))):
                if tag == "d" and not train:
                    continue
                kname = "ks%s%d" % (tag, ci)
                if b.get("fv" + kname[2:]):
                    continue
                if b[kname] <= 1 and self.m.conv3d_fwd_slab_pick(G, B, *vol, c_in, c_out, pd):
                    # kd-slab union staging (k_conv_fwd_slab): the padded conv2 data gradient
                    tab = e(self.m.conv3d_fwd_slab_table_size(B, *vol, pd), dt=torch.int32)
                    self.m.conv3d_fwd_slab_table(_p(tab), B, *vol, pd, st0)
                    b["fs" + kname] = tab
                elif b[kname] <= 1 and self.m.conv3d_fwd_tri_pick(G, B, *vol, c_in, c_out, pd):
                    tab = e(self.m.conv3d_fwd_tri_table_size(B, *vol, pd), dt=torch.int32)
                    self.m.conv3d_fwd_tri_table(_p(tab), B, *vol, pd, st0)
                    b["ft" + kname] = tab
        if train:
            for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
                b["w%dt" % ci] = e(G, cin, 27, cout)
                b["ns%d" % ci] = self.m.conv3d_wgrad_nsplit(G, B, sp[0], sp[1], sp[2], cin, cout, pad)
            # wgrad with kd-slab (k_conv_wgrad_slab) or three-tap (k_conv_wgrad_tri) union staging, each with its own
            # split factor, where the shape allows
            for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
                b["wslab%d" % ci] = bool(self.m.conv3d_wgrad_slab_pick(G, B, *sp, cin, cout, pad))
                b["tri%d" % ci] = not b["wslab%d" % ci] and bool(self.m.conv3d_wgrad_tri_pick(G, B, *sp, cin, cout, pad))
                if b["wslab%d" % ci]:
                    b["ns%d" % ci] = self.m.conv3d_wgrad_slab_nsplit(G, B, *sp, cin, cout, pad)
                elif b["tri%d" % ci]:
                    b["ns%d" % ci] = self.m.conv3d_wgrad_tri_nsplit(G, B, *sp, cin, cout, pad)
            wg_sz = max(b["ns%d" % ci] * G * cout * 27 * cin for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5))
            b.update(
                wgpart=e(wg_sz, dt=f32),
                dp5=e(NB, 1, 2, 1, 128), dy5=e(NB, 5, 7, 5, 128), dx5=e(NB, 5, 7, 5, 192),
                dy4=e(NB, 5, 7, 5, 192), dx4=e(NB, 5, 7, 5, 192), dy3=e(NB, 5, 7, 5, 192),
                dx3=e(NB, 5, 7, 5, 128), dy2=e(NB, 17, 21, 17, 128), dp1=e(NB, 19, 23, 19, 64),
                bnpart=e(G * 64 * 256 * 2, dt=f32), coef=e(G, 192, 3, dt=f32),
                c1part=e(NB * 19 * self.m.conv1_wgrad_nq(NB), 64, 126, dt=f32),
            )
            # per-layer output-position tables for the LDS-DMA wgrad kernel (shared by all clients and steps)
            st0 = ops.stream()
            for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
                mg = B * (sp[0] + 2 * pad - 2) * (sp[1] + 2 * pad - 2) * (sp[2] + 2 * pad - 2)
                b["pt%d" % ci] = e(mg, 2, dt=torch.int32)
                self.m.conv3d_pos_table(_p(b["pt%d" % ci]), B, sp[0], sp[1], sp[2], pad, st0)
            for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
                if b["wslab%d" % ci]:
                    b["stab%d" % ci] = e(self.m.conv3d_wgrad_slab_table_size(B, *sp, pad), dt=torch.int32)
                    self.m.conv3d_wgrad_slab_table(_p(b["stab%d" % ci]), B, *sp, pad, st0)
                elif b["tri%d" % ci]:
                    b["stab%d" % ci] = e(self.m.conv3d_wgrad_tri_table_size(B, *sp, pad), dt=torch.int32)
                    self.m.conv3d_wgrad_tri_table(_p(b["stab%d" % ci]), B, *sp, pad, st0)
            # the weight-gradient branch of this launch shape (one per shape: side lanes run shapes concurrently)
            if d.type == "cuda":
                b["wstream"] = torch.cuda.Stream(device=d)
        if _BPACK:
            self._batched_pack_plan(G, b, train)
        self._cache[key] = b
        return b

    def _batched_pack_plan(self, G, b, train):
        """conv2-5 weight images of all G clients in one buffer, packed by two launches per step (``pack.hip``
        ``pack_convs``: a plain grid over the four layers, then a transpose grid) instead of two per layer;
        ``b["w%dp"]`` / ``b["w%dt"]`` become views of that buffer."""
        import numpy as np

        from .resnet2d_hip import _PACK_DTYPE
        if self.m.pack_desc_bytes() != _PACK_DTYPE.itemsize:
            raise RuntimeError("pack.hip PackDesc layout changed")
        desc = np.zeros(4, dtype=_PACK_DTYPE)
        off = nplain = ntrans = 0
        views = []
        for i, (ci, bi, cin, cout, pad, sp) in enumerate((L2, L3, L4, L5)):
            dd = desc[i]
            dd["src_off"] = self.o["features.%d.weight" % ci]
            dd["cout"], dd["cin_p"], dd["cin_src"], dd["kt"] = cout, cin, cin, 27
            dd["blk_plain"], dd["blk_t"], dd["blk_plain1"] = nplain, ntrans, 0
            dd["slot"][:] = np.arange(26, -1, -1)  # stride 1: the flipped kernel
            n = G * cout * 27 * cin
            dd["wp_off"], off, nplain = off, off + n, nplain + cout * self.m.pack_plain_chunks(cin, 27)
            vt = None
            if train:
                dd["wt_off"], vt, off = off, off, off + n
                ntrans += ((cin + 63) // 64) * ((cout + 63) // 64) * 27
            else:
                dd["wt_off"] = -1
            views.append((ci, cin, cout, int(dd["wp_off"]), vt))
        buf = torch.empty(off, dtype=torch.bfloat16, device=self.dev)
        for ci, cin, cout, op, ot in views:
            n = G * cout * 27 * cin
            b["w%dp" % ci] = buf[op:op + n].view(G, cout, 27, cin)
            if ot is not None:
                b["w%dt" % ci] = buf[ot:ot + n].view(G, cin, 27, cout)
        lds = max(self.m.pack_plain_lds(L[2], 27) for L in (L2, L3, L4, L5))  # one channel chunk of a 3x3x3 row
        b["bpack"] = (torch.from_numpy(desc.view(np.uint8).copy()).to(self.dev), nplain, ntrans, lds, buf)

    def _conv(self, b, key, x, w, bias, y, stats, G, B, D, H, W, cin, cout, pad, st, theta=None, ci=None):
        """conv3d_fwd, or its split-K form when ``b[key]`` (chosen at allocation) is > 1.  With ``theta`` the bias
        of conv ``ci`` is read straight from the flat parameter rows (row stride P), no per-step copy."""
        ks = b[key]
        if b.get("fv" + key[2:]):  # whole-sample union B operand (k_conv_fwd_vol)
            if theta is not None:
                o = self.o["features.%d.bias" % ci]
                bptr, bld = theta.data_ptr() + 4 * o, theta.stride(0)
            else:
                bptr, bld = _p(bias), 0
            self.m.conv3d_fwd_vol(_p(x), _p(w), bptr, bld, _p(y), _p(stats), G, B, D, H, W, cin, cout, pad, st)
            return
        ft, fs = b.get("ft" + key), b.get("fs" + key)
        if ft is not None or fs is not None:  # union-staged B operand (k_conv_fwd_slab / k_conv_fwd_tri)
            if theta is not None:
                o = self.o["features.%d.bias" % ci]
                bptr, bld = theta.data_ptr() + 4 * o, theta.stride(0)
            else:
                bptr, bld = _p(bias), 0
            fn = self.m.conv3d_fwd_slab if fs is not None else self.m.conv3d_fwd_tri
            fn(_p(x), _p(w), bptr, bld, _p(y), _p(stats), G, B, D, H, W, cin, cout, pad, _p(fs if fs is not None else ft), st)
            return
        if theta is not None and ks <= 1:
            o = self.o["features.%d.bias" % ci]
            self.m.conv3d_fwd_bld(_p(x), _p(w), theta.data_ptr() + 4 * o, theta.stride(0), _p(y), _p(stats), G, B, D,
                                  H, W, cin, cout, pad, st)
            return
        if theta is not None:
            o = self.o["features.%d.bias" % ci]
            bias.copy_(theta[:, o:o + cout])
        if ks > 1:
            self.m.conv3d_fwd_splitk(_p(x), _p(w), _p(bias), _p(y), _p(stats), _p(b["fpart"]), ks, G, B, D, H, W, cin,
                                     cout, pad, st)
        else:
            self.m.conv3d_fwd(_p(x), _p(w), _p(bias), 0, 0, _p(y), _p(stats), G, B, D, H, W, cin, cout, pad, st)

    # ---------------------------------------------------------------------------------------------
    def _pack(self, theta, G, b, train, prepacked=False):
        """Weight images of this step.  ``prepacked``: the previous optimizer step already wrote the conv2-5 forward
        images from these rows (``fused_plan``), so only conv1's pack and the data-gradient transposes run."""
        m, st = self.m, ops.stream()
        P = theta.stride(0)
        m.pack_conv1_w(_p(theta), P, self.o["features.0.weight"], self.o["features.1.weight"], G, 1.0 / 255.0,
                       _p(b["w1p"]), _p(b["w125"]), st)
        if "bpack" in b:
            tab, nplain, ntrans, lds, buf = b["bpack"]
            if nplain and not prepacked or ntrans:
                m.pack_convs(_p(tab), 4, 0 if prepacked else nplain, 0, ntrans, lds, _p(theta), P, G, _p(buf), st)
            return
        assert not prepacked, "prepacked weight images need the batched pack plan (NIDT_AX_BPACK=1)"
        for (ci, bi, cin, cout, pad, sp) in (L2, L3, L4, L5):
            m.pack_conv_w(_p(theta), P, self.o["features.%d.weight" % ci], G, cout, cin, 1.0, _p(b["w%dp" % ci]),
                          _p(b["w%dt" % ci]) if train else 0, st)

    def _bn(self, ci, bi, C, G, B, sp, theta, bufs, b, train):
        """BN coefficients for conv ``ci`` (train: from the conv epilogue stats; eval: running stats, which also
        leaves the running mean / invstd in ``m``/``i`` for an eval-mode backward)."""
        m, st = self.m, ops.stream()
        P, Q = theta.stride(0), bufs.stride(0)
        og, ob = self.o["features.%d.weight" % bi], self.o["features.%d.bias" % bi]
        orm, orv = self.ob["features.%d.running_mean" % bi], self.ob["features.%d.running_var" % bi]
        if train:
            onbt = self.ob["features.%d.num_batches_tracked" % bi]
            Mg = B * sp[0] * sp[1] * sp[2]
            m.bn_finalize(_p(b["st%d" % ci]), b["npb%d" % ci], b["bp%d" % ci], Mg, G, C, _p(theta), P, og, ob, _p(bufs), Q,
                          orm, orv, onbt, BN_MOM, BN_EPS, _p(b["s%d" % ci]), _p(b["t%d" % ci]), _p(b["m%d" % ci]),
                          _p(b["i%d" % ci]), 1, st)
        else:
            m.bn_eval(G, C, _p(theta), P, og, ob, _p(bufs), Q, orm, orv, BN_EPS, _p(b["s%d" % ci]),
                      _p(b["t%d" % ci]), _p(b["m%d" % ci]), _p(b["i%d" % ci]), st)

    def fused_plan(self, G, B, P):
        """Plan of the optimizer step that writes the conv2-5 forward images of the next (G, B) train step itself
        (``optim.hip`` ``local_opt_pack``, as the 2-D engine's ``WeightPacker.fused_plan``): the batched pack's
        descriptor table (plain-grid block prefixes over the four layers), its plain block count, the {start, length}
        table of the other parameter ranges of a P-wide row (4096 per block), LDS bytes, the image buffer."""
        key = ("fused", G, B, int(P))
        plan = self._cache.get(key)
        if plan is not None:
            return plan
        b = self._bufs(G, B, True)
        tab, nplain, ntrans, lds, buf = b["bpack"]
        spans = sorted((self.o["features.%d.weight" % L[0]], self.o["features.%d.weight" % L[0]] + L[3] * 27 * L[2])
                       for L in (L2, L3, L4, L5))
        rest, pos = [], 0
        for a_, b_ in spans + [(int(P), int(P))]:
            while pos < a_:
                n = min(4096, a_ - pos)
                rest.append((pos, n))
                pos += n
            pos = max(pos, b_)
        rt_ = torch.tensor(rest if rest else [(0, 0)], dtype=torch.int64).to(self.dev)
        plan = (tab, 4, nplain, rt_, len(rest), lds, buf)
        self._cache[key] = plan
        return plan

    def forward(self, theta, bufs, x8, mom, idx, G, B, train, bn_train=None, prepacked=False):
        """Runs the forward; returns the scratch dict (logits in ``b['logits']``).  ``train`` keeps what the backward
        needs; ``bn_train`` (default = ``train``) selects batch statistics (+ running-stat update) vs running stats."""
        bn_train = train if bn_train is None else bn_train
        assert theta.stride(1) == 1 and bufs.stride(1) == 1 and theta.shape[0] == G and bufs.shape[0] == G
        assert theta.shape[1] == self.P and bufs.shape[1] == self.Q and theta.dtype == torch.float32
        assert idx.dtype == torch.int32 and idx.numel() == G * B and x8.dtype == torch.uint8
        assert x8.dim() == 5 and tuple(x8.shape[1:]) == (61, 73, 61, 8) and x8.is_contiguous()
        m, st = self.m, ops.stream()
        b = self._bufs(G, B, train)
        NB = G * B
        P, Q = theta.stride(0), bufs.stride(0)
        self._pack(theta, G, b, train, prepacked)
        # ---- conv1 + BN1 + ReLU + pool1 ----
        if bn_train:
            assert mom is not None and mom.dtype == torch.float64 and mom.shape[1] == NM
            m.conv1_bnstats(_p(mom), _p(idx), B, G, _p(b["Mb"]), _p(b["w125"]), _p(theta), P,
                            self.o["features.0.bias"], self.o["features.1.weight"], self.o["features.1.bias"],
                            _p(bufs), Q, self.ob["features.1.running_mean"], self.ob["features.1.running_var"],
                            self.ob["features.1.num_batches_tracked"], BN_MOM, BN_EPS, 1, _p(b["s1"]), _p(b["t1"]),
                            _p(b["m1"]), _p(b["i1"]), _p(b["mu"]), _p(b["covw"]), st)
        else:
            m.bn_eval(G, 64, _p(theta), P, self.o["features.1.weight"], self.o["features.1.bias"], _p(bufs), Q,
                      self.ob["features.1.running_mean"], self.ob["features.1.running_var"], BN_EPS, _p(b["s1"]),
                      _p(b["t1"]), _p(b["m1"]), _p(b["i1"]), st)
            ob = self.o["features.0.bias"]
            b["t1"].add_(b["s1"] * theta[:, ob:ob + 64])  # fold conv1 bias: the kernel convolves without it
        m.conv1_fwd_pool(_p(x8), _p(idx), _p(b["w1p"]), _p(b["s1"]), _p(b["t1"]), NB, B, _p(b["p1"]), _p(b["a1"]), st)
        # ---- conv2 + BN2 + ReLU + pool2 ----
        ci, bi, cin, cout, pad, sp = L2
        self._conv(b, "ksf4", b["p1"], b["w4p"], b["bias4"], b["y2"], b["st4"] if bn_train else None,
                   G, B, 19, 23, 19, 64, 128, 0, st, theta, 4)
        self._bn(4, 5, 128, G, B, (17, 21, 17), theta, bufs, b, bn_train)
        m.bn_relu_pool(_p(b["y2"]), _p(b["s4"]), _p(b["t4"]), _p(b["p2"]), _p(b["a2"]), NB, B, 17, 21, 17, 128, st)
        # ---- conv3 ----
        self._conv(b, "ksf8", b["p2"], b["w8p"], b["bias8"], b["y3"], b["st8"] if bn_train else None,
                   G, B, 5, 7, 5, 128, 192, 1, st, theta, 8)
        self._bn(8, 9, 192, G, B, (5, 7, 5), theta, bufs, b, bn_train)
        # BN3+ReLU materialised once (read by conv4 fwd and by conv4's wgrad im2col 27x)
        m.bn_relu_apply(_p(b["y3"]), _p(b["s8"]), _p(b["t8"]), _p(b["h3"]), NB * 175, 192, B * 175, st)
        # ---- conv4 ----
        self._conv(b, "ksf11", b["h3"], b["w11p"], b["bias11"], b["y4"], b["st11"] if bn_train else None,
                   G, B, 5, 7, 5, 192, 192, 1, st, theta, 11)
        self._bn(11, 12, 192, G, B, (5, 7, 5), theta, bufs, b, bn_train)
        m.bn_relu_apply(_p(b["y4"]), _p(b["s11"]), _p(b["t11"]), _p(b["h4"]), NB * 175, 192, B * 175, st)
        # ---- conv5 + BN5 + ReLU + pool ----
        self._conv(b, "ksf14", b["h4"], b["w14p"], b["bias14"], b["y5"], b["st14"] if bn_train else None,
                   G, B, 5, 7, 5, 192, 128, 1, st, theta, 14)
        self._bn(14, 15, 128, G, B, (5, 7, 5), theta, bufs, b, bn_train)
        m.bn_relu_pool(_p(b["y5"]), _p(b["s14"]), _p(b["t14"]), _p(b["p5"]), _p(b["a5"]), NB, B, 5, 7, 5, 128, st)
        return b

    # ---------------------------------------------------------------------------------------------
    def train_step(self, theta, bufs, grads, x8, mom, idx, labels, G, B, keep=0.5, seed=0, cids=None, seed_dev=None,
                   bn_train=True, prepacked=False):
        """Forward + backward for G clients; writes ``grads`` [G,P], updates BN running stats in ``bufs``.
        Returns the per-client mean loss tensor [G] (device).  ``seed_dev`` (int64 device scalar, optional) is
        added to ``seed`` inside the kernel, so a captured hipGraph can advance the dropout stream on device.
        ``bn_train=False``: gradient of the model in ``eval()`` mode (running-stat BN, no dropout, no running-stat
        update) — DisPFL's ``screen_gradients`` (``DisPFL/my_model_trainer.py:166-189``)."""
        assert grads.shape == theta.shape and grads.stride(1) == 1 and grads.stride(0) == theta.stride(0)
        assert labels.dtype == torch.float32 and labels.numel() == G * B and B <= 32
        m, st = self.m, ops.stream()
        if not bn_train:
            keep = 1.0
        ev = 0 if bn_train else 1
        b = self.forward(theta, bufs, x8, mom, idx, G, B, True, bn_train=bn_train, prepacked=prepacked)
        NB = G * B
        P = theta.stride(0)
        o = self.o
        m.head(_p(b["p5"]), _p(theta), P, o["classifier.1.weight"], o["classifier.1.bias"], o["classifier.4.weight"],
               o["classifier.4.bias"], _p(labels), _p(b["logits"]), _p(b["loss"]), _p(grads), grads.stride(0), _p(b["dp5"]), G, B, 1,
               float(keep), int(seed) & ((1 << 64) - 1), _p(cids), _p(seed_dev), st)
        nchunk = 64

        def bn_bwd(pool, ci, bi, C, sp, dsrc, pout, amax, dy, y):
            m.bn_bwd(pool, _p(y), _p(dsrc), _p(pout), _p(amax), _p(b["s%d" % ci]), _p(b["t%d" % ci]),
                     _p(b["m%d" % ci]), _p(b["i%d" % ci]), NB, B, sp[0], sp[1], sp[2], C, _p(b["bnpart"]), nchunk,
                     _p(theta), P, o["features.%d.weight" % bi], _p(grads), P, o["features.%d.weight" % bi],
                     o["features.%d.bias" % bi], o["features.%d.bias" % ci], _p(b["coef"]), _p(dy), ev, st)

        # Weight gradients are off the critical path (nothing in the step reads them before the optimizer), so
        # with a wgrad stream they run on a branch forked from the data-gradient chain: the one-block-per-CU
        # conv3-5 grids fill each other's idle CUs, and the MFMA-bound conv2 wgrad runs beside the VALU-bound
        # conv1 sparse wgrad.  All wgrads are ordered on that one branch, so they share ``wgpart``.
        cur = torch.cuda.current_stream()
        ws = b.get("wstream") if _wgrad_branch(G) else None
        wst = ws.cuda_stream if ws is not None else st

        def fork():
            if ws is not None:
                ws.wait_stream(cur)

        def wgrad(ci, x, xs, xt, dy, sp, cin, cout, pad):
            if b.get("wslab%d" % ci) and xs is None:
                m.conv3d_wgrad_slab(_p(x), _p(dy), _p(b["wgpart"]), _p(grads), P, o["features.%d.weight" % ci], G, B,
                                    sp[0], sp[1], sp[2], cin, cout, pad, b["ns%d" % ci], 1.0, _p(b["stab%d" % ci]), wst)
                return
            if b.get("tri%d" % ci) and xs is None:
                m.conv3d_wgrad_tri(_p(x), _p(dy), _p(b["wgpart"]), _p(grads), P, o["features.%d.weight" % ci], G, B,
                                   sp[0], sp[1], sp[2], cin, cout, pad, b["ns%d" % ci], 1.0, _p(b["stab%d" % ci]), wst)
                return
            m.conv3d_wgrad(_p(x), _p(xs), _p(xt), _p(dy), _p(b["wgpart"]), _p(grads), P, o["features.%d.weight" % ci],
                           G, B, sp[0], sp[1], sp[2], cin, cout, pad, b["ns%d" % ci], 1.0, _p(b["pt%d" % ci]), wst)

        # layer 5: pool5 -> BN5 -> conv5
        bn_bwd(1, 14, 15, 128, (5, 7, 5), b["dp5"], b["p5"], b["a5"], b["dy5"], b["y5"])
        fork()
        wgrad(14, b["h4"], None, None, b["dy5"], (5, 7, 5), 192, 128, 1)
        self._conv(b, "ksd14", b["dy5"], b["w14t"], None, b["dx5"], None, G, B, 5, 7, 5, 128, 192, 1, st)
        # layer 4
        bn_bwd(0, 11, 12, 192, (5, 7, 5), b["dx5"], None, None, b["dy4"], b["y4"])
        fork()
        wgrad(11, b["h3"], None, None, b["dy4"], (5, 7, 5), 192, 192, 1)
        self._conv(b, "ksd11", b["dy4"], b["w11t"], None, b["dx4"], None, G, B, 5, 7, 5, 192, 192, 1, st)
        # layer 3
        bn_bwd(0, 8, 9, 192, (5, 7, 5), b["dx4"], None, None, b["dy3"], b["y3"])
        fork()
        wgrad(8, b["p2"], None, None, b["dy3"], (5, 7, 5), 128, 192, 1)
        self._conv(b, "ksd8", b["dy3"], b["w8t"], None, b["dx3"], None, G, B, 5, 7, 5, 192, 128, 1, st)
        # layer 2: pool2 -> BN2 -> conv2
        bn_bwd(1, 4, 5, 128, (17, 21, 17), b["dx3"], b["p2"], b["a2"], b["dy2"], b["y2"])
        early = _wg2_early(G)
        if ws is None or early:
            fork()
            wgrad(4, b["p1"], None, None, b["dy2"], (19, 23, 19), 64, 128, 0)
        self._conv(b, "ksd4", b["dy2"], b["w4t"], None, b["dp1"], None, G, B, 17, 21, 17, 128, 64, 2, st)
        if ws is not None and not early:
            fork()
            wgrad(4, b["p1"], None, None, b["dy2"], (19, 23, 19), 64, 128, 0)
        # layer 1: sparse wgrad through pool1/ReLU/BN1 (closed form; eval mode: running mean minus the conv bias)
        emean = None
        if not bn_train:
            ob1 = o["features.0.bias"]
            emean = (b["m1"] - theta[:, ob1:ob1 + 64]).contiguous()
        m.conv1_wgrad(_p(x8), _p(idx), _p(b["dp1"]), _p(b["p1"]), _p(b["a1"]), NB, B, _p(b["c1part"]), _p(b["w125"]),
                      _p(b["mu"]), _p(b["covw"]), _p(b["i1"]), _p(theta), P, o["features.1.weight"], _p(grads), P,
                      o["features.0.weight"], o["features.0.bias"], o["features.1.weight"], o["features.1.bias"],
                      1.0 / 255.0, _p(emean), st)
        if ws is not None:
            cur.wait_stream(ws)  # join: the optimizer reads every weight gradient
        return b["loss"]

    def eval_logits(self, theta, bufs, x8, idx, G, B):
        """Eval-mode (running-stat BN, no dropout) logits [G*B] for client g's samples idx[g*B:(g+1)*B]."""
        m, st = self.m, ops.stream()
        b = self.forward(theta, bufs, x8, None, idx, G, B, False)
        P = theta.stride(0)
        o = self.o
        m.head(_p(b["p5"]), _p(theta), P, o["classifier.1.weight"], o["classifier.1.bias"], o["classifier.4.weight"],
               o["classifier.4.bias"], 0, _p(b["logits"]), 0, 0, P, 0, G, B, 0, 1.0, 0, 0, 0, st)
        return b["logits"]
