"""GPU numerics tests: every HIP kernel against a plain PyTorch fp32 reference of the same op.

All tests run in one process on the GPU box (``pytest -m gpu``).  Shapes are the real AlexNet3D shapes at the
ABCD input (1x121x145x121) with small client/batch counts, and every launch's operands are validated on the
host by the Python wrappers first.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from neuroimagedisttraining_amd.engine.executor import padded_rows

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _m():
    from neuroimagedisttraining_amd import ops
    return ops.ext()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _cl(x):  # NCDHW -> NDHWC
    return x.permute(0, 2, 3, 4, 1).contiguous()


def _cf(x):  # NDHWC -> NCDHW
    return x.permute(0, 4, 1, 2, 3).contiguous()


# ------------------------------------------------------------------------------------------------
def test_polyphase_and_moments():
    from neuroimagedisttraining_amd.ops.reference import polyphase, unpolyphase
    from neuroimagedisttraining_amd.data.synthetic_fl import conv1_moments_reference, to_hip_store
    torch.manual_seed(0)
    vol = torch.randint(0, 256, (2, 121, 145, 121), dtype=torch.uint8, device=DEV)
    x8, mom = to_hip_store(vol)
    torch.cuda.synchronize()
    assert torch.equal(x8, polyphase(vol))
    assert torch.equal(unpolyphase(x8), vol)
    ref = conv1_moments_reference(vol[:1].cpu())
    assert torch.equal(mom[:1].cpu(), ref), "moments must be exact (integer-valued fp64)"


@pytest.mark.parametrize("cin,cout,pad,sp,xf", [(64, 128, 0, (19, 23, 19), False), (128, 192, 1, (5, 7, 5), False),
                                                (192, 192, 1, (5, 7, 5), True), (192, 128, 1, (5, 7, 5), True),
                                                (128, 64, 2, (17, 21, 17), False)])
@pytest.mark.parametrize("G,B", [(2, 3), (8, 16), (16, 16)])  # 64-, 128- (5x7x5 at G=8) and 256-position blocks
def test_conv3d_fwd_stats(cin, cout, pad, sp, xf, G, B):
    m = _m()
    torch.manual_seed(1)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    w = (torch.randn(G, cout, 27, cin, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(G, cout, device=DEV)
    xs = torch.rand(G, cin, device=DEV) + 0.5 if xf else None
    xt = torch.randn(G, cin, device=DEV) * 0.2 if xf else None
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    y = torch.empty(G * B, Do, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16)
    mg = B * (sp[0] + 2 * pad - 2) * (sp[1] + 2 * pad - 2) * (sp[2] + 2 * pad - 2)
    bp = m.conv3d_fwd_bp(cin, cout, 1 if xf else 0, G, mg)
    npb = m.conv3d_fwd_nblocks(B, *sp, pad, bp)
    stats = torch.empty(G, npb, cout, 2, device=DEV)
    m.conv3d_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr(), xs.data_ptr() if xf else 0, xt.data_ptr() if xf else 0,
                 y.data_ptr(), stats.data_ptr(), G, B, *sp, cin, cout, pad, _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        xin = x[g * B:(g + 1) * B].float()
        if xf:
            xin = torch.relu(xin * xs[g] + xt[g]).bfloat16().float()
        wg = w[g].float().view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3)
        ys.append(_cl(F.conv3d(_cf(xin), wg, bias[g], 1, pad)))
    yr = torch.cat(ys, 0)
    assert _relerr(y.float(), yr) < 1e-2
    # statistics: merged block stats == batch mean / biased var per (client, channel)
    Mg = B * Do * Ho * Wo
    cnt = torch.tensor([min(bp, Mg - b * bp) for b in range(npb)], device=DEV, dtype=torch.float64)
    mean_b, m2_b = stats[..., 0].double(), stats[..., 1].double()
    mean = (mean_b * cnt.view(1, -1, 1)).sum(1) / Mg
    var = (m2_b + cnt.view(1, -1, 1) * (mean_b - mean.unsqueeze(1)) ** 2).sum(1) / Mg
    yr_g = yr.view(G, Mg, cout).double()
    assert _relerr(mean, yr_g.mean(1)) < 1e-3
    assert _relerr(var, yr_g.var(1, unbiased=False)) < 1e-3
    if not xf and bp == 256 and m.conv3d_fwd_tri_ok(B, *sp, cin, cout, pad):
        _check_tri(m, x, w, bias, y, yr, stats, G, B, sp, cin, cout, pad)
    if not xf and bp == 256 and m.conv3d_fwd_slab_ok(B, *sp, cin, cout, pad):
        _check_slab(m, x, w, bias, y, stats, G, B, sp, cin, cout, pad)


@pytest.mark.parametrize("cin,cout,pad,sp,G,B", [(192, 128, 0, (7, 9, 7), 2, 3), (192, 128, 0, (7, 9, 7), 8, 16),
                                                 (64, 128, 0, (19, 23, 19), 2, 2)])
def test_conv3d_fwd_stats_large_mean(cin, cout, pad, sp, G, B):
    """Conv outputs whose channel mean is 50-100x their spread (positive inputs and weights, no padding, so every
    output sums the same number of taps): the one-pass statistics epilogue must not lose the variance to fp32
    cancellation (its sums are shifted by a sample of the channel)."""
    m = _m()
    torch.manual_seed(3)
    x = (torch.rand(G * B, *sp, cin, device=DEV) + 0.5).bfloat16()
    w = (torch.rand(G, cout, 27, cin, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(G, cout, device=DEV) * 0.1
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    y = torch.empty(G * B, Do, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16)
    Mg = B * Do * Ho * Wo
    bp = m.conv3d_fwd_bp(cin, cout, 0, G, Mg)
    npb = m.conv3d_fwd_nblocks(B, *sp, pad, bp)
    stats = torch.empty(G, npb, cout, 2, device=DEV)
    m.conv3d_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, 0, y.data_ptr(), stats.data_ptr(), G, B, *sp, cin,
                 cout, pad, _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        wg = w[g].double().view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3)
        ys.append(_cl(F.conv3d(_cf(x[g * B:(g + 1) * B].double()), wg, bias[g].double(), 1, pad)))
    yr_g = torch.cat(ys, 0).view(G, Mg, cout)
    cnt = torch.tensor([min(bp, Mg - b * bp) for b in range(npb)], device=DEV, dtype=torch.float64)
    mean_b, m2_b = stats[..., 0].double(), stats[..., 1].double()
    mean = (mean_b * cnt.view(1, -1, 1)).sum(1) / Mg
    var = (m2_b + cnt.view(1, -1, 1) * (mean_b - mean.unsqueeze(1)) ** 2).sum(1) / Mg
    vr = yr_g.var(1, unbiased=False)
    assert float((yr_g.mean(1).abs() / vr.sqrt()).median()) > 50  # the regime this test is for
    assert _relerr(mean, yr_g.mean(1)) < 1e-5
    assert _relerr(var, vr) < 2e-3


def _check_tri(m, x, w, bias, y, yr, stats, G, B, sp, cin, cout, pad):
    # union-staged B operand (k_conv_fwd_tri) against the per-tap kernel and, without bias, the fp32 oracle
    tab = torch.empty(m.conv3d_fwd_tri_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
    m.conv3d_fwd_tri_table(tab.data_ptr(), B, *sp, pad, _st())
    y3 = torch.empty_like(y)
    st3 = torch.empty_like(stats)
    m.conv3d_fwd_tri(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, y3.data_ptr(), st3.data_ptr(), G, B, *sp, cin,
                     cout, pad, tab.data_ptr(), _st())
    y4 = torch.empty_like(y)  # no bias / statistics (the dgrad form)
    m.conv3d_fwd_tri(x.data_ptr(), w.data_ptr(), 0, 0, y4.data_ptr(), 0, G, B, *sp, cin, cout, pad, tab.data_ptr(),
                     _st())
    torch.cuda.synchronize()
    # same products; the k order differs when Cin > 64 (triplet-major vs tap-major) -> fp32 rounding only
    assert (y3.float() - y.float()).abs().max() <= 1e-2 * y.float().abs().max()
    assert _relerr(st3, stats) < 1e-4
    assert _relerr(y4.float(), (yr.view(G, -1, cout) - bias.view(G, 1, cout)).view_as(yr)) < 1e-2


def _check_slab(m, x, w, bias, y, stats, G, B, sp, cin, cout, pad):
    # kd-slab union staging (k_conv_fwd_slab): same products as the per-tap kernel, slab-major k order
    tab = torch.empty(m.conv3d_fwd_slab_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
    m.conv3d_fwd_slab_table(tab.data_ptr(), B, *sp, pad, _st())
    y5 = torch.empty_like(y)
    st5 = torch.empty_like(stats)
    m.conv3d_fwd_slab(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, y5.data_ptr(), st5.data_ptr(), G, B, *sp,
                      cin, cout, pad, tab.data_ptr(), _st())
    torch.cuda.synchronize()
    assert (y5.float() - y.float()).abs().max() <= 1e-2 * y.float().abs().max()
    assert _relerr(st5, stats) < 1e-4


@pytest.mark.parametrize("cin,cout,pad,sp", [(64, 128, 0, (19, 23, 19)), (128, 64, 2, (17, 21, 17)),
                                             (64, 64, 1, (10, 12, 11)), (128, 128, 1, (8, 14, 20)),
                                             (64, 64, 1, (31, 37, 31))])
@pytest.mark.parametrize("G,B", [(2, 16), (3, 5)])
def test_conv3d_fwd_slab_matches_fp32(cin, cout, pad, sp, G, B):
    """kd-slab union forward / data gradient (k_conv_fwd_slab): bands crossing output rows, depth planes and
    samples, padded geometries whose border planes skip depth taps, with and without bias — against fp32 conv3d."""
    m = _m()
    assert m.conv3d_fwd_slab_ok(B, *sp, cin, cout, pad)
    torch.manual_seed(3)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    w = (torch.randn(G, cout, 27, cin, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(G, cout, device=DEV)
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    tab = torch.empty(m.conv3d_fwd_slab_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
    m.conv3d_fwd_slab_table(tab.data_ptr(), B, *sp, pad, _st())
    y = torch.empty(G * B, Do, Ho, Wo, cout, device=DEV, dtype=torch.bfloat16)
    y0 = torch.empty_like(y)
    m.conv3d_fwd_slab(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, y.data_ptr(), 0, G, B, *sp, cin, cout, pad,
                      tab.data_ptr(), _st())
    m.conv3d_fwd_slab(x.data_ptr(), w.data_ptr(), 0, 0, y0.data_ptr(), 0, G, B, *sp, cin, cout, pad, tab.data_ptr(),
                      _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        wg = w[g].float().view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3)
        ys.append(_cl(F.conv3d(_cf(x[g * B:(g + 1) * B].float()), wg, None, 1, pad)))
    yr = torch.cat(ys, 0)
    assert _relerr(y0.float(), yr) < 1e-2
    assert _relerr(y.float(), (yr.view(G, -1, cout) + bias.view(G, 1, cout)).view_as(yr)) < 1e-2


@pytest.mark.parametrize("cin,cout,pad,sp", [(128, 192, 1, (5, 7, 5)), (192, 192, 1, (5, 7, 5)),
                                             (192, 128, 1, (5, 7, 5)), (64, 64, 0, (6, 8, 6)), (64, 128, 2, (3, 4, 3)),
                                             (128, 64, 1, (4, 4, 4))])
@pytest.mark.parametrize("G,B", [(2, 16), (3, 5)])
def test_conv3d_fwd_vol_matches_fp32(cin, cout, pad, sp, G, B):
    """Whole-sample union forward / data gradient (k_conv_fwd_vol: one padded sample per 64-channel chunk serves all
    27 taps, per-sample statistics blocks): output with and without bias against fp32 conv3d, and the per-sample
    (mean, M2) statistics against the oracle."""
    m = _m()
    assert m.conv3d_fwd_vol_ok(B, *sp, cin, cout, pad)
    torch.manual_seed(7)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    w = (torch.randn(G, cout, 27, cin, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(G, cout, device=DEV)
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    S = Do * Ho * Wo
    y = torch.full((G * B, Do, Ho, Wo, cout), float("nan"), device=DEV, dtype=torch.bfloat16)
    y0 = torch.full_like(y, float("nan"))
    stats = torch.full((G, B, cout, 2), float("nan"), device=DEV)
    m.conv3d_fwd_vol(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, y.data_ptr(), stats.data_ptr(), G, B, *sp, cin,
                     cout, pad, _st())
    m.conv3d_fwd_vol(x.data_ptr(), w.data_ptr(), 0, 0, y0.data_ptr(), 0, G, B, *sp, cin, cout, pad, _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        wg = w[g].float().view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3)
        ys.append(_cl(F.conv3d(_cf(x[g * B:(g + 1) * B].float()), wg, None, 1, pad)))
    yr = torch.cat(ys, 0)
    assert torch.isfinite(y.float()).all() and torch.isfinite(y0.float()).all()
    assert _relerr(y0.float(), yr) < 1e-2
    yb = (yr.view(G, -1, cout) + bias.view(G, 1, cout)).view_as(yr)
    assert _relerr(y.float(), yb) < 1e-2
    ys_ = yb.view(G, B, S, cout).double()
    mean = ys_.mean(2)
    m2 = ((ys_ - mean.unsqueeze(2)) ** 2).sum(2)
    assert _relerr(stats[..., 0].double(), mean) < 1e-3
    assert _relerr(stats[..., 1].double(), m2) < 1e-3


@pytest.mark.parametrize("cin,cout,hw", [(64, 64, (32, 32)), (128, 128, (16, 16)), (64, 128, (16, 32)),
                                         (256, 256, (16, 16)), (64, 64, (64, 64)), (128, 64, (32, 32))])
@pytest.mark.parametrize("G,B", [(1, 3), (3, 2)])
def test_conv2d_fwd_slab_matches_fp32(cin, cout, hw, G, B):
    """2-D 3x3 stride-1 pad-1 conv on the kd-slab kernel (conv2d_fwd_slab: 9-tap weights, one union per channel
    chunk; the 64x64 shape takes the 416-row unions) against fp32 conv2d, per client."""
    m = _m()
    H, W = hw
    assert m.conv2d_fwd_slab_ok(B, H, W, cin, cout)
    torch.manual_seed(5)
    x = torch.randn(G * B, H, W, cin, device=DEV).bfloat16()
    w = (torch.randn(G, cout, 9, cin, device=DEV) * 0.05).bfloat16()
    tab = torch.empty(m.conv3d_fwd_slab_table_size(B, 1, H, W, 1), device=DEV, dtype=torch.int32)
    m.conv3d_fwd_slab_table(tab.data_ptr(), B, 1, H, W, 1, _st())
    y = torch.full((G * B, H, W, cout), float("nan"), device=DEV, dtype=torch.bfloat16)
    m.conv2d_fwd_slab(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, H, W, cin, cout, tab.data_ptr(), _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        wg = w[g].float().view(cout, 3, 3, cin).permute(0, 3, 1, 2)
        ys.append(F.conv2d(x[g * B:(g + 1) * B].float().permute(0, 3, 1, 2), wg, None, 1, 1).permute(0, 2, 3, 1))
    yr = torch.cat(ys, 0)
    assert torch.isfinite(y.float()).all()
    assert _relerr(y.float(), yr) < 1e-2


@pytest.mark.parametrize("cin,cout,G", [(128, 192, 16), (192, 192, 16), (192, 128, 24), (128, 192, 1), (192, 128, 2)])
@pytest.mark.parametrize("ksplit,stats_on", [(2, True), (3, True), (2, False), (4, True)])
def test_conv3d_fwd_splitk(cin, cout, G, ksplit, stats_on):
    """Split-K forward (few clients per GPU): fp32 partials + finish kernel == fp32 oracle; BN block stats too
    (256-position blocks, and the 64-position blocks of one- or two-client launches, which pick ks > 1 themselves)."""
    m = _m()
    B, pad, sp = 16, 1, (5, 7, 5)
    torch.manual_seed(3)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    w = (torch.randn(G, cout, 27, cin, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(G, cout, device=DEV)
    Mg = B * 5 * 7 * 5
    bp = m.conv3d_fwd_bp(cin, cout, 0, G, Mg)
    assert bp == (256 if G >= 16 else 64)
    if G <= 2:
        assert m.conv3d_fwd_ksplit(cin, cout, G, Mg) > 1
    npb = m.conv3d_fwd_nblocks(B, *sp, pad, bp)
    y = torch.empty(G * B, *sp, cout, device=DEV, dtype=torch.bfloat16)
    stats = torch.empty(G, npb, cout, 2, device=DEV)
    part = torch.empty(ksplit * G * Mg * cout, device=DEV)
    m.conv3d_fwd_splitk(x.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(), stats.data_ptr() if stats_on else 0,
                        part.data_ptr(), ksplit, G, B, *sp, cin, cout, pad, _st())
    y1 = torch.empty_like(y)
    m.conv3d_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr(), 0, 0, y1.data_ptr(), 0, G, B, *sp, cin, cout, pad, _st())
    torch.cuda.synchronize()
    ys = []
    for g in range(G):
        wg = w[g].float().view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3)
        ys.append(_cl(F.conv3d(_cf(x[g * B:(g + 1) * B].float()), wg, bias[g], 1, pad)))
    yr = torch.cat(ys, 0)
    assert _relerr(y.float(), yr) < 1e-2
    assert (y.float() - y1.float()).abs().max() <= 2e-2 * yr.abs().max()  # same as the unsplit kernel up to rounding
    if stats_on:
        cnt = torch.tensor([min(bp, Mg - b * bp) for b in range(npb)], device=DEV, dtype=torch.float64)
        mean_b, m2_b = stats[..., 0].double(), stats[..., 1].double()
        mean = (mean_b * cnt.view(1, -1, 1)).sum(1) / Mg
        var = (m2_b + cnt.view(1, -1, 1) * (mean_b - mean.unsqueeze(1)) ** 2).sum(1) / Mg
        yr_g = yr.view(G, Mg, cout).double()
        assert _relerr(mean, yr_g.mean(1)) < 1e-3
        assert _relerr(var, yr_g.var(1, unbiased=False)) < 1e-3


@pytest.mark.parametrize("cin,cout,pad,sp,xf", [(64, 128, 0, (19, 23, 19), False), (128, 192, 1, (5, 7, 5), False),
                                                (192, 192, 1, (5, 7, 5), True), (192, 128, 1, (5, 7, 5), True)])
def test_conv3d_wgrad_and_dgrad(cin, cout, pad, sp, xf):
    m = _m()
    G, B = 2, 2
    torch.manual_seed(2)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    xs = torch.rand(G, cin, device=DEV) + 0.5 if xf else None
    xt = torch.randn(G, cin, device=DEV) * 0.2 if xf else None
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    dy = torch.randn(G * B, Do, Ho, Wo, cout, device=DEV).bfloat16()
    P = cout * cin * 27 + 7
    grad = torch.zeros(G, P, device=DEV)
    ns = m.conv3d_wgrad_nsplit(G, B, *sp, cin, cout, pad)
    part = torch.empty(ns * G * cout * 27 * cin, device=DEV)
    Mg = B * Do * Ho * Wo
    ptab = torch.empty(Mg, 2, device=DEV, dtype=torch.int32)
    m.conv3d_pos_table(ptab.data_ptr(), B, *sp, pad, _st())
    m.conv3d_wgrad(x.data_ptr(), xs.data_ptr() if xf else 0, xt.data_ptr() if xf else 0, dy.data_ptr(), part.data_ptr(),
                   grad.data_ptr(), P, 3, G, B, *sp, cin, cout, pad, ns, 1.0, ptab.data_ptr(), _st())
    if not xf:  # the register-staged fallback kernel must agree with the LDS-DMA one
        grad0 = torch.zeros_like(grad)
        m.conv3d_wgrad(x.data_ptr(), 0, 0, dy.data_ptr(), part.data_ptr(), grad0.data_ptr(), P, 3, G, B, *sp, cin,
                       cout, pad, ns, 1.0, 0, _st())
        torch.cuda.synchronize()
        assert _relerr(grad0, grad) < 1e-5
    if not xf and m.conv3d_wgrad_tri_ok(B, *sp, cin, cout, pad):  # three-tap union staging: same sums, other order
        stab = torch.empty(m.conv3d_wgrad_tri_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
        m.conv3d_wgrad_tri_table(stab.data_ptr(), B, *sp, pad, _st())
        for ns_t in sorted({1, ns, 3}):
            part_t = torch.empty(ns_t * G * cout * 27 * cin, device=DEV)
            grad_t = torch.zeros_like(grad)
            m.conv3d_wgrad_tri(x.data_ptr(), dy.data_ptr(), part_t.data_ptr(), grad_t.data_ptr(), P, 3, G, B, *sp, cin,
                               cout, pad, ns_t, 1.0, stab.data_ptr(), _st())
            torch.cuda.synchronize()
            assert _relerr(grad_t, grad) < 1e-4, ns_t
    # dgrad through the fwd kernel with flipped/transposed weights (packed from fp32 PyTorch layout)
    wt32 = torch.randn(G, cout, cin, 3, 3, 3, device=DEV) * 0.05
    theta = wt32.view(G, -1).contiguous()
    wp = torch.empty(G, cout, 27, cin, device=DEV, dtype=torch.bfloat16)
    wtt = torch.empty(G, cin, 27, cout, device=DEV, dtype=torch.bfloat16)
    m.pack_conv_w(theta.data_ptr(), theta.stride(0), 0, G, cout, cin, 1.0, wp.data_ptr(), wtt.data_ptr(), _st())
    dx = torch.empty(G * B, *sp, cin, device=DEV, dtype=torch.bfloat16)
    m.conv3d_fwd(dy.data_ptr(), wtt.data_ptr(), 0, 0, 0, dx.data_ptr(), 0, G, B, Do, Ho, Wo, cout, cin, 2 - pad, _st())
    torch.cuda.synchronize()
    for g in range(G):
        xin = x[g * B:(g + 1) * B].float()
        if xf:
            xin = torch.relu(xin * xs[g] + xt[g]).bfloat16().float()
        xin = _cf(xin).requires_grad_(True)
        wref = wt32[g].bfloat16().float().requires_grad_(True)
        out = F.conv3d(xin, wref, None, 1, pad)
        out.backward(_cf(dy[g * B:(g + 1) * B].float()))
        dw = grad[g, 3:3 + cout * cin * 27].view(cout, cin, 3, 3, 3)
        assert _relerr(dw, wref.grad) < 1e-2
        if not xf:
            assert _relerr(dx[g * B:(g + 1) * B].float(), _cl(xin.grad)) < 1e-2
        # wp layout check
        assert torch.equal(wp[g].view(cout, 3, 3, 3, cin).permute(0, 4, 1, 2, 3), wt32[g].bfloat16())


@pytest.mark.parametrize("cin,cout,pad,sp", [(64, 128, 0, (19, 23, 19)), (128, 192, 1, (5, 7, 5)),
                                             (192, 128, 1, (5, 7, 5)), (128, 64, 2, (5, 7, 5))])
def test_conv3d_wgrad_tri_matches_fp32(cin, cout, pad, sp):
    """Three-tap union wgrad (k_conv_wgrad_tri) at B = 16 (steps crossing depth slices and samples, padded
    geometries, 64- and 128-channel blocks) against the fp32 autograd weight gradient."""
    m = _m()
    G, B = 2, 16
    assert m.conv3d_wgrad_tri_ok(B, *sp, cin, cout, pad)
    torch.manual_seed(4)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    dy = torch.randn(G * B, Do, Ho, Wo, cout, device=DEV).bfloat16()
    P = cout * cin * 27 + 5
    stab = torch.empty(m.conv3d_wgrad_tri_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
    m.conv3d_wgrad_tri_table(stab.data_ptr(), B, *sp, pad, _st())
    ns = m.conv3d_wgrad_tri_nsplit(G, B, *sp, cin, cout, pad)
    part = torch.empty(ns * G * cout * 27 * cin, device=DEV)
    grad = torch.zeros(G, P, device=DEV)
    m.conv3d_wgrad_tri(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grad.data_ptr(), P, 5, G, B, *sp, cin, cout, pad,
                       ns, 1.0, stab.data_ptr(), _st())
    torch.cuda.synchronize()
    for g in range(G):
        xin = _cf(x[g * B:(g + 1) * B].float())
        wref = torch.zeros(cout, cin, 3, 3, 3, device=DEV, requires_grad=True)
        F.conv3d(xin, wref, None, 1, pad).backward(_cf(dy[g * B:(g + 1) * B].float()))
        assert _relerr(grad[g, 5:5 + cout * cin * 27].view(cout, cin, 3, 3, 3), wref.grad) < 1e-4


@pytest.mark.parametrize("cin,cout,pad,sp", [(64, 128, 0, (19, 23, 19)), (128, 192, 1, (5, 7, 5)),
                                             (192, 128, 1, (5, 7, 5)), (64, 64, 1, (10, 12, 11))])
@pytest.mark.parametrize("ns", [1, 3, 0])
def test_conv3d_wgrad_slab_matches_fp32(cin, cout, pad, sp, ns):
    """kd-slab union wgrad (k_conv_wgrad_slab: 12 waves, all nine (kh, kw) taps from one union per step) at B = 16
    (steps crossing rows, depth slices and samples; padded geometries; split factors 1, 3 and the cost model's)
    against the fp32 autograd weight gradient."""
    m = _m()
    G, B = 2, 16
    assert m.conv3d_wgrad_slab_ok(B, *sp, cin, cout, pad)
    torch.manual_seed(5)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16()
    Do, Ho, Wo = [s + 2 * pad - 2 for s in sp]
    dy = torch.randn(G * B, Do, Ho, Wo, cout, device=DEV).bfloat16()
    P = cout * cin * 27 + 5
    stab = torch.empty(m.conv3d_wgrad_slab_table_size(B, *sp, pad), device=DEV, dtype=torch.int32)
    m.conv3d_wgrad_slab_table(stab.data_ptr(), B, *sp, pad, _st())
    ns = ns or m.conv3d_wgrad_slab_nsplit(G, B, *sp, cin, cout, pad)
    part = torch.empty(ns * G * cout * 27 * cin, device=DEV)
    grad = torch.zeros(G, P, device=DEV)
    m.conv3d_wgrad_slab(x.data_ptr(), dy.data_ptr(), part.data_ptr(), grad.data_ptr(), P, 5, G, B, *sp, cin, cout,
                        pad, ns, 1.0, stab.data_ptr(), _st())
    torch.cuda.synchronize()
    for g in range(G):
        xin = _cf(x[g * B:(g + 1) * B].float())
        wref = torch.zeros(cout, cin, 3, 3, 3, device=DEV, requires_grad=True)
        F.conv3d(xin, wref, None, 1, pad).backward(_cf(dy[g * B:(g + 1) * B].float()))
        assert _relerr(grad[g, 5:5 + cout * cin * 27].view(cout, cin, 3, 3, 3), wref.grad) < 1e-4


def _signed_gamma(G, C):
    """gamma in (0.5, 1.5) with ~1/4 negative and a few ~0 entries (training can drive gamma through zero)."""
    g = torch.rand(G, C, device=DEV) + 0.5
    g[:, ::4] *= -1
    g[:, 5::16] = 1e-4
    return g


def test_bn_relu_pool_and_bwd():
    m = _m()
    G, B, C = 2, 2, 128
    D, H, W = 17, 21, 17
    torch.manual_seed(3)
    y = torch.randn(G * B, D, H, W, C, device=DEV).bfloat16()
    scale = _signed_gamma(G, C)
    shift = torch.randn(G, C, device=DEV) * 0.3
    out = torch.empty(G * B, D // 3, H // 3, W // 3, C, device=DEV, dtype=torch.bfloat16)
    am = torch.empty_like(out, dtype=torch.uint8)
    m.bn_relu_pool(y.data_ptr(), scale.data_ptr(), shift.data_ptr(), out.data_ptr(), am.data_ptr(), G * B, B, D, H, W, C,
                   _st())
    torch.cuda.synchronize()
    z = y.float().view(G, B, D, H, W, C) * scale.view(G, 1, 1, 1, 1, C) + shift.view(G, 1, 1, 1, 1, C)
    zr = _cf(z.view(G * B, D, H, W, C))
    pr, ir = F.max_pool3d(torch.relu(zr), 3, 3, return_indices=True)
    assert _relerr(out.float(), _cl(pr)) < 1e-2
    # backward through pool -> relu -> BN(train) vs autograd
    gamma = _signed_gamma(G, C)
    beta = torch.randn(G, C, device=DEV) * 0.3
    P = 4 * C
    theta = torch.zeros(G, P, device=DEV)
    theta[:, :C] = gamma
    theta[:, C:2 * C] = beta
    yf = y.float().view(G, B * D * H * W, C).double()
    mean = yf.mean(1).float()
    invstd = (1.0 / torch.sqrt(yf.var(1, unbiased=False) + 1e-5)).float()
    sc = (gamma * invstd).contiguous()
    sh = (beta - mean * sc).contiguous()
    m.bn_relu_pool(y.data_ptr(), sc.data_ptr(), sh.data_ptr(), out.data_ptr(), am.data_ptr(), G * B, B, D, H, W, C, _st())
    dp = torch.randn_like(out, dtype=torch.float32).bfloat16()
    grad = torch.zeros(G, P, device=DEV)
    part = torch.empty(G * 64 * C * 2, device=DEV)
    coef = torch.empty(G, C, 3, device=DEV)
    dy = torch.empty_like(y)
    m.bn_bwd(1, y.data_ptr(), dp.data_ptr(), out.data_ptr(), am.data_ptr(), sc.data_ptr(), sh.data_ptr(),
             mean.data_ptr(), invstd.data_ptr(), G * B, B, D, H, W, C, part.data_ptr(), 64, theta.data_ptr(), P, 0,
             grad.data_ptr(), P, 0, C, 2 * C, coef.data_ptr(), dy.data_ptr(), 0, _st())
    torch.cuda.synchronize()
    for g in range(G):
        # fp64 CPU autograd oracle (first-max pooling semantics, no library BN/pool kernels involved)
        yi = _cf(y[g * B:(g + 1) * B].double().cpu()).requires_grad_(True)
        gm = gamma[g].double().cpu().requires_grad_(True)
        bt = beta[g].double().cpu().requires_grad_(True)
        o = F.max_pool3d(torch.relu(F.batch_norm(yi, None, None, gm, bt, True, 0.1, 1e-5)), 3, 3)
        o.backward(_cf(dp[g * B:(g + 1) * B].double().cpu()))
        assert _relerr(grad[g, :C].cpu(), gm.grad) < 1e-3
        assert _relerr(grad[g, C:2 * C].cpu(), bt.grad) < 1e-3
        assert _relerr(dy[g * B:(g + 1) * B].float().cpu(), _cl(yi.grad)) < 1e-2
        assert float(grad[g, 2 * C:3 * C].abs().max()) == 0.0  # conv bias grad before BN is exactly 0


def _alexnet_setup(G, B, seed=0, signed_gamma=False):
    from neuroimagedisttraining_amd.data.volumes import make_synthetic_abcd
    from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    torch.manual_seed(seed)
    store = make_synthetic_abcd(G * B, seed=seed + 1, device=DEV)
    x8, mom = to_hip_store(store.volumes)
    model = AlexNet3D_Dropout(num_classes=1)
    pl = ParamLayout.from_tensors(list(model.named_parameters()))
    bl = ParamLayout.from_tensors(list(model.named_buffers()))
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    theta = padded_rows(G, pl.total, DEV)
    theta.copy_(torch.stack([pl.flatten_state(dict(AlexNet3D_Dropout(num_classes=1).named_parameters()), DEV)
                             for _ in range(G)]))
    bufs = padded_rows(G, bl.total, DEV)
    bufs.copy_(bl.flatten_state(dict(model.named_buffers()), DEV).unsqueeze(0).expand(G, bl.total))
    # non-trivial BN affine params so the BN backward paths are exercised
    for i, n in enumerate(pl.names):
        if n.startswith("features.") and int(n.split(".")[1]) in (1, 5, 9, 12, 15):
            o, k = pl.offsets[i], pl.numel(i)
            if n.endswith("weight"):
                theta[:, o:o + k] = 0.75 + 0.5 * torch.rand(G, k, device=DEV)
                if signed_gamma:  # negative and near-zero gammas (sign folding of the fused conv1 forward)
                    theta[:, o:o + k:4] *= -1
                    theta[:, o + 5:o + k:16] = 1e-3
            else:
                theta[:, o:o + k] = 0.1 * torch.randn(G, k, device=DEV)
    return store, x8, mom, pl, bl, theta, bufs


def _pool_at(h, amax):
    """max_pool3d(3,3) whose window choices are the HIP kernel's argmax (both sides route gradients alike)."""
    Bn, C, D, H, W = h.shape
    Dp, Hp, Wp = D // 3, H // 3, W // 3
    a = amax.long().permute(0, 4, 1, 2, 3)
    pd = torch.arange(Dp, device=h.device).view(1, 1, Dp, 1, 1)
    ph = torch.arange(Hp, device=h.device).view(1, 1, 1, Hp, 1)
    pw = torch.arange(Wp, device=h.device).view(1, 1, 1, 1, Wp)
    flat = ((3 * pd + a // 9) * H + 3 * ph + (a // 3) % 3) * W + 3 * pw + a % 3
    return torch.gather(h.reshape(Bn, C, -1), 2, flat.reshape(Bn, C, -1)).view(Bn, C, Dp, Hp, Wp)


def _routed_reference(b, theta, pl, vols, labels, G, B, keep, seed):
    """fp64 autograd of AlexNet3D_Dropout in which every discrete decision (max-pool argmax, ReLU masks,
    dropout masks) is taken from the HIP forward.  bf16 activations make near-ties flip those decisions
    relative to an unconstrained fp64 run (a flip moves a whole gradient entry), so the engine is checked
    against the same computation graph; the decisions themselves are checked by the forward comparisons."""
    from neuroimagedisttraining_amd.ops.reference import dropout_keep
    m1 = torch.from_numpy(dropout_keep(seed, G, B, 256, keep, 0)).to(DEV)
    m2 = torch.from_numpy(dropout_keep(seed, G, B, 64, keep, 1)).to(DEV)
    grads, logits = [], []
    cfg = {0: (2, 0), 4: (1, 0), 8: (1, 1), 11: (1, 1), 14: (1, 1)}
    for g in range(G):
        sl = slice(g * B, (g + 1) * B)
        row = theta[g].detach().double().clone().requires_grad_(True)
        pv = {n: row[o:o + pl.numel(i)].view(pl.shapes[i]) for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
        h = (vols[sl].double() / 255.0).unsqueeze(1)
        for ci, bi in zip((0, 4, 8, 11, 14), (1, 5, 9, 12, 15)):
            s_, pd = cfg[ci]
            y = F.conv3d(h, pv["features.%d.weight" % ci], pv["features.%d.bias" % ci], s_, pd)
            z = F.batch_norm(y, None, None, pv["features.%d.weight" % bi], pv["features.%d.bias" % bi], True, 0.1, 1e-5)
            if ci in (0, 4, 14):
                ours = {0: b["p1"], 4: b["p2"], 14: b["p5"]}[ci][sl]
                h = _pool_at(z, {0: b["a1"], 4: b["a2"], 14: b["a5"]}[ci][sl]) * (_cf(ours.double()) > 0)
            else:
                yb = b["y%d" % {8: 3, 11: 4}[ci]][sl].float()
                h = z * _cf(((yb * b["s%d" % ci][g] + b["t%d" % ci][g]) > 0).double())
        f = h.flatten(1) * m1[g].double() / keep
        fo = _cf(b["p5"][sl].double()).flatten(1) * m1[g].double() / keep
        z1o = F.linear(fo, pv["classifier.1.weight"].detach(), pv["classifier.1.bias"].detach())
        zz = F.linear(f, pv["classifier.1.weight"], pv["classifier.1.bias"]) * (z1o > 0) * m2[g].double() / keep
        out = F.linear(zz, pv["classifier.4.weight"], pv["classifier.4.bias"])
        F.binary_cross_entropy_with_logits(out, labels[sl].double().view(B, 1)).backward()
        grads.append(row.grad)
        logits.append(out.detach().view(-1))
    return torch.stack(grads), torch.cat(logits)


@pytest.mark.parametrize("keep,G,B,signed", [(1.0, 2, 4, False), (0.5, 2, 4, False), (0.5, 2, 4, True),
                                              (0.5, 8, 16, True)])
def test_alexnet_train_step_matches_autograd(keep, G, B, signed):
    from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D
    from neuroimagedisttraining_amd.ops.reference import train_step_reference
    store, x8, mom, pl, bl, theta, bufs = _alexnet_setup(G, B, signed_gamma=signed)
    net = HipAlexNet3D(pl, bl, DEV)
    grads = padded_rows(G, pl.total, DEV)
    bufs_h = padded_rows(G, bl.total, DEV)
    bufs_h.copy_(bufs)
    idx = torch.arange(G * B, dtype=torch.int32, device=DEV)
    loss = net.train_step(theta, bufs_h, grads, x8, mom, idx, store.labels.float(), G, B, keep=keep, seed=77)
    torch.cuda.synchronize()
    b = net._cache[(G, B, True)]
    # (1) unconstrained fp64 reference: forward, loss and BN running statistics
    bufs_r = bufs.clone()
    gfree, lr_, logit_r = train_step_reference(pl, bl, theta, bufs_r, store.volumes, store.labels.float(), B,
                                               keep=keep, seed=77, dtype=torch.float64)
    assert _relerr(b["logits"], logit_r) < 3e-2
    assert _relerr(loss, lr_) < 3e-2
    assert _relerr(bufs_h, bufs_r) < 1e-2
    # (2) gradients against the decision-routed fp64 graph
    gr, _ = _routed_reference(b, theta, pl, store.volumes, store.labels, G, B, keep, 77)
    errs = {}
    for i, n in enumerate(pl.names):
        o, k = pl.offsets[i], pl.numel(i)
        if n.startswith("features.") and n.endswith(".bias") and int(n.split(".")[1]) in (0, 4, 8, 11, 14):
            assert float(grads[:, o:o + k].abs().max()) == 0.0  # conv bias before train-mode BN: exactly 0
            continue
        errs[n] = _relerr(grads[:, o:o + k], gr[:, o:o + k])
    print("grad rel errors", errs)
    bad = {n: e for n, e in errs.items() if e > 3e-2}
    assert not bad, bad
    # (3) the free-running fp64 gradient still points the same way (cosine over the whole model)
    cos = F.cosine_similarity(grads.double().flatten(), gfree.double().flatten(), dim=0)
    assert float(cos) > 0.9, float(cos)


@pytest.mark.parametrize("signed", [False, True])
def test_conv1_fused_fwd_and_sparse_wgrad(signed):
    """conv1 -> BN(train, stats from patch moments) -> ReLU -> pool, and the closed-form backward, vs fp64 autograd
    (``signed``: negative and near-zero gammas — the fused forward folds sign(gamma) into its weights)."""
    from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D
    m = _m()
    G, B = 2, 2
    store, x8, mom, pl, bl, theta, bufs = _alexnet_setup(G, B, seed=9, signed_gamma=signed)
    net = HipAlexNet3D(pl, bl, DEV)
    idx = torch.arange(G * B, dtype=torch.int32, device=DEV)
    b = net._bufs(G, B, True)
    net._pack(theta, G, b, True)
    o = net.o
    st = _st()
    P, Q = theta.stride(0), bufs.stride(0)
    m.conv1_bnstats(mom.data_ptr(), idx.data_ptr(), B, G, b["Mb"].data_ptr(), b["w125"].data_ptr(), theta.data_ptr(), P,
                    o["features.0.bias"], o["features.1.weight"], o["features.1.bias"], bufs.data_ptr(), Q,
                    net.ob["features.1.running_mean"], net.ob["features.1.running_var"],
                    net.ob["features.1.num_batches_tracked"], 0.1, 1e-5, 0, b["s1"].data_ptr(), b["t1"].data_ptr(),
                    b["m1"].data_ptr(), b["i1"].data_ptr(), b["mu"].data_ptr(), b["covw"].data_ptr(), st)
    m.conv1_fwd_pool(x8.data_ptr(), idx.data_ptr(), b["w1p"].data_ptr(), b["s1"].data_ptr(), b["t1"].data_ptr(), G * B, B,
                     b["p1"].data_ptr(), b["a1"].data_ptr(), st)
    torch.manual_seed(11)
    dp = torch.randn(G * B, 19, 23, 19, 64, device=DEV).bfloat16()
    grads = padded_rows(G, pl.total, DEV)
    m.conv1_wgrad(x8.data_ptr(), idx.data_ptr(), dp.data_ptr(), b["p1"].data_ptr(), b["a1"].data_ptr(), G * B, B,
                  b["c1part"].data_ptr(), b["w125"].data_ptr(), b["mu"].data_ptr(), b["covw"].data_ptr(),
                  b["i1"].data_ptr(), theta.data_ptr(), P, o["features.1.weight"], grads.data_ptr(), P,
                  o["features.0.weight"], o["features.0.bias"], o["features.1.weight"], o["features.1.bias"],
                  1.0 / 255.0, 0, st)
    torch.cuda.synchronize()
    ow, og, ob = o["features.0.weight"], o["features.1.weight"], o["features.1.bias"]
    for g in range(G):
        # the kernel convolves with bf16(w/255): use exactly those weights in the oracle
        w_eff = (b["w125"][g].double() * 255.0).view(64, 1, 5, 5, 5).detach().clone().requires_grad_(True)
        gm = theta[g, og:og + 64].double().detach().clone().requires_grad_(True)
        bt = theta[g, ob:ob + 64].double().detach().clone().requires_grad_(True)
        x = (store.volumes[g * B:(g + 1) * B].double() / 255.0).unsqueeze(1)
        y = F.conv3d(x, w_eff, None, 2, 0)
        z = F.batch_norm(y, None, None, gm, bt, True, 0.1, 1e-5)
        assert _relerr(b["p1"][g * B:(g + 1) * B].float(), _cl(F.max_pool3d(torch.relu(z), 3, 3).detach())) < 1e-2
        ours = b["p1"][g * B:(g + 1) * B]
        pr = _pool_at(z, b["a1"][g * B:(g + 1) * B]) * (_cf(ours.double()) > 0)
        pr.backward(_cf(dp[g * B:(g + 1) * B].double()))
        e_w = _relerr(grads[g, ow:ow + 8000], w_eff.grad.view(-1))
        e_g = _relerr(grads[g, og:og + 64], gm.grad)
        e_b = _relerr(grads[g, ob:ob + 64], bt.grad)
        print("conv1 grad errors", e_w, e_g, e_b)
        assert e_w < 2e-2 and e_g < 2e-2 and e_b < 2e-2, (e_w, e_g, e_b)


@pytest.mark.parametrize("NB,B", [(4, 2), (128, 16)])
def test_conv1_fwd_wave_tile_matches_pipe(NB, B):
    """The wave-tile fused forward (k_conv1_fwd_w64: a wave owns all 64 channels of 15 columns, DPP pooling, packed
    epilogue) against the channel-split pipe kernel: each mode packs the same fp32 weights with pack_conv1_w into the
    slot order it reads (both the RO = 0 layout by default; NIDT_C1_TAPORD=2 gives w64 the all-b128 layout, another
    MFMA k order), so the pooled bf16 outputs agree within 1 bf16 ulp of the output scale and the argmax bytes except
    at near-ties (random volumes, signed scales, per-client weights)."""
    m = _m()
    g = torch.Generator(device=DEV).manual_seed(5)
    G = NB // B
    x8 = torch.randint(0, 256, (NB, 61, 73, 61, 8), dtype=torch.uint8, device=DEV, generator=g)
    idx = torch.randperm(NB, device=DEV, generator=g).int()
    theta = torch.randn(G, 8000, device=DEV, generator=g) * 0.05
    scale = torch.randn(G, 64, device=DEV, generator=g) * 0.02
    shift = torch.randn(G, 64, device=DEV, generator=g)
    outs = []
    for mode in (0, 1):
        m.conv1_fwd_mode(mode)
        w8 = torch.zeros(G, 64, 128, dtype=torch.int16, device=DEV)
        w125 = torch.zeros(G, 64, 125, device=DEV)
        m.pack_conv1_w(theta.data_ptr(), 8000, 0, -1, G, 1.0 / 255.0, w8.data_ptr(), w125.data_ptr(), _st())
        p1 = torch.full((NB, 19, 23, 19, 64), float("nan"), device=DEV).bfloat16()
        a1 = torch.full((NB, 19, 23, 19, 64), 255, dtype=torch.uint8, device=DEV)
        m.conv1_fwd_pool(x8.data_ptr(), idx.data_ptr(), w8.data_ptr(), scale.data_ptr(), shift.data_ptr(), NB, B,
                         p1.data_ptr(), a1.data_ptr(), _st())
        torch.cuda.synchronize()
        outs.append((p1, a1, w125))
    m.conv1_fwd_mode(-1)
    (p0, a0, w0), (p1, a1, w1) = outs
    assert torch.equal(w0, w1)  # the effective weights do not depend on the slot order
    assert torch.isfinite(p1.float()).all() and int(a1.max()) < 27
    d = (p0.float() - p1.float()).abs()
    assert float(d.max()) <= float(p0.float().abs().max()) * 2 ** -7, float(d.max())
    assert float((a0 != a1).float().mean()) < 1e-3


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("NB,B", [(4, 2), (256, 16)])  # few samples (row / slab splits) and many
def test_conv1_wgrad_smfmac_matches_valu_gather(NB, B, mode):
    """The 2:4-sparse matrix-core conv1 weight gradients — k_conv1_wgrad_smf (mode 1, x-ordered K) and k_conv1_wgrad_mx
    (mode 2, the default: argmax row in the sparsity index, blocks over pd-slab ranges) — give the same per-client S / D
    sums and gradients as the VALU gather (k_conv1_wgrad_split) on random inputs: every argmax offset, ReLU-dead cells,
    signed bf16 gradients."""
    m = _m()
    g = torch.Generator(device=DEV).manual_seed(3)
    x8 = torch.randint(0, 256, (NB, 61, 73, 61, 8), dtype=torch.uint8, device=DEV, generator=g)
    idx = torch.randperm(NB, device=DEV, generator=g).int()
    shp = (NB, 19, 23, 19, 64)
    dp = torch.randn(shp, device=DEV, generator=g).bfloat16()
    pout = torch.randn(shp, device=DEV, generator=g).bfloat16()           # ~half the cells ReLU-dead
    amax = torch.randint(0, 27, shp, dtype=torch.uint8, device=DEV, generator=g)
    G = NB // B
    nq = m.conv1_wgrad_nq(NB)
    npb = m.conv1_wgrad_mx_npb(NB)
    nblk = (19 + npb - 1) // npb
    parts, grads = [], []
    P = 8000 + 64 * 4
    for mode in (0, mode):
        part = torch.full((NB * 19 * nq, 64, 126), float("nan"), device=DEV)
        grad = torch.zeros(G, P, device=DEV)
        theta = torch.ones(G, P, device=DEV)
        w125 = torch.randn(G, 64, 125, device=DEV, generator=g) * 0 + 0.01
        mu = torch.full((G, 125), 100.0, device=DEV)
        covw = torch.full((G, 64, 125), 0.5, device=DEV)
        inv = torch.full((G, 64), 2.0, device=DEV)
        m.conv1_wgrad_mode(mode)
        m.conv1_wgrad(x8.data_ptr(), idx.data_ptr(), dp.data_ptr(), pout.data_ptr(), amax.data_ptr(), NB, B,
                      part.data_ptr(), w125.data_ptr(), mu.data_ptr(), covw.data_ptr(), inv.data_ptr(), theta.data_ptr(),
                      P, 8000, grad.data_ptr(), P, 0, 8000 + 64, 8000 + 128, 8000 + 192, 1.0 / 255.0, 0, _st())
        torch.cuda.synchronize()
        nsl = B * 19 * nq if mode != 2 else B * nblk  # slabs per client
        part = part[:G * nsl]
        assert torch.isfinite(part).all()
        parts.append(part.view(G, nsl, 64, 126).double().sum(1))
        grads.append(grad)
    m.conv1_wgrad_mode(-1)
    # per-client slab sums: fp32 sums of bf16 x uint8 products in two different orders
    assert _relerr(parts[1], parts[0]) < 1e-5, _relerr(parts[1], parts[0])
    assert float((parts[1] - parts[0]).abs().max()) <= 1e-4 * float(parts[0].abs().max())
    assert _relerr(grads[1], grads[0]) < 1e-5


@pytest.mark.parametrize("signed", [False, True])
def test_alexnet_eval_matches_reference(signed):
    from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D
    from neuroimagedisttraining_amd.ops.reference import eval_logits_reference
    G, B = 2, 3
    store, x8, mom, pl, bl, theta, bufs = _alexnet_setup(G, B, seed=5, signed_gamma=signed)
    for i, n in enumerate(bl.names):
        o, k = bl.offsets[i], bl.numel(i)
        if n.endswith("running_mean"):
            bufs[:, o:o + k] = 0.1 * torch.randn(G, k, device=DEV)
        if n.endswith("running_var"):
            bufs[:, o:o + k] = 0.5 + torch.rand(G, k, device=DEV)
    net = HipAlexNet3D(pl, bl, DEV)
    idx = torch.arange(G * B, dtype=torch.int32, device=DEV)
    out = net.eval_logits(theta, bufs, x8, idx, G, B)
    ref = eval_logits_reference(pl, bl, theta, bufs, store.volumes, B, dtype=torch.float64)
    assert _relerr(out, ref) < 3e-2


def test_clip_sgd_mask_matches_reference():
    m = _m()
    G, P = 3, 2570241
    torch.manual_seed(4)
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    theta = padded_rows(G, P, DEV)
    theta.copy_(torch.randn(G, P, device=DEV))
    grad = padded_rows(G, P, DEV)
    grad.copy_(torch.randn(G, P, device=DEV) * 0.01)
    grad[1] *= 1000  # exercises clipping
    mask = (torch.rand(P, device=DEV) > 0.5).float()
    ref = theta.clone()
    from neuroimagedisttraining_amd.ops.reference import clip_sgd_mask_reference
    clip_sgd_mask_reference(ref, grad.clone(), mask, 0.01, 5e-4)
    ws = torch.empty(m.clip_sgd_mask_workspace(G, P), device=DEV)
    g0 = grad.clone()
    th0 = theta.clone()
    m.clip_sgd_mask(theta.data_ptr(), grad.data_ptr(), 0, mask.data_ptr(), ws.data_ptr(), 0, 0, G, P, theta.stride(0),
                    0.01, 5e-4, 0.0, 1, 10.0, 0, 1, _st())
    torch.cuda.synchronize()
    assert _relerr(theta, ref) < 1e-6
    n1 = float(g0[1, :P].double().norm())
    assert _relerr(grad[1, :P], g0[1, :P] * (10.0 / (n1 + 1e-6))) < 1e-5  # keep_grad: clipped gradient written back
    # keep_grad = 0: identical weights, gradient untouched
    grad2 = padded_rows(G, P, DEV)  # same row stride as theta (the kernel takes one stride)
    grad2.copy_(g0)
    theta.copy_(th0)
    m.clip_sgd_mask(theta.data_ptr(), grad2.data_ptr(), 0, mask.data_ptr(), ws.data_ptr(), 0, 0, G, P, theta.stride(0),
                    0.01, 5e-4, 0.0, 1, 10.0, 0, 0, _st())
    torch.cuda.synchronize()
    assert _relerr(theta, ref) < 1e-6 and torch.equal(grad2, g0)


def test_radix_select_matches_topk():
    m = _m()
    torch.manual_seed(5)
    v = torch.rand(2568064, device=DEV) ** 3
    v = v / v.sum()
    k = int(v.numel() * 0.5)
    st = torch.empty(4, dtype=torch.int32, device=DEV)
    hist = torch.empty(256, dtype=torch.int32, device=DEV)
    m.radix_select_kth(v.data_ptr(), v.numel(), k, st.data_ptr(), hist.data_ptr(), _st())
    mask = torch.empty_like(v)
    m.threshold_mask(v.data_ptr(), v.numel(), st.data_ptr(), mask.data_ptr(), _st())
    thr = torch.topk(v, k, sorted=True).values[-1]
    assert torch.equal(mask, (v >= thr).float())


def test_weighted_rows_sum():
    m = _m()
    C, P = 5, 1000003
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    rows = padded_rows(C, P, DEV)
    rows.copy_(torch.randn(C, P, device=DEV))
    w = torch.rand(C, device=DEV)
    out = torch.empty(P, device=DEV)
    m.weighted_rows_sum(rows.data_ptr(), w.data_ptr(), C, P, rows.stride(0), 0.0, out.data_ptr(), _st())
    torch.cuda.synchronize()
    assert _relerr(out, (w.view(-1, 1) * rows).sum(0)) < 1e-6


@pytest.mark.parametrize("cin,cout,pad,sp", [(64, 128, 0, (9, 11, 9)), (128, 192, 1, (5, 7, 5))])
def test_torch_library_conv3d_k3_autograd(cin, cout, pad, sp):
    """nidt::conv3d_k3 custom op (LDS-DMA fwd, dgrad, row-group wgrad) vs F.conv3d autograd per client."""
    from neuroimagedisttraining_amd.ops import library  # noqa: F401  (registers torch.ops.nidt.*)
    G, B = 2, 2
    torch.manual_seed(3)
    x = torch.randn(G * B, *sp, cin, device=DEV).bfloat16().requires_grad_(True)
    w = (torch.randn(G, cout, cin, 3, 3, 3, device=DEV) * 0.05).requires_grad_(True)
    b = torch.randn(G, cout, device=DEV).requires_grad_(True)
    y = torch.ops.nidt.conv3d_k3(x, w, b, pad)
    dy = torch.randn_like(y)
    y.backward(dy)
    for g in range(G):
        xr = _cf(x[g * B:(g + 1) * B].detach().float()).requires_grad_(True)
        wr = w[g].detach().bfloat16().float().requires_grad_(True)
        br = b[g].detach().clone().requires_grad_(True)
        yr = F.conv3d(xr, wr, br, 1, pad)
        yr.backward(_cf(dy[g * B:(g + 1) * B].float()))
        assert _relerr(y[g * B:(g + 1) * B].float(), _cl(yr.detach())) < 1e-2
        assert _relerr(x.grad[g * B:(g + 1) * B].float(), _cl(xr.grad)) < 1e-2
        assert _relerr(w.grad[g], wr.grad) < 1e-2
        assert _relerr(b.grad[g], br.grad) < 1e-3


def test_torch_library_kth_and_weighted_sum():
    from neuroimagedisttraining_amd.ops import library  # noqa: F401
    v = torch.rand(100003, device=DEV)
    k = 777
    assert float(torch.ops.nidt.kth_largest(v, k)) == float(torch.topk(v, k).values[-1])
    rows = torch.randn(5, 1001, device=DEV)
    wts = torch.rand(5, device=DEV)
    assert torch.allclose(torch.ops.nidt.weighted_rows_sum(rows, wts), (wts[:, None] * rows).sum(0), atol=1e-5)


@pytest.mark.parametrize("cin,cout,pad", [(64, 64, 1), (256, 256, 1), (512, 512, 1), (128, 256, 0)])
def test_hip_conv3d_module_matches_conv3d(cin, cout, pad):
    """HipConv3d (nidt::conv3d_k3, incl. the 512-channel LDS-DMA paths) == F.conv3d fwd + both gradients."""
    from neuroimagedisttraining_amd.ops.modules import HipConv3d
    torch.manual_seed(3)
    conv = HipConv3d(cin, cout, 3, 1, pad, bias=False).to(DEV)
    x = torch.randn(2, cin, 6, 7, 5, device=DEV).to(memory_format=torch.channels_last_3d)
    xa = x.clone().requires_grad_(True)
    y = conv(xa.bfloat16())
    g = torch.randn_like(y.float())
    y.float().backward(g)
    xr = x.bfloat16().float().requires_grad_(True)
    wr = conv.weight.detach().bfloat16().float().requires_grad_(True)
    yr = F.conv3d(xr, wr, None, 1, pad)
    yr.backward(g)
    assert _relerr(y.float(), yr) < 1e-2
    assert _relerr(xa.grad, xr.grad) < 2e-2
    assert _relerr(conv.weight.grad, wr.grad) < 2e-2


def test_resnet3d_bottleneck_with_hip_convs_trains():
    from neuroimagedisttraining_amd.models.resnet3d import resnet3d_50
    from neuroimagedisttraining_amd.ops.modules import HipConv3d, use_hip_convs
    torch.manual_seed(0)
    m = resnet3d_50(num_classes=1, width=16).to(DEV)
    ref = resnet3d_50(num_classes=1, width=16).to(DEV)
    ref.load_state_dict(m.state_dict())
    n = use_hip_convs(m)
    assert n > 0 and sum(isinstance(c, HipConv3d) for c in m.modules()) == n
    assert list(m.state_dict().keys()) == list(ref.state_dict().keys())
    x = torch.randn(2, 1, 32, 36, 32, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(x)
        out_ref = ref(x)
    assert torch.isfinite(out).all() and _relerr(out.float(), out_ref.float()) < 5e-2
    out.float().sum().backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_hip_graph_local_steps_match_eager():
    """FLRunner with hipGraph-captured local steps == the eager launch sequence, bit for bit (same kernels, same
    arguments; only the step-varying scalars move to device memory)."""
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes, to_hip_store
    from neuroimagedisttraining_amd.engine.executor import FLConfig, FLRunner, HipEngine
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.parallel import runtime as rt
    info = rt.DistInfo(device=torch.device(DEV))
    vol, labels, splits = build_fl_volumes(list(range(3)), 3, 32, 8, DEV, seed=5)
    x8, mom = to_hip_store(vol)
    outs = []
    for graphs in (False, True):
        torch.manual_seed(0)
        model = AlexNet3D_Dropout(num_classes=1)
        eng = HipEngine(model, x8, mom, labels, DEV)
        cfg = FLConfig(comm_round=2, epochs=2, batch_size=16, dense_ratio=0.5, seed=3, hip_graphs=graphs)
        r = FLRunner(eng, [splits[c] for c in range(3)], cfg, info, model, algorithm="salientgrads")
        r.generate_global_mask_snip()
        for k in range(2):
            r.run_round(k)
        torch.cuda.synchronize()
        if graphs:
            assert any(isinstance(v, tuple) for v in r._graphs.values()), "no step was captured"
        outs.append((r.w_global.clone(), r.b_global.clone(), r.stat_info["global_test_acc"]))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]


def test_modp_matmul_matches_numpy():
    """K22: TurboAggregate's mod-p encoding product on the GPU == the exact host reference."""
    import numpy as np
    from neuroimagedisttraining_amd.algorithms import turboaggregate as TA
    rng = np.random.RandomState(0)
    p = 2 ** 31 - 1
    A = rng.randint(0, p, size=(7, 5)).astype(np.int64)
    B = rng.randint(0, p, size=(5, 70001)).astype(np.int64)
    ref = np.zeros((7, 70001), dtype=np.int64)
    for k in range(5):
        ref = (ref + (A[:, k:k + 1] * B[k:k + 1, :]) % p) % p
    got = TA.matmul_mod_device(A, B, p)
    assert np.array_equal(got, ref)
    assert np.array_equal(TA._matmul_mod(A, B, p), ref)  # dispatches to the device above the size threshold


def test_rows_nnz_matches_count_nonzero():
    """The per-row non-zero counter of the communication accounting (optim.hip rows_nnz) vs torch."""
    from neuroimagedisttraining_amd.engine.runner import FLRunner
    g = torch.Generator(device=DEV).manual_seed(3)
    for R, K in ((5, 2570241), (1, 1001), (3, 7)):
        m = padded_rows(R, K, DEV)
        m.copy_(torch.randn(R, K, device=DEV, generator=g) * (torch.rand(R, K, device=DEV, generator=g) < 0.3))
        m[0, :3] = torch.tensor([-0.0, float("nan"), 0.0], device=DEV)
        stub = FLRunner.__new__(FLRunner)
        stub.device = torch.device(DEV)
        assert torch.equal(stub._rows_nnz(m), torch.count_nonzero(m, dim=1)), (R, K)
        one = torch.zeros(K + 1, device=DEV)[1:]  # a [K] row at a 4-byte offset: torch fallback path
        assert int(stub._rows_nnz(one.view(1, -1))[0]) == 0
