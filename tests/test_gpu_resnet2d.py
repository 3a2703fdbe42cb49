"""GPU tests of the client-batched ResNet-18-GN (CIFAR) path: the generalised conv kernels (9-tap 2-D 3x3 at stride
1/2, 1x1 stride-2 projections, the channel-padded stem) against fp32 PyTorch convolutions, and the full lockstep
train step against the engine's fp32 CPU twin (itself checked against per-client autograd in
tests/test_cpu_resnet2d.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


CONVS = [  # (cin, cout, k, stride, pad, hw)
    (64, 64, 3, 1, 1, 32),
    (3, 64, 3, 1, 1, 32),
    (64, 128, 3, 2, 1, 32),
    (64, 128, 1, 2, 0, 32),
    (128, 256, 3, 2, 1, 16),
    (256, 256, 3, 1, 1, 8),
    (256, 512, 1, 2, 0, 8),
    (512, 512, 3, 1, 1, 4),
    (64, 128, 3, 2, 1, 15),   # odd input: the last odd-phase row/column of dX has no dy row below it
    (64, 64, 3, 1, 1, 64),    # Tiny-ImageNet layer-1 maps
    (64, 128, 3, 2, 1, 64),
]


@pytest.mark.parametrize("cin,cout,k,stride,pad,hw", CONVS)
def test_grouped_conv2d_fwd_dgrad_wgrad(cin, cout, k, stride, pad, hw):
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupedConv
    dev = _dev()
    torch.manual_seed(cin * 7 + cout + k + stride)
    G, B = 3, 2
    conv = GroupedConv(0, cout, cin, k, stride, pad, hip=True)
    P = conv.numel
    ld = (P + 63) // 64 * 64
    theta = torch.zeros(G, ld, device=dev)[:, :P]
    theta.copy_(torch.randn(G, P, device=dev) * (2.0 / (cin * k * k)) ** 0.5)
    x = torch.zeros(G * B, hw, hw, conv.cin_p, device=dev, dtype=torch.bfloat16)
    x[..., :cin] = torch.randn(G * B, hw, hw, cin, device=dev).to(torch.bfloat16)
    y = conv.fwd(x, theta, G)
    # fp32 reference on the same (bf16-rounded) operands
    xr = x[..., :cin].float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = theta.view(G, cout, cin, k, k).to(torch.bfloat16).float().requires_grad_(True)
    ref = torch.cat([F.conv2d(xr[g * B:(g + 1) * B], wr[g], stride=stride, padding=pad) for g in range(G)])
    assert tuple(y.shape) == (G * B, ref.shape[2], ref.shape[3], cout)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2
    dy = torch.randn_like(y.float()).to(torch.bfloat16)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    grads = torch.zeros(G, ld, device=dev)[:, :P]
    dx = conv.bwd(dy, x, theta, grads, G, need_dx=(cin % 64 == 0))
    torch.cuda.synchronize()
    assert _rel(grads.view(G, cout, cin, k, k), wr.grad) < 2e-2
    if dx is not None:
        if k == 1 and stride == 2:  # half-resolution gradient of the even pixels (res_grad_s2 adds it)
            assert tuple(dx.shape) == (G * B, ref.shape[2], ref.shape[3], conv.cin_p)
            assert float(xr.grad[:, :, 1::2].abs().max()) == 0.0 and float(xr.grad[:, :, :, 1::2].abs().max()) == 0.0
            assert _rel(dx.permute(0, 3, 1, 2)[:, :cin], xr.grad[:, :, ::2, ::2]) < 2e-2
        else:
            assert tuple(dx.shape) == tuple(x.shape)
            assert _rel(dx.permute(0, 3, 1, 2)[:, :cin], xr.grad) < 2e-2


@pytest.mark.parametrize("cin,cout,k,stride,pad,hw", [(512, 512, 3, 1, 1, 4), (256, 256, 3, 1, 1, 8),
                                                      (256, 512, 3, 2, 1, 8)])
def test_conv_fwd_splitk_matches_single_pass(cin, cout, k, stride, pad, hw):
    """Split-K forward (``conv_fwd_gk``, partial sums + k_fwd_splitk_sum) at several split factors against the
    single-pass kernel and fp32 PyTorch; the small-grid deep layers pick ks > 1 by themselves."""
    from neuroimagedisttraining_amd import ops
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupedConv, _stream
    dev = _dev()
    m = ops.ext()
    torch.manual_seed(cin + cout + stride)
    G, B = 3, 2
    conv = GroupedConv(0, cout, cin, k, stride, pad, hip=True)
    kt = k * k
    assert m.conv_fwd_g_ksplit(G, B, 1, hw, hw, cin, cout, kt, stride, pad, 0) > 1
    theta = torch.randn(G, conv.numel, device=dev) * (2.0 / (cin * kt)) ** 0.5
    wp, _ = conv._wp(theta, G, False)
    x = torch.randn(G * B, hw, hw, cin, device=dev).to(torch.bfloat16)
    Ho, Wo = conv.out_hw(hw, hw)
    y1 = torch.empty(G * B, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
    m.conv_fwd_g(x.data_ptr(), wp.data_ptr(), y1.data_ptr(), G, B, 1, hw, hw, cin, cout, kt, stride, pad, 0,
                 _stream())
    xr = x.float().permute(0, 3, 1, 2)
    wr = theta.view(G, cout, cin, k, k).to(torch.bfloat16).float()
    ref = torch.cat([F.conv2d(xr[g * B:(g + 1) * B], wr[g], stride=stride, padding=pad) for g in range(G)])
    for ks in (2, 5, 8):
        part = torch.full((ks * G * B * Ho * Wo * cout,), float("nan"), device=dev)
        yk = torch.empty_like(y1)
        m.conv_fwd_gk(x.data_ptr(), wp.data_ptr(), yk.data_ptr(), part.data_ptr(), ks, G, B, 1, hw, hw, cin, cout, kt,
                      stride, pad, 0, _stream())
        torch.cuda.synchronize()
        assert torch.isfinite(yk.float()).all(), ks
        assert _rel(yk, y1) < 1e-2, ks
        assert _rel(yk.permute(0, 3, 1, 2), ref) < 1e-2, ks


def test_resnet18gn_train_step_matches_cpu_twin():
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    torch.manual_seed(0)
    G, B = 4, 8
    x8, y = synthetic_cifar(G * B, seed=3)
    m = customized_resnet18(class_num=10)
    hip = ResNetHipEngine(m, x8, y, dev)
    cpu = ResNetHipEngine(m, x8, y, "cpu")
    P = hip.players.total
    th = torch.cat([torch.cat([p.detach().reshape(-1) for p in customized_resnet18(class_num=10).parameters()])[None]
                    for _ in range(G)])
    th_d, gr_d = padded_rows(G, P, dev), padded_rows(G, P, dev)
    th_c, gr_c = padded_rows(G, P, "cpu"), padded_rows(G, P, "cpu")
    th_d.copy_(th)
    th_c.copy_(th)
    idx = torch.arange(G * B, dtype=torch.int32)
    ld = hip.train_step(th_d, None, gr_d, idx.to(dev), G, B, 1.0, 0)
    lc = cpu.train_step(th_c, None, gr_c, idx, G, B, 1.0, 0)
    torch.cuda.synchronize()
    assert torch.allclose(ld.cpu(), lc, atol=3e-2), (ld, lc)
    for g in range(G):
        a, b = gr_d[g].cpu(), gr_c[g]
        cos = float(a @ b / (a.norm() * b.norm()))
        assert cos > 0.98, (g, cos)
    lg = hip.eval_logits(th_d, None, idx.to(dev), G, B)
    assert lg.shape == (G * B, 10) and torch.isfinite(lg).all()


def test_resnet18gn_hip_runners_graphs_match_eager():
    """SubAvg and DisPFL on the ResNet engine: hipGraph-replayed local steps == eager, bit for bit."""
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
    from neuroimagedisttraining_amd.models import customized_resnet18
    from neuroimagedisttraining_amd.parallel import runtime as rt
    dev = _dev()
    info = rt.init_distributed(prefer_gpu=True)
    C, ntr, nte = 4, 20, 8
    x8, y = synthetic_cifar(C * (ntr + nte), seed=5)
    splits = [ClientSplit(train=np.arange(c * (ntr + nte), c * (ntr + nte) + ntr - 3 * c),
                          test=np.arange(c * (ntr + nte) + ntr, (c + 1) * (ntr + nte))) for c in range(C)]
    for alg in ("subavg", "dispfl"):
        outs = []
        for graphs in (False, True):
            torch.manual_seed(0)
            m = customized_resnet18(class_num=10)
            eng = ResNetHipEngine(m, x8, y, dev)
            cfg = FLConfig(comm_round=2, epochs=2, batch_size=8, dense_ratio=0.3, seed=1, frac=0.5, lr=0.05,
                           frequency_of_the_test=1, final_round=False, hip_graphs=graphs)
            r = make_runner(alg, eng, splits, cfg, info, m)
            for k in range(2):
                r.run_round(k)
            torch.cuda.synchronize()
            outs.append(r.theta.clone())
        assert torch.isfinite(outs[0]).all()
        assert torch.equal(outs[0], outs[1]), alg


@pytest.mark.parametrize("hw,C", [(32, 64), (16, 128), (8, 256), (4, 512), (64, 64), (32, 128), (6, 64), (7, 128)])
@pytest.mark.parametrize("res,dy_bf16", [(False, True), (True, False)])
def test_groupnorm_kernels_match_torch(hw, C, res, dy_bf16):
    """gn.hip forward (affine + residual + ReLU) and backward (ReLU mask, dgamma/dbeta rows) vs the fp32 CPU
    twin on the same bf16 inputs."""
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupNormG
    dev = _dev()
    torch.manual_seed(hw + C)
    G, B = 3, 2
    N = G * B
    theta = torch.zeros(G, 2 * C + 64, device=dev)
    theta[:, :C] = torch.randn(G, C, device=dev)           # signed gammas
    theta[:, C:2 * C] = torch.randn(G, C, device=dev)
    t = (torch.randn(N, hw, hw, C, device=dev) * 3 + 1).to(torch.bfloat16)
    r = torch.randn(N, hw, hw, C, device=dev).to(torch.bfloat16) if res else None
    hipgn, cpugn = GroupNormG(0, C, C, hip=True), GroupNormG(0, C, C, hip=False)
    y, st = hipgn.fwd(t, theta, G, res=r, relu=True)
    yc, stc = cpugn.fwd(t.cpu(), theta.cpu(), G, res=r.cpu() if res else None, relu=True)
    assert _rel(y.cpu(), yc) < 1e-2
    dy = torch.randn(N, hw, hw, C, device=dev)
    dy = dy.to(torch.bfloat16) if dy_bf16 else dy
    gh = torch.zeros_like(theta)
    gc = torch.zeros_like(theta.cpu())
    dt = hipgn.bwd(dy, y, t, st, theta, gh, G)
    dtc = cpugn.bwd(dy.cpu(), yc, t.cpu(), stc, theta.cpu(), gc, G)
    torch.cuda.synchronize()
    assert _rel(dt.cpu(), dtc) < 2e-2
    assert _rel(gh.cpu()[:, :2 * C], gc[:, :2 * C]) < 1e-3


def test_tap_slots_twin_matches_kernel_plan():
    from neuroimagedisttraining_amd import ops
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    _dev()
    m = ops.ext()
    for kt, st in ((9, 1), (9, 2), (1, 2), (1, 1)):
        py = R.tap_slots(kt, st) if kt != 9 or st != 2 else None
        got = list(m.conv_tap_slots(kt, st))
        assert sorted(got) == list(range(kt))
        if py is not None:
            assert got == py
    # the 2-D phase order of the Python twin (used by the CPU path) equals the kernel's
    import neuroimagedisttraining_amd.engine.resnet2d_hip as RR
    real = RR.torch.cuda.is_available
    RR.torch.cuda.is_available = lambda: False
    try:
        assert RR.tap_slots(9, 2) == list(m.conv_tap_slots(9, 2))
    finally:
        RR.torch.cuda.is_available = real


@pytest.mark.parametrize("hw", [32, 64])
def test_fused_input_stage_matches_twin(hw):
    """img.hip (gather + RandomCrop(pad 4) + flip with on-device draws + normalise + channel pad) == the CPU twin
    with the same (step seed, client, position) draws; without augmentation == plain normalisation."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    G, B = 3, 5
    g = np.random.default_rng(hw)
    x8 = torch.from_numpy(g.integers(0, 256, size=(40, hw, hw, 3)).astype(np.uint8))
    idx = torch.from_numpy(g.permutation(40)[:G * B].astype(np.int32))
    mean, std = (R.TINY_MEAN, R.TINY_STD) if hw == 64 else (R.CIFAR_MEAN, R.CIFAR_STD)
    L = ParamLayout.from_tensors(list(customized_resnet18(class_num=10).named_parameters()))
    hip = R.GroupedResNet18GN(L, dev, mean=mean, std=std)
    cpu = R.GroupedResNet18GN(L, "cpu", mean=mean, std=std)
    seed_dev = torch.tensor([123456], dtype=torch.int64, device=dev)
    cids = [7, 2, 11]
    cids_dev = torch.tensor(cids, dtype=torch.int32, device=dev)
    assert hip.stem.fold  # [STEM-FOLD] is the default on the HIP path
    xc = cpu.input(x8, idx, (seed_dev.cpu(), 5 << 40, None, cids, B))
    xcp = cpu.input(x8, idx)
    for fold in (False, True):
        hip.stem.fold = fold
        xa = hip.input(x8.to(dev), idx.to(dev), (seed_dev, 5 << 40, cids_dev, cids, B))
        xp = hip.input(x8.to(dev), idx.to(dev))
        torch.cuda.synchronize()
        ea, ep = (R.fold_window(xc), R.fold_window(xcp)) if fold else (xc, xcp)
        live = 27 if fold else 3
        assert xa.shape == (G * B, hw, hw, 64) and float(xa[..., live:].float().abs().max()) == 0.0
        assert torch.allclose(xa.cpu().float(), ea.float(), atol=2e-2, rtol=0), fold
        assert torch.allclose(xp.cpu().float(), ep.float(), atol=2e-2, rtol=0), fold
        assert not torch.allclose(xa.float(), xp.float(), atol=0.1)


def test_stem_fold_matches_padded_stem():
    """[STEM-FOLD]: the stem as a 1x1 conv over the window-folded input == the channel-padded 9-tap stem (forward
    output and the stem's weight-gradient row), same weights, same augmented batch."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    torch.manual_seed(1)
    G, B, hw = 3, 4, 32
    m = customized_resnet18(class_num=10)
    L = ParamLayout.from_tensors(list(m.named_parameters()))
    net = R.GroupedResNet18GN(L, dev)
    P = L.total
    th = padded_rows(G, P, dev)
    th.copy_(torch.randn(G, P, device=dev) * 0.1)
    x8 = torch.from_numpy(np.random.default_rng(2).integers(0, 256, size=(G * B, hw, hw, 3)).astype(np.uint8)).to(dev)
    idx = torch.arange(G * B, dtype=torch.int32, device=dev)
    st = net.stem
    outs = []
    for fold in (False, True):
        st.fold = fold
        x = net.input(x8, idx)
        net.packer.pack(th, G, True, key=("t", fold))
        y = st.fwd(x, th, G, train=True, packed=True)
        dy = (torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(3))).to(y.dtype)
        gr = padded_rows(G, P, dev)
        gr.zero_()
        st.bwd(dy, x, th, gr, G, False)
        torch.cuda.synchronize()
        outs.append((y.float(), gr[:, st.off:st.off + st.numel].clone()))
    (y0, g0), (y1, g1) = outs
    assert _rel(y1, y0) < 1e-2
    assert _rel(g1, g0) < 1e-3


def test_tiny_resnet18_train_step_matches_cpu_twin():
    """64x64 Tiny-ImageNet ResNet-18-GN (200 classes, streaming GroupNorm on the 64x64 maps, sub-pixel dgrads) on
    the HIP path vs the engine's fp32 CPU twin (itself checked against autograd in tests/test_cpu_augment.py)."""
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine
    from neuroimagedisttraining_amd.models import tiny_resnet18
    dev = _dev()
    torch.manual_seed(0)
    G, B = 3, 4
    g = np.random.default_rng(8)
    x8 = torch.from_numpy(g.integers(0, 256, size=(G * B, 64, 64, 3)).astype(np.uint8))
    y = torch.from_numpy(g.integers(0, 200, size=G * B))
    m = tiny_resnet18(class_num=200)
    hip = ResNetHipEngine(m, x8, y, dev)
    cpu = ResNetHipEngine(m, x8, y, "cpu")
    P = hip.players.total
    th = torch.cat([p.detach().reshape(-1) for p in tiny_resnet18(class_num=200).parameters()])[None].expand(G, -1)
    th_d, gr_d = padded_rows(G, P, dev), padded_rows(G, P, dev)
    th_c, gr_c = padded_rows(G, P, "cpu"), padded_rows(G, P, "cpu")
    th_d.copy_(th)
    th_c.copy_(th)
    idx = torch.arange(G * B, dtype=torch.int32)
    sd = torch.tensor([99], dtype=torch.int64)
    ld = hip.train_step(th_d, None, gr_d, idx.to(dev), G, B, 1.0, 7, cids=[0, 1, 2], seed_dev=sd.to(dev))
    lc = cpu.train_step(th_c, None, gr_c, idx, G, B, 1.0, 7, cids=[0, 1, 2], seed_dev=sd)
    torch.cuda.synchronize()
    assert torch.allclose(ld.cpu(), lc, atol=3e-2), (ld, lc)
    for gi in range(G):
        a, b = gr_d[gi].cpu(), gr_c[gi]
        cos = float(a @ b / (a.norm() * b.norm()))
        assert cos > 0.98, (gi, cos)
    lg = hip.eval_logits(th_d, None, idx.to(dev), G, B)
    assert lg.shape == (G * B, 200) and torch.isfinite(lg).all()


@pytest.mark.parametrize("hw,K,G,B", [(4, 10, 3, 16), (8, 200, 2, 5), (4, 100, 1, 7)])
def test_fused_cls_head_matches_torch_head(hw, K, G, B, monkeypatch):
    """``cls_head_train`` (pool + linear + CrossEntropy forward/backward, two launches) against the engine's torch
    head on the same final map: per-client losses, dW / db rows and the bf16 input gradient."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    torch.manual_seed(K + B)
    L = ParamLayout.from_tensors(list(customized_resnet18(class_num=K).named_parameters()))
    net = R.GroupedResNet18GN(L, dev)
    P = L.total
    ld = (P + 63) // 64 * 64
    theta = torch.zeros(G, ld, device=dev)[:, :P]
    theta.copy_(torch.randn(G, P, device=dev) * 0.05)
    a = torch.relu(torch.randn(G * B, hw, hw, 512, device=dev)).to(torch.bfloat16)
    y = torch.randint(0, K, (G * B,), device=dev)
    assert net._fused_head(theta)
    g1 = torch.zeros(G, ld, device=dev)[:, :P]
    l1, da1 = net._head_train(a, theta, g1, y, G, B)
    monkeypatch.setenv("NIDT_CLS_HEAD", "0")
    assert not net._fused_head(theta)
    g0 = torch.zeros(G, ld, device=dev)[:, :P]
    l0, da0 = net._head_train(a, theta, g0, y, G, B)
    torch.cuda.synchronize()
    assert _rel(l1, l0) < 1e-5
    sl = slice(net.lw_off, net.lw_off + K * 512)
    assert _rel(g1[:, sl], g0[:, sl]) < 1e-5
    sb = slice(net.lb_off, net.lb_off + K)
    assert _rel(g1[:, sb], g0[:, sb]) < 1e-5
    assert da1.dtype == da0.dtype == torch.bfloat16 and da1.shape == da0.shape
    assert _rel(da1, da0) < 1e-2
    assert float(g1[:, :net.lw_off].abs().max()) == 0.0  # nothing outside the head rows written


@pytest.mark.parametrize("mask_mode", [0, 1])
@pytest.mark.parametrize("wt", [False, True])
def test_optimizer_written_images_equal_pack(mask_mode, wt, monkeypatch):
    """[PACK-FUSE] local_opt(pack_next=True) (optim.hip k_local_step_pack) updates theta, momentum and gradients bit for
    bit like the plain step, writes the forward images k_pack_plain would write from the updated rows, and the next
    step (which skips the plain pack) gives the same loss and gradients.  [PACK-WT] (wt): the tiled step
    (k_local_step_pack_wt) also writes the data-gradient images, bit for bit those of k_pack_trans."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    monkeypatch.setattr(R, "_PACK_WT", wt)
    from neuroimagedisttraining_amd.engine import masks as MK
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet2d_hip import ResNetHipEngine, synthetic_cifar
    from neuroimagedisttraining_amd.engine.runner import StepSpec
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    torch.manual_seed(3)
    G, B = 3, 8
    m = customized_resnet18(class_num=10)
    x8, y = synthetic_cifar(G * B, seed=2)
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
    out = {}
    for fused in (False, True):
        eng = ResNetHipEngine(m, x8, y, dev)
        P = eng.players.total
        theta = padded_rows(G, P, dev)
        theta.copy_(flat.expand(G, -1) + 0.01 * torch.randn(G, P, device=dev, generator=torch.Generator(dev).manual_seed(5)))
        grads, mom = padded_rows(G, P, dev), padded_rows(G, P, dev)
        spec = StepSpec()
        if mask_mode:
            keep = (torch.rand(G, P, device=dev, generator=torch.Generator(dev).manual_seed(7)) < 0.4).float()
            spec = StepSpec(mask_mode=1, bits=MK.pack_bits(keep))
            theta.mul_(keep)
        idx = torch.arange(G * B, dtype=torch.int32, device=dev)
        seed = torch.tensor([11], dtype=torch.int64, device=dev)
        losses = []
        for step in range(3):
            losses.append(eng.train_step(theta, None, grads, idx, G, B, 1.0, 1 << 40, seed_dev=seed).clone())
            eng.local_opt(theta, grads, mom, spec, 0.05, 5e-4, 0.9, 10.0, pack_next=fused and step < 2)
            if fused and step == 0:  # step 1 then runs on the images written by step 0's optimizer (checked here)
                pk = eng.net.packer
                key = pk.last[0]
                assert key in pk.fresh and pk.fresh[key][2] == wt
                buf, views = pk._plans[key][4], pk._plans[key][5]
                fwd = [buf[o:o + int(np.prod(shp))] for (o, shp), _ in views]  # the forward images
                if wt:  # ... and the data-gradient images
                    fwd += [buf[vt[0]:vt[0] + int(np.prod(vt[1]))] for _, vt in views if vt is not None]
                got = [v.clone() for v in fwd]
                pk.fresh.clear()
                pk.pack(theta, G, True, key=key)  # the plain pack from the updated rows
                torch.cuda.synchronize()
                for li, (a, b) in enumerate(zip(got, fwd)):
                    assert torch.equal(a, b), (step, li)
                pk.fresh[key] = (theta.data_ptr(), theta._version, wt)  # restore: the next step reuses the images
        torch.cuda.synchronize()
        out[fused] = (theta.clone(), mom.clone(), torch.stack(losses))
    assert torch.equal(out[False][0], out[True][0])
    assert torch.equal(out[False][1], out[True][1])
    assert torch.equal(out[False][2], out[True][2])


@pytest.mark.parametrize("B,hw,cin,cout", [(6, 8, 64, 64), (5, 8, 256, 256), (3, 8, 128, 256), (4, 6, 64, 128),
                                           (16, 4, 512, 512), (13, 4, 256, 512), (9, 4, 512, 128)])
def test_slab_batched_depth_matches_fp32(B, hw, cin, cout):
    """[SLAB-BD] 2-D 3x3 convs whose blocks span several samples, as the depth planes of one volume restricted to
    depth tap 1 (conv2d_fwd_slab_bd), against fp32 F.conv2d per client on the same bf16 operands."""
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    m = ops.ext()
    if not m.conv2d_fwd_slab_bd_ok(B, hw, hw, cin, cout):
        pytest.skip("shape not eligible")
    G = 2
    torch.manual_seed(B * hw + cin)
    x = torch.randn(G * B, hw, hw, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(G, cout, 9, cin, device=dev) * (9 * cin) ** -0.5).to(torch.bfloat16)
    y = torch.empty(G * B, hw, hw, cout, device=dev, dtype=torch.bfloat16)
    tab = torch.empty(m.conv2d_fwd_slab_bd_table_size(B, hw, hw, cin, cout), device=dev, dtype=torch.int32)
    m.conv2d_fwd_slab_bd_table(tab.data_ptr(), B, hw, hw, cin, cout, ops.stream())
    m.conv2d_fwd_slab_bd(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, hw, hw, cin, cout, tab.data_ptr(), ops.stream())
    torch.cuda.synchronize()
    for g in range(G):
        xr = x[g * B:(g + 1) * B].float().permute(0, 3, 1, 2)
        wr = w[g].float().view(cout, 3, 3, cin).permute(0, 3, 1, 2)
        ref = F.conv2d(xr, wr, padding=1).permute(0, 2, 3, 1)
        assert _rel(y[g * B:(g + 1) * B].float(), ref) < 1e-2, g


@pytest.mark.parametrize("P,shared,src", [(1000, False, False), (1000, True, True), (4103, False, True), (37, False, False)])
def test_masked_rows_matches_unpack(P, shared, src):
    """masks.masked_rows (optim.hip k_masked_rows) == the torch unpack-and-multiply, tails and shared masks included."""
    from neuroimagedisttraining_amd.engine import masks as MK
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    dev = _dev()
    C = 5
    torch.manual_seed(P)
    rows = padded_rows(C, P, dev)
    rows[:, :P] = torch.randn(C, P, device=dev)
    keep = torch.rand(1 if shared else C, P, device=dev) < 0.4
    bits = MK.pack_bits(keep)
    s = torch.randn(P, device=dev) if src else None
    ref = ((s.view(1, -1) if src else rows[:, :P]) * keep.float()).clone()
    out = MK.masked_rows(rows, bits, src=s, P=P)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :P], ref.expand(C, -1))


@pytest.mark.parametrize("P", [1000, 4103, 37, 64])
def test_unpack_bits_kernel_matches_torch(P):
    """masks.unpack_bits on the device (k_unpack_bits, bool and fp32) == the torch bit arithmetic on the CPU."""
    from neuroimagedisttraining_amd.engine import masks as MK
    dev = _dev()
    torch.manual_seed(P)
    keep = torch.rand(3, P) < 0.3
    bits = MK.pack_bits(keep)
    for dt in (torch.bool, torch.float32):
        got = MK.unpack_bits(bits.to(dev), P, dt).cpu()
        assert torch.equal(got, MK.unpack_bits(bits, P, dt)), dt
        assert torch.equal(got.bool(), keep)


def test_gn_recomputed_masks_bit_identical(monkeypatch):
    """[GN-RMASK] + [OMASK]: the block's first GroupNorm backward recomputing its ReLU mask from t, and the residual
    gradient carrying the previous block's output mask (so the second / shortcut norms read no mask), give the same
    loss and gradient rows bit for bit as the mask-tensor backward (CIFAR and Tiny map sizes)."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    for hw in (32, 64):
        G, B = 3, 4
        g = np.random.default_rng(hw)
        x8 = torch.from_numpy(g.integers(0, 256, size=(G * B, hw, hw, 3)).astype(np.uint8))
        y = torch.from_numpy(g.integers(0, 10, size=G * B))
        m = customized_resnet18(class_num=10)
        P = sum(p.numel() for p in m.parameters())
        flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
        res = []
        for on in (False, True):
            monkeypatch.setattr(R, "_GN_RMASK", on)
            monkeypatch.setattr(R, "_OMASK2D", on)
            eng = R.ResNetHipEngine(m, x8, y, dev)
            th, gr = padded_rows(G, P, dev), padded_rows(G, P, dev)
            th.copy_(flat.expand(G, -1))
            gr.zero_()
            idx = torch.arange(G * B, dtype=torch.int32, device=dev)
            loss = eng.train_step(th, None, gr, idx, G, B, 1.0, 0)
            torch.cuda.synchronize()
            res.append((loss.clone(), gr.clone()))
        assert torch.equal(res[0][0], res[1][0]), hw
        assert torch.isfinite(res[1][1]).all() and float(res[1][1].abs().sum()) > 0
        assert torch.equal(res[0][1], res[1][1]), (hw, float((res[0][1] - res[1][1]).abs().max()))


@pytest.mark.parametrize("hw", [32, 64])
def test_gn_epilogue_statistics_match_gn_kernel(hw, monkeypatch):
    """[GN-EPI]: GroupNorm forward from the slab conv epilogue's per-block statistics (conv2d_fwd_slab_stats +
    k_gn_apply) against the per-sample k_gn_fwd on the same conv output: the normalised activations agree to bf16
    rounding, the saved (mean, rstd) to fp32 rounding of the pre-/post-bf16 sums, and a whole train step's loss and
    gradient rows stay close to the k_gn_fwd path (the statistics come from the fp32 accumulators, not the bf16 t)."""
    from neuroimagedisttraining_amd.engine import resnet2d_hip as R
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.models import customized_resnet18
    dev = _dev()
    torch.manual_seed(hw)
    G, B, C = 3, 4, 64
    conv = R.GroupedConv(0, C, C, 3, 1, 1, hip=True)
    gn = R.GroupNormG(conv.numel, conv.numel + C, C, hip=True)
    P = conv.numel + 2 * C
    theta = torch.zeros(G, (P + 63) // 64 * 64, device=dev)[:, :P]
    theta[:, :conv.numel] = torch.randn(G, conv.numel, device=dev) * (2.0 / (9 * C)) ** 0.5
    theta[:, conv.numel:] = torch.randn(G, 2 * C, device=dev)
    x = torch.randn(G * B, hw, hw, C, device=dev).to(torch.bfloat16)
    t = conv.fwd(x, theta, G, gn_stats=True)
    assert conv.gn_part is not None and conv.gn_part[1] == hw * hw // 256
    r = torch.randn_like(t.float()).to(torch.bfloat16)
    y1, s1 = gn.fwd(t, theta, G, res=r, relu=True, part=conv.gn_part)
    y0, s0 = gn.fwd(t, theta, G, res=r, relu=True)
    torch.cuda.synchronize()
    assert _rel(y1, y0) < 1e-2
    assert torch.allclose(s1[..., 0], s0[..., 0], atol=2e-2) and torch.allclose(s1[..., 1], s0[..., 1], rtol=1e-2)
    # whole step
    m = customized_resnet18(class_num=10)
    g = np.random.default_rng(hw)
    x8 = torch.from_numpy(g.integers(0, 256, size=(G * B, hw, hw, 3)).astype(np.uint8))
    yl = torch.from_numpy(g.integers(0, 10, size=G * B))
    Pm = sum(p.numel() for p in m.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
    res = []
    for on in (False, True):
        monkeypatch.setattr(R, "_GN_EPI", on)
        eng = R.ResNetHipEngine(m, x8, yl, dev)
        th, gr = padded_rows(G, Pm, dev), padded_rows(G, Pm, dev)
        th.copy_(flat.expand(G, -1))
        loss = eng.train_step(th, None, gr, torch.arange(G * B, dtype=torch.int32, device=dev), G, B, 1.0, 0)
        torch.cuda.synchronize()
        res.append((loss.clone(), gr.clone()))
    assert torch.allclose(res[0][0], res[1][0], atol=2e-2), (res[0][0], res[1][0])
    for gi in range(G):
        a, b = res[0][1][gi], res[1][1][gi]
        assert float(a @ b / (a.norm() * b.norm())) > 0.99
