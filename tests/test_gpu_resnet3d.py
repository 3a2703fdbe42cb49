"""GPU tests of the client-batched 3D ResNet (config 5) path: BatchNorm3d kernels (bnr.hip), the generalised conv
kernels at 3D shapes (1x1x1 GEMM up to 2048 channels, 3x3x3 stride 2 on odd extents, 1x1x1 stride-2 projections)
against fp32 PyTorch, and a whole lockstep train step of a Bottleneck ResNet-50 against per-client autograd."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / (b.norm() + 1e-12))


CONVS = [  # cin, cout, k, stride, (D, H, W)
    (64, 64, 3, 1, (9, 11, 9)),
    (64, 128, 3, 2, (9, 11, 9)),
    (128, 64, 1, 1, (8, 10, 8)),
    (256, 512, 1, 2, (9, 11, 9)),
    (1024, 2048, 1, 1, (3, 4, 3)),
    (512, 512, 3, 1, (4, 5, 4)),
    (64, 128, 3, 2, (8, 10, 8)),    # even extents: every sub-pixel phase full
    (128, 256, 1, 2, (8, 9, 8)),
]


@pytest.mark.parametrize("cin,cout,k,stride,dims", CONVS)
def test_gconv3_fwd_dgrad_wgrad(cin, cout, k, stride, dims):
    from neuroimagedisttraining_amd.engine.resnet3d_hip import GConv3
    dev = _dev()
    torch.manual_seed(cin + cout + k)
    G, B = 2, 2
    conv = GConv3(0, cout, cin, k, stride, (k - 1) // 2)
    P = conv.numel
    theta = torch.zeros(G, P + (-P) % 64, device=dev)[:, :P]
    theta.copy_(torch.randn(G, P, device=dev) * (2.0 / (cin * k ** 3)) ** 0.5)
    x = torch.randn(G * B, *dims, cin, device=dev).to(torch.bfloat16)
    y = conv.fwd(x, theta, G, train=True)
    xr = x.float().permute(0, 4, 1, 2, 3).requires_grad_(True)
    wr = theta.view(G, cout, cin, k, k, k).to(torch.bfloat16).float().requires_grad_(True)
    ref = torch.cat([F.conv3d(xr[g * B:(g + 1) * B], wr[g], stride=stride, padding=(k - 1) // 2) for g in range(G)])
    assert tuple(y.shape) == (G * B, *ref.shape[2:], cout)
    assert _rel(y.permute(0, 4, 1, 2, 3), ref) < 1e-2
    dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
    ref.backward(dy.float().permute(0, 4, 1, 2, 3))
    grads = torch.zeros_like(theta)
    dx = conv.bwd(dy, x, theta, grads, G)
    torch.cuda.synchronize()
    assert _rel(grads.view(G, cout, cin, k, k, k), wr.grad) < 2e-2
    if k == 1 and stride == 2:  # half-resolution gradient of the even voxels (res_grad_s2 adds it)
        g_ = xr.grad
        assert float(g_[:, :, 1::2].abs().max()) == 0 and float(g_[:, :, :, 1::2].abs().max()) == 0
        assert float(g_[:, :, :, :, 1::2].abs().max()) == 0
        assert tuple(dx.shape) == (G * B, *ref.shape[2:], cin)
        assert _rel(dx.permute(0, 4, 1, 2, 3), g_[:, :, ::2, ::2, ::2]) < 2e-2
        return
    assert tuple(dx.shape) == tuple(x.shape)
    assert _rel(dx.permute(0, 4, 1, 2, 3), xr.grad) < 2e-2


def test_weight_packer_images_exact():
    """pack.hip (chunked plain grid, 1x1 grid, transpose grid) for a mix of layers — 3x3x3 at 64/192/512 input
    channels (one, three, eight 64-channel chunks), a channel-padded 2-D stem (cin 3 -> 64), 3x3 and 1x1 — against the
    permuted fp32 rows rounded to bf16, bit for bit; the dgrad image with the taps in each layer's slot order."""
    from neuroimagedisttraining_amd.engine.resnet2d_hip import GroupedConv, WeightPacker
    from neuroimagedisttraining_amd.engine.resnet3d_hip import GConv3
    dev = _dev()
    specs = [("3", 128, 64, 3, 1), ("3", 64, 192, 3, 1), ("3", 64, 512, 3, 2), ("3", 256, 128, 1, 1),
             ("2", 64, 3, 3, 1), ("2", 128, 64, 3, 2), ("2", 128, 64, 1, 2)]
    convs, off = [], 0
    for kind, cout, cin, k, st in specs:
        c = GConv3(off, cout, cin, k, st, (k - 1) // 2) if kind == "3" else \
            GroupedConv(off, cout, cin, k, st, (k - 1) // 2, True)
        convs.append(c)
        off += c.numel + 3  # unaligned layer offsets exercise the scalar source path
    G = 3
    theta = torch.randn(G, off + 64, device=dev)[:, :off]
    pk = WeightPacker(convs, dev)
    pk.pack(theta, G, True)
    torch.cuda.synchronize()
    for c in convs:
        w = theta[:, c.off:c.off + c.numel].reshape(G, c.cout, c.cin, c.kt)
        ref = torch.zeros(G, c.cout, c.kt, c.cin_p, device=dev)
        ref[..., :c.cin] = w.permute(0, 1, 3, 2)
        ref = ref.to(torch.bfloat16)
        assert torch.equal(c.wp[0].view(torch.int16), ref.view(torch.int16)), (c.cout, c.cin, c.kt)
        if c.wt is not None:
            slots = list(c.slots)
            rt = torch.empty(G, c.cin_p, c.kt, c.cout, device=dev, dtype=torch.bfloat16)
            for t in range(c.kt):
                rt[:, :, slots[t], :] = ref[:, :, t, :].transpose(1, 2)
            assert torch.equal(c.wt[0].view(torch.int16), rt.view(torch.int16)), (c.cout, c.cin, c.kt)


G1_SHAPES = [(64, 256), (64, 128), (64, 64), (128, 256), (128, 128), (128, 64), (256, 128), (256, 64), (512, 64),
             (512, 128), (256, 1024)]


@pytest.mark.parametrize("K,N", G1_SHAPES)
def test_gemm1x1_matches_fp32(K, N):
    """gemm1x1.hip (every tile configuration) against a per-client fp32 matmul of the same bf16 operands, with a
    row count that leaves a partial last m-tile and blocks with different tile counts."""
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    m = ops.ext()
    assert m.gemm1x1_ok(K, N)
    torch.manual_seed(K + N)
    G = 3
    # a row count with a partial last m-tile, and one where some block's tile count T has T % 3 == 2 (its last tile's
    # out-of-range DMA targets the stage array the [STATS] reduction reuses: the drain before that reduction)
    bm = 32 if K == 512 else 64
    mgs = [2 * 64 * 9 + 37]
    for mg in range(64 * 3, 64 * 400, 64 * 7 + 11):
        nch, nmt = m.gemm1x1_chunks(G, mg, K, N), (mg + bm - 1) // bm
        if any(((nmt - 1 - mb) // nch + 1) % 3 == 2 for mb in range(min(nch, nmt))):
            mgs.append(mg)
            break
    assert len(mgs) == 2
    for Mg in mgs:
        _gemm1x1_case(m, dev, G, Mg, K, N)


def _gemm1x1_case(m, dev, G, Mg, K, N):
    x = torch.randn(G, Mg, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(G, N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    y = torch.full((G, Mg, N), float("nan"), device=dev).to(torch.bfloat16)
    nch = m.gemm1x1_chunks(G, Mg, K, N)
    part = torch.full((nch, G, N, 2), float("nan"), device=dev)
    m.gemm1x1_g(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, Mg, K, N, part.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
    ref = torch.bmm(x.float(), w.float().transpose(1, 2))
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    assert _rel(y, ref) < 5e-3
    assert float((y.float() - ref).abs().max()) <= 2 ** -7 * float(ref.abs().max())
    # [STATS] epilogue: per-client channel sums of the stored bf16 outputs and of their squares
    ps = part.double().sum(0)
    yf = y.double()
    assert _rel(ps[..., 0], yf.sum(1)) < 1e-5 and _rel(ps[..., 1], (yf * yf).sum(1)) < 1e-5
    y2 = torch.empty_like(y)
    m.gemm1x1_g(x.data_ptr(), w.data_ptr(), y2.data_ptr(), G, Mg, K, N, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(y2.view(torch.int16), y.view(torch.int16))  # the statistics do not change the output


W1_SHAPES = [(64, 64), (256, 64), (64, 256), (128, 128), (128, 256), (256, 128), (512, 128), (128, 512),
             (1024, 2048)]


@pytest.mark.parametrize("N,K", W1_SHAPES)
def test_wgrad1x1_matches_fp32(N, K):
    """wgrad1x1.hip (every tile configuration; one chunk = gradient rows written by the kernel, several = partials +
    k_wgrad_reduce) against a per-client fp32 dY^T X of the same bf16 operands, with a partial last m-tile; the rows
    around each client's gradient slice stay untouched."""
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    m = ops.ext()
    assert m.wgrad1x1_ok(N, K)
    torch.manual_seed(N + K)
    G, Mg = 3, 64 * 37 + 21
    x = torch.randn(G, Mg, K, device=dev).to(torch.bfloat16)
    dy = torch.randn(G, Mg, N, device=dev).to(torch.bfloat16)
    ref = torch.bmm(dy.float().transpose(1, 2), x.float()) * 0.5
    off, ld = 7, N * K + 19
    for nmb in sorted({1, 3, m.wgrad1x1_chunks(G, Mg, N, K)}):
        rows = torch.full((G, ld), -3.0, device=dev)
        part = torch.empty(max(nmb, 1) * G * N * K, device=dev)
        m.wgrad1x1_g(x.data_ptr(), dy.data_ptr(), part.data_ptr(), rows.data_ptr(), ld, off, G, Mg, N, K, nmb, 0.5,
                     torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = rows[:, off:off + N * K].view(G, N, K)
        assert _rel(got, ref) < 1e-5, nmb
        assert float(rows[:, :off].sub(-3.0).abs().max()) == 0 and float(rows[:, off + N * K:].sub(-3.0).abs().max()) == 0


def test_gemm1x1_operand_above_2_31_elements():
    """An X operand of more than 2^31 elements (64-bit client bases): the last client's last rows — the largest
    offsets — against a chunked fp32 reference."""
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    m = ops.ext()
    G, Mg, K, N = 32, 270001, 256, 64
    assert G * Mg * K > 2 ** 31
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.empty(G, Mg, K, device=dev, dtype=torch.bfloat16)
    for g in range(G):  # chunked fill: no fp32 temporary of the whole operand
        x[g].copy_(torch.randn(Mg, K, device=dev, generator=gen))
    w = (torch.randn(G, N, K, device=dev, generator=gen) * K ** -0.5).to(torch.bfloat16)
    y = torch.empty(G, Mg, N, device=dev, dtype=torch.bfloat16)
    m.gemm1x1_g(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, Mg, K, N, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for g, rows in ((G - 1, slice(Mg - 4096, Mg)), (G // 2, slice(0, 4096)), (0, slice(Mg - 100, Mg))):
        ref = x[g, rows].float() @ w[g].float().t()
        assert _rel(y[g, rows], ref) < 5e-3, g
    del x, y
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dims", [(9, 11, 9), (8, 10, 8)])
def test_res_grad_s2_3d_matches_torch(dims):
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    N, C = 3, 64
    D, H, W = dims
    dx1 = torch.randn(N, D, H, W, C, device=dev).to(torch.bfloat16)
    sub = torch.randn(N, (D + 1) // 2, (H + 1) // 2, (W + 1) // 2, C, device=dev).to(torch.bfloat16)
    out = torch.empty(N, D, H, W, C, device=dev)
    ops.ext().res_grad_s2(out.data_ptr(), dx1.data_ptr(), sub.data_ptr(), N, D, H, W, C, 0,
                          torch.cuda.current_stream().cuda_stream)
    want = dx1.float().clone()
    want[:, ::2, ::2, ::2] += sub.float()
    outb = torch.empty(N, D, H, W, C, device=dev, dtype=torch.bfloat16)  # the engines' bf16 gradient stream
    ops.ext().res_grad_s2(outb.data_ptr(), dx1.data_ptr(), sub.data_ptr(), N, D, H, W, C, 1,
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(out, want)
    assert torch.equal(outb, want.to(torch.bfloat16))


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_res_grad_dtypes_match_torch(flags):
    """out = dx1 + da * (mask > 0) (identity block) and out = dx1 + dx2 (projection), fp32 or bf16 in and out."""
    from neuroimagedisttraining_amd import ops
    dev = _dev()
    n = 4 * 9 * 64
    dx1 = torch.randn(n, device=dev).to(torch.bfloat16)
    dx2 = torch.randn(n, device=dev).to(torch.bfloat16)
    da = torch.randn(n, device=dev).to(torch.bfloat16 if flags & 2 else torch.float32)
    mask = torch.relu(torch.randn(n, device=dev)).to(torch.bfloat16)
    odt = torch.bfloat16 if flags & 1 else torch.float32
    st = torch.cuda.current_stream().cuda_stream
    o1, o2 = torch.empty(n, device=dev, dtype=odt), torch.empty(n, device=dev, dtype=odt)
    ops.ext().res_grad(o1.data_ptr(), dx1.data_ptr(), 0, da.data_ptr(), mask.data_ptr(), n, flags, st)
    ops.ext().res_grad(o2.data_ptr(), dx1.data_ptr(), dx2.data_ptr(), 0, 0, n, flags, st)
    torch.cuda.synchronize()
    assert torch.equal(o1, (dx1.float() + da.float() * (mask > 0)).to(odt))
    assert torch.equal(o2, (dx1.float() + dx2.float()).to(odt))


@pytest.mark.parametrize("C,dims,res", [(64, (6, 7, 6), True), (256, (3, 4, 3), False), (2048, (1, 2, 1), True)])
def test_bnr_train_eval_fwd_bwd_match_torch(C, dims, res):
    from neuroimagedisttraining_amd.engine.resnet3d_hip import GBN3
    dev = _dev()
    torch.manual_seed(C)
    G, B = 3, 2
    theta = torch.zeros(G, 2 * C + 64, device=dev)
    theta[:, :C] = torch.randn(G, C, device=dev)
    theta[:, C:2 * C] = torch.randn(G, C, device=dev)
    bufs = torch.zeros(G, 2 * C + 64, device=dev)
    bufs[:, C:2 * C] = 1.0
    bn = GBN3(0, C, C, 0, C, 2 * C)
    t = (torch.randn(G * B, *dims, C, device=dev) * 2 + 0.5).to(torch.bfloat16)
    r = torch.randn_like(t.float()).to(torch.bfloat16) if res else None
    y, st = bn.fwd(t, theta, bufs, G, True, res=r, relu=True)
    tr = t.float().requires_grad_(True)
    gam = theta[:, :C].clone().requires_grad_(True)
    bet = theta[:, C:2 * C].clone().requires_grad_(True)
    rm = torch.zeros(G, C, device=dev)
    rv = torch.ones(G, C, device=dev)
    outs = []
    for g in range(G):
        xg = tr[g * B:(g + 1) * B].permute(0, 4, 1, 2, 3)
        o = F.batch_norm(xg, rm[g], rv[g], gam[g], bet[g], training=True, momentum=0.1, eps=1e-5)
        o = o.permute(0, 2, 3, 4, 1)
        if res:
            o = o + r[g * B:(g + 1) * B].float()
        outs.append(torch.relu(o))
    ref = torch.cat(outs)
    assert _rel(y, ref) < 1e-2
    assert torch.allclose(bufs[:, :C], rm, atol=1e-4, rtol=1e-3) and torch.allclose(bufs[:, C:2 * C], rv, atol=1e-3,
                                                                                     rtol=1e-3)
    assert torch.all(bufs[:, 2 * C] == 1.0)
    dy = torch.randn(y.shape, device=dev)
    ref.backward(dy)
    grads = torch.zeros_like(theta)
    dt = bn.bwd(dy, y, t, st, theta, grads, G)
    torch.cuda.synchronize()
    assert _rel(dt, tr.grad) < 2e-2
    assert _rel(grads[:, :C], gam.grad) < 1e-2 and _rel(grads[:, C:2 * C], bet.grad) < 1e-2
    # eval mode: running statistics
    ye, _ = bn.fwd(t, theta, bufs, G, False)
    refe = torch.cat([F.batch_norm(t[g * B:(g + 1) * B].float().permute(0, 4, 1, 2, 3), bufs[g, :C], bufs[g, C:2 * C],
                                   theta[g, :C], theta[g, C:2 * C], training=False, eps=1e-5).permute(0, 2, 3, 4, 1)
                      for g in range(G)])
    assert _rel(ye, refe) < 1e-2


def _bf16_faithful(model, conv_dtype=torch.bfloat16):
    """Round the reference's activations to bf16 where the HIP path stores them (conv outputs, ReLU outputs, the
    projection BN output), so the comparison checks the wiring, not bf16 error growth through 16 blocks with
    batch statistics over a few voxels."""
    def rnd(mod, inp, out):
        return out.to(conv_dtype).float()
    for name, mod in model.named_modules():
        if isinstance(mod, (torch.nn.Conv3d, torch.nn.ReLU)) or name.endswith("downsample.1"):
            mod.register_forward_hook(rnd)
    return model


def test_resnet3d_lockstep_step_matches_per_client_autograd():
    """A 4-stage Bottleneck 3D ResNet (one block per stage, every block with a projection) on 72x80x72 volumes:
    enough voxels per BatchNorm statistic that bf16 rounding does not swamp the comparison (the full ResNet-50 is
    wiring-checked in fp32 by tests/test_cpu_resnet3d.py; its deepest BN layers see 16 voxels per channel)."""
    from torch.func import functional_call
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
    from neuroimagedisttraining_amd.models.resnet3d import Bottleneck, ResNet3D
    dev = _dev()
    torch.manual_seed(0)
    G, B = 2, 2
    vol = torch.randint(0, 256, (G * B, 72, 80, 72), dtype=torch.uint8, device=dev)
    lab = torch.tensor([0.0, 1.0, 1.0, 0.0], device=dev)
    resnet3d_50 = lambda num_classes: ResNet3D(Bottleneck, [1, 1, 1, 1], num_classes)  # noqa: E731
    m = resnet3d_50(num_classes=1)
    eng = ResNet3DHipEngine(m, vol, lab, dev)
    L, Lb = eng.players, eng.blayers
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
    bflat = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()]).to(dev)
    th, gr = padded_rows(G, L.total, dev), padded_rows(G, L.total, dev)
    bu = padded_rows(G, Lb.total, dev)
    th.copy_(flat.expand(G, -1))
    bu.copy_(bflat.expand(G, -1))
    idx = torch.arange(G * B, dtype=torch.int32, device=dev)
    losses = eng.train_step(th, bu, gr, idx, G, B, 1.0, 0)
    torch.cuda.synchronize()
    mref = _bf16_faithful(resnet3d_50(num_classes=1).to(dev))
    mref.train()
    ctx = torch.backends.cudnn.flags(enabled=False)  # native BN backward (see test_stem_hip_fwd_bwd_match_torch)
    ctx.__enter__()
    conv_names = {n + ".weight" for n, mod in mref.named_modules() if isinstance(mod, torch.nn.Conv3d)}
    for g in range(G):
        row = flat.clone().requires_grad_(True)
        pv = {n: (row[o:o + L.numel(i)].view(L.shapes[i]).to(torch.bfloat16).float() if n in conv_names else
                  row[o:o + L.numel(i)].view(L.shapes[i])) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        bv = {n: bflat[o:o + Lb.numel(i)].view(Lb.shapes[i]).clone().to(Lb.dtypes[i])
              for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets))}
        x = vol[g * B:(g + 1) * B].float().unsqueeze(1) / 255.0  # the HIP stem reads exact uint8 values
        out = functional_call(mref, {**pv, **bv}, (x,))
        loss = F.binary_cross_entropy_with_logits(out.view(-1), lab[g * B:(g + 1) * B])
        loss.backward()
        assert abs(float(loss) - float(losses[g])) < 0.02, (float(loss), float(losses[g]))
        for i, (n, o) in enumerate(zip(L.names, L.offsets)):
            if n.endswith("conv2.weight") or n in ("conv1.weight", "fc.weight"):
                a, b = gr[g, o:o + L.numel(i)], row.grad[o:o + L.numel(i)]
                cos = float(a @ b / (a.norm() * b.norm()))
                assert cos > 0.9, (n, cos)
        # running statistics advanced like nn.BatchNorm3d
        for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets)):
            if n.endswith("running_mean"):
                assert torch.allclose(bu[g, o:o + Lb.numel(i)], bv[n].float(), atol=2e-2, rtol=5e-2), n
    ctx.__exit__(None, None, None)
    lg = eng.eval_logits(th, bu, idx, G, B)
    assert lg.shape == (G * B, 1) and torch.isfinite(lg).all()


@pytest.mark.parametrize("env", ["NIDT_R3D_OMASK", "NIDT_R3D_TMASK", "NIDT_R3D_RESBN"])
def test_resnet3d_omask_bit_identical(monkeypatch, env):
    """[OMASK]: the residual-gradient kernel applying the previous block's ReLU mask (BN3 / downsample-BN backward and
    identity shortcuts then read no mask) gives bit-identical gradients, losses and running statistics to masking in
    the BN backward — identity and projection blocks, stride-2 projections.  [TMASK]: bn1 / bn2 backward recomputing
    their ReLU mask from the pre-BN tensor, likewise bit-identical to reading the stored output.  [RESBN]: the
    residual-gradient pass reducing the next bn3 / downsample-BN backward statistics, bit-identical to their own pass."""
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
    from neuroimagedisttraining_amd.models.resnet3d import Bottleneck, ResNet3D
    dev = _dev()
    torch.manual_seed(3)
    G, B = 2, 2
    vol = torch.randint(0, 256, (G * B, 40, 44, 40), dtype=torch.uint8, device=dev)
    lab = torch.tensor([0.0, 1.0, 1.0, 0.0], device=dev)
    m = ResNet3D(Bottleneck, [2, 2, 1, 1], 1)
    eng = ResNet3DHipEngine(m, vol, lab, dev)
    L, Lb = eng.players, eng.blayers
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
    bflat = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()]).to(dev)
    idx = torch.arange(G * B, dtype=torch.int32, device=dev)
    outs = []
    for om in ("0", "1"):
        monkeypatch.setenv(env, om)
        th, gr, bu = padded_rows(G, L.total, dev), padded_rows(G, L.total, dev), padded_rows(G, Lb.total, dev)
        th.copy_(flat.expand(G, -1) + 0.01 * torch.randn(G, L.total, device=dev, generator=torch.Generator(
            device=dev).manual_seed(1)))
        bu.copy_(bflat.expand(G, -1))
        gr.zero_()
        losses = eng.train_step(th, bu, gr, idx, G, B, 1.0, 0)
        torch.cuda.synchronize()
        outs.append((losses.clone(), gr.clone(), bu.clone()))
    (l0, g0, b0), (l1, g1, b1) = outs
    assert torch.equal(l0, l1) and torch.equal(b0, b1)
    assert float(g0.abs().sum()) > 0 and torch.equal(g0, g1)


def test_resnet3d_pack_fuse_per_group_bit_identical(monkeypatch):
    """[PACK-FUSE-G]: FedAvg rounds through the runner with two row groups of one launch shape (step-major plan: the
    groups' steps interleave), the optimizer writing each group's next-step weight images into that group's buffer,
    give bit-identical client rows and global model to packing every step from theta."""
    import numpy as np
    from neuroimagedisttraining_amd.engine import resnet3d_hip as R3
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, FLRunner
    from neuroimagedisttraining_amd.models.resnet3d import Bottleneck, ResNet3D
    from neuroimagedisttraining_amd.parallel import runtime as rt
    dev = _dev()
    torch.manual_seed(5)
    nc, ntr, nte = 4, 8, 2
    vol = torch.randint(0, 256, (nc * (ntr + nte), 40, 44, 40), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 2, (nc * (ntr + nte),), device=dev).float()
    splits = [ClientSplit(np.arange(c * 10, c * 10 + ntr), np.arange(c * 10 + ntr, c * 10 + 10)) for c in range(nc)]
    model = ResNet3D(Bottleneck, [1, 1, 1, 1], 1)
    out = []
    for fuse in (False, True):
        monkeypatch.setattr(R3, "_PACK_FUSE_G", fuse)
        monkeypatch.setattr(R3.ResNet3DHipEngine, "fused_pack", fuse)
        eng = R3.ResNet3DHipEngine(model, vol, lab, dev)
        info = rt.DistInfo(0, 1, 0, torch.device(dev), "none")
        r = FLRunner(eng, splits, FLConfig(comm_round=2, epochs=1, batch_size=2, lr=0.01, seed=3, frac=1.0, group=2),
                     info, model)
        for k in range(2):
            r.run_round(k)
        torch.cuda.synchronize()
        if fuse:
            assert any(len(k) == 4 for k in eng.net.packer._plans), "no per-group image buffer was used"
            assert eng.net.packer.fresh_hits > 0, "no step reused optimizer-written images"
        out.append((r.theta.clone(), r.w_global.clone()))
    (t0, w0), (t1, w1) = out
    assert torch.equal(t0, t1) and torch.equal(w0, w1)


@pytest.mark.parametrize("G,B,dims", [(2, 1, (121, 145, 121)), (2, 2, (21, 26, 22)), (3, 1, (9, 128, 13)),
                                        (2, 2, (15, 20, 10))])
def test_stem_hip_fwd_bwd_match_torch(G, B, dims):
    """stem.hip (polyphase 7^3/s2 conv on MFMA + BN statistics, BN+ReLU+3^3/s2 max-pool, the backward with the MFMA
    weight gradient) against fp32 PyTorch autograd of Conv3d(1, 64, 7, 2, 3) -> BatchNorm3d -> ReLU -> MaxPool3d,
    per client; full ABCD extents and odd/even small ones (the ABCD and 15 x 20 x 10 extents, 8-byte polyphase rows,
    take the one-block-for-all-jd weight gradient k_stem_wgrad4, the others k_stem_wgrad).  The reference rounds the
    weights and the conv output to bf16 where the HIP path stores them."""
    from neuroimagedisttraining_amd.engine.resnet3d_hip import GroupedResNet3D
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.flat import ParamLayout
    from neuroimagedisttraining_amd.models.resnet3d import Bottleneck, ResNet3D
    dev = _dev()
    torch.manual_seed(G * 100 + dims[0])
    m = ResNet3D(Bottleneck, [1, 1, 1, 1], 1)
    L = ParamLayout.from_tensors(list(m.named_parameters()))
    Lb = ParamLayout.from_tensors(list(m.named_buffers()))
    net = GroupedResNet3D(L, Lb, dev)
    N = G * B
    th = padded_rows(G, L.total, dev)
    th.copy_(torch.randn(G, L.total, device=dev) * 0.05)
    o = dict(zip(L.names, L.offsets))
    th[:, o["bn1.weight"]:o["bn1.weight"] + 64] = 1 + 0.2 * torch.randn(G, 64, device=dev)
    bu = padded_rows(G, Lb.total, dev)
    bo = dict(zip(Lb.names, Lb.offsets))
    bu[:, bo["bn1.running_var"]:bo["bn1.running_var"] + 64] = 1.0
    store = torch.randint(0, 256, (N + 3, *dims), dtype=torch.uint8, device=dev)
    idx = torch.randperm(N + 3, device=dev)[:N].to(torch.int32)
    out, saved = net._stem_hip(store, idx, th, bu, G, True)
    da = torch.randn(out.shape, device=dev).to(torch.bfloat16).float()  # the engine's gradient stream is bf16
    gr = torch.zeros_like(th)
    net._stem_hip_bwd(saved, da, th, gr, G)
    torch.cuda.synchronize()
    x = store[idx.long()].float().unsqueeze(1) / 255.0
    # PyTorch's native kernels, not MIOpen: MIOpen's BatchNorm backward misses part of dbeta for some channels at
    # these small shapes (sum of the BN-output gradient != beta.grad by a constant), which the weight gradient of
    # the conv below amplifies (tools/debug/stem_debug.py, profiles/r3_stem_debug.txt)
    ctx = torch.backends.cudnn.flags(enabled=False)
    ctx.__enter__()
    for g in range(G):
        w = th[g, o["conv1.weight"]:o["conv1.weight"] + 64 * 343].view(64, 1, 7, 7, 7).to(torch.bfloat16).float()
        w.requires_grad_(True)
        gam = th[g, o["bn1.weight"]:o["bn1.weight"] + 64].clone().requires_grad_(True)
        bet = th[g, o["bn1.bias"]:o["bn1.bias"] + 64].clone().requires_grad_(True)
        rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
        c = F.conv3d(x[g * B:(g + 1) * B], w, stride=2, padding=3)
        c = c + (c.to(torch.bfloat16).float() - c).detach()  # bf16 store, straight-through gradient
        z = F.max_pool3d(torch.relu(F.batch_norm(c, rm, rv, gam, bet, True, 0.1, 1e-5)), 3, 2, 1)
        ref = z.permute(0, 2, 3, 4, 1)
        assert tuple(out[g * B:(g + 1) * B].shape) == tuple(ref.shape)
        assert _rel(out[g * B:(g + 1) * B], ref) < 1e-2, g
        ref.backward(da[g * B:(g + 1) * B])
        gw = gr[g, o["conv1.weight"]:o["conv1.weight"] + 64 * 343].view(64, 1, 7, 7, 7)
        assert _rel(gw, w.grad) < 2e-2, (g, _rel(gw, w.grad))
        assert _rel(gr[g, o["bn1.weight"]:o["bn1.weight"] + 64], gam.grad) < 2e-2
        assert _rel(gr[g, o["bn1.bias"]:o["bn1.bias"] + 64], bet.grad) < 1e-2
        assert torch.allclose(bu[g, bo["bn1.running_mean"]:bo["bn1.running_mean"] + 64], rm, atol=1e-4, rtol=1e-3)
        assert torch.allclose(bu[g, bo["bn1.running_var"]:bo["bn1.running_var"] + 64], rv, atol=1e-4, rtol=1e-3)
    # eval mode: the running statistics just written
    oute, none = net._stem_hip(store, idx, th, bu, G, False)
    assert none is None
    for g in range(G):
        w = th[g, o["conv1.weight"]:o["conv1.weight"] + 64 * 343].view(64, 1, 7, 7, 7).to(torch.bfloat16).float()
        c = F.conv3d(x[g * B:(g + 1) * B], w, stride=2, padding=3).to(torch.bfloat16).float()
        z = F.batch_norm(c, bu[g, bo["bn1.running_mean"]:bo["bn1.running_mean"] + 64],
                         bu[g, bo["bn1.running_var"]:bo["bn1.running_var"] + 64],
                         th[g, o["bn1.weight"]:o["bn1.weight"] + 64], th[g, o["bn1.bias"]:o["bn1.bias"] + 64], False)
        ref = F.max_pool3d(torch.relu(z), 3, 2, 1).permute(0, 2, 3, 4, 1)
        assert _rel(oute[g * B:(g + 1) * B], ref) < 1e-2
    ctx.__exit__(None, None, None)
