"""Diagnostics for stem.hip: per-stage comparison (conv output, pooled, dz, dgamma/dbeta, dW by tap plane)
against fp32 autograd for one client.  Usage: python tools/debug/stem_debug.py D H W [B]"""
import sys
import os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from neuroimagedisttraining_amd import ops  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    D, H, W = (int(v) for v in sys.argv[1:4])
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    dev = torch.device("cuda")
    m, st = ops.ext(), torch.cuda.current_stream().cuda_stream
    torch.manual_seed(0)
    G, N, C = 1, B, 64
    x8 = torch.randint(0, 256, (N, D, H, W), dtype=torch.uint8, device=dev)
    idx = torch.arange(N, dtype=torch.int32, device=dev)
    P = 64 * 343 + 128
    theta = torch.zeros(1, P + 64, device=dev)
    theta[0, :64 * 343] = torch.randn(64 * 343, device=dev) * 0.05
    theta[0, 64 * 343:64 * 343 + 64] = 1 + 0.2 * torch.randn(64, device=dev)
    theta[0, 64 * 343 + 64:64 * 343 + 128] = 0.1 * torch.randn(64, device=dev)
    ow, og, ob = 0, 64 * 343, 64 * 343 + 64
    bufs = torch.zeros(1, 192, device=dev)
    bufs[0, 64:128] = 1
    sz = m.stem_sizes(N, D, H, W)
    Od, Oh, Ow = (D - 1) // 2 + 1, (H - 1) // 2 + 1, (W - 1) // 2 + 1
    Qd, Qh, Qw = (Od - 1) // 2 + 1, (Oh - 1) // 2 + 1, (Ow - 1) // 2 + 1
    xp = torch.empty(sz[0], device=dev, dtype=torch.uint8)
    xq = torch.empty(sz[0], device=dev, dtype=torch.uint8)
    m.stem_polyphase(x8.data_ptr(), idx.data_ptr(), N, D, H, W, xp.data_ptr(), xq.data_ptr(), st)
    y = torch.empty(N, Od, Oh, Ow, C, device=dev, dtype=torch.bfloat16)
    stats = torch.empty(sz[3], device=dev)
    wk = torch.empty(sz[5], device=dev, dtype=torch.bfloat16)
    m.stem_fwd(xp.data_ptr(), theta.data_ptr(), theta.stride(0), ow, N, B, D, H, W, wk.data_ptr(), y.data_ptr(),
               stats.data_ptr(), st)
    coef = torch.empty(4, C, device=dev)
    m.bn_finalize(stats.data_ptr(), B * Od, Oh * Ow, B * Od * Oh * Ow, 1, C, theta.data_ptr(), theta.stride(0), og, ob,
                  bufs.data_ptr(), bufs.stride(0), 0, 64, 128, 0.1, 1e-5, *[coef[i].data_ptr() for i in range(4)], 1,
                  st)
    out = torch.empty(N, Qd, Qh, Qw, C, device=dev, dtype=torch.bfloat16)
    amax = torch.empty(N, Qd, Qh, Qw, C, device=dev, dtype=torch.uint8)
    m.stem_pool(y.data_ptr(), coef[0].data_ptr(), coef[1].data_ptr(), N, B, D, H, W, out.data_ptr(), amax.data_ptr(),
                st)
    da = torch.randn(out.shape, device=dev).to(torch.bfloat16)  # bf16 pooled gradient (the engine's stream)
    grads = torch.zeros_like(theta)
    dz = torch.empty_like(y)
    part = torch.empty(sz[3], device=dev)
    bco = torch.empty(C * 3, device=dev)
    slab = torch.empty(sz[4], device=dev)
    m.stem_bwd(da.data_ptr(), amax.data_ptr(), y.data_ptr(), xq.data_ptr(), *[coef[i].data_ptr() for i in range(4)], N,
               B, D, H, W, theta.data_ptr(), theta.stride(0), og, grads.data_ptr(), grads.stride(0), ow, og, ob,
               dz.data_ptr(), part.data_ptr(), bco.data_ptr(), slab.data_ptr(), st)
    torch.cuda.synchronize()
    # reference (NIDT_DEBUG_MIOPEN=1: with MIOpen's BatchNorm, whose backward misses part of dbeta at small shapes)
    torch.backends.cudnn.enabled = os.environ.get("NIDT_DEBUG_MIOPEN") == "1"
    x = x8.float().unsqueeze(1) / 255
    w = theta[0, :64 * 343].view(64, 1, 7, 7, 7).to(torch.bfloat16).float().requires_grad_(True)
    gam = theta[0, og:og + 64].clone().requires_grad_(True)
    bet = theta[0, ob:ob + 64].clone().requires_grad_(True)
    c = F.conv3d(x, w, stride=2, padding=3)
    c.retain_grad()
    cb = c + (c.to(torch.bfloat16).float() - c).detach()
    bn = F.batch_norm(cb, torch.zeros(64, device=dev), torch.ones(64, device=dev), gam, bet, True, 0.1, 1e-5)
    bn.retain_grad()
    r = torch.relu(bn)
    z = F.max_pool3d(r, 3, 2, 1)
    z.permute(0, 2, 3, 4, 1).backward(da.float())
    print("conv y rel", rel(y.permute(0, 4, 1, 2, 3), c))
    print("pooled rel", rel(out.permute(0, 4, 1, 2, 3), z))
    print("mean rel", rel(coef[2], c.mean((0, 2, 3, 4))), "invstd rel",
          rel(coef[3], 1 / torch.sqrt(cb.var((0, 2, 3, 4), unbiased=False) + 1e-5)))
    dzr = bn.grad * (bn > 0)  # gradient wrt relu input = dz (wrt BN output) masked
    print("dz rel", rel(dz.permute(0, 4, 1, 2, 3), bn.grad), "(masked ref)", rel(dz.permute(0, 4, 1, 2, 3), dzr))
    print("dgamma rel", rel(grads[0, og:og + 64], gam.grad), "dbeta rel", rel(grads[0, ob:ob + 64], bet.grad))
    dzp = dz.permute(0, 4, 1, 2, 3).float()
    print("dbeta ours", grads[0, ob:ob + 4].tolist(), "ref", bet.grad[:4].tolist())
    print("sum dz(ours,bf16)", dzp.sum((0, 2, 3, 4))[:4].tolist(), "sum bn.grad", bn.grad.sum((0, 2, 3, 4))[:4].tolist())
    bad = (dzp - bn.grad).abs() > 0.02 * bn.grad.abs() + 1e-3
    print("dz mismatches", int(bad.sum()), "of", bad.numel(), "nonzero ours", int((dzp != 0).sum()), "ref",
          int((bn.grad != 0).sum()))
    if bad.any():
        nz = bad.nonzero()[:8]
        for q in nz.tolist():
            n_, c_, d_, h_, w_ = q
            print("  at", q, "ours", float(dzp[n_, c_, d_, h_, w_]), "ref", float(bn.grad[n_, c_, d_, h_, w_]),
                  "bn", float(bn[n_, c_, d_, h_, w_]))
    # dy = a dz + b y + d vs autograd's gradient at the conv output
    a_, b_, d_ = bco.view(64, 3).unbind(1)
    dy = a_ * dz.float() + b_ * y.float() + d_
    print("dy rel", rel(dy.permute(0, 4, 1, 2, 3), c.grad))
    gw = grads[0, :64 * 343].view(64, 1, 7, 7, 7)
    print("dW rel", rel(gw, w.grad))
    for kd in range(7):
        print(" kd", kd, "rel", round(rel(gw[:, :, kd], w.grad[:, :, kd]), 5), " kh", kd, round(rel(gw[:, :, :, kd], w.grad[:, :, :, kd]), 5),
              " kw", kd, round(rel(gw[..., kd], w.grad[..., kd]), 5))
    # dW from the reference dy (isolates the wgrad kernel)
    dyr = dy.permute(0, 4, 1, 2, 3).contiguous()
    wg = torch.nn.grad.conv3d_weight(x, w.shape, dyr, stride=2, padding=3)
    print("dW(kernel) vs conv3d_weight(our dy) rel", rel(gw, wg))


if __name__ == "__main__":
    main()
