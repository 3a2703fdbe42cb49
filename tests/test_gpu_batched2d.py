"""GPU check of the vmapped client-batched engine for the non-ResNet image models (engine/batched2d.py): a bf16
lockstep step on the MI355X against the fp32 CPU step on the same rows and augmentation draws, then one SubAvg
round through the fused HIP optimizer."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_batched2d_gpu_step_tracks_fp32_and_round_runs():
    from neuroimagedisttraining_amd.engine.batched2d import BatchedModuleEngine
    from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, padded_rows
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.engine.resnet2d_hip import CIFAR_MEAN, CIFAR_STD, synthetic_cifar
    from neuroimagedisttraining_amd.models import create_model
    from neuroimagedisttraining_amd.parallel import runtime as rt
    G, B = 4, 8
    torch.manual_seed(0)
    model = create_model("cnn_cifar10", dataset="cifar10", class_num=10)
    x8, y = synthetic_cifar(G * B, seed=1)
    L = None
    out = {}
    for dev in ("cpu", "cuda"):
        eng = BatchedModuleEngine(create_model("cnn_cifar10", dataset="cifar10", class_num=10), x8, y, dev,
                                  CIFAR_MEAN, CIFAR_STD)
        L = eng.players
        theta = padded_rows(G, L.total, dev)
        theta.copy_(torch.cat([p.detach().reshape(-1) for p in model.parameters()]).to(dev).expand(G, -1))
        grads = padded_rows(G, L.total, dev)
        loss = eng.train_step(theta, None, grads, torch.arange(G * B, dtype=torch.int32, device=dev), G, B, 1.0,
                              1 << 40, cids=[3, 1, 4, 2], seed_dev=torch.tensor([9], dtype=torch.int64, device=dev))
        out[dev] = (loss.float().cpu(), grads.float().cpu())
    assert torch.allclose(out["cpu"][0], out["cuda"][0], atol=3e-2), (out["cpu"][0], out["cuda"][0])
    for g in range(G):
        a, b = out["cpu"][1][g], out["cuda"][1][g]
        cos = float(torch.dot(a, b) / (a.norm() * b.norm()))
        assert cos > 0.99, (g, cos)
    N, per = 6, 12
    x8, y = synthetic_cifar(N * per, seed=3)
    splits = [ClientSplit(np.arange(c * per, c * per + 9), np.arange(c * per + 9, (c + 1) * per)) for c in range(N)]
    eng = BatchedModuleEngine(model, x8, y, "cuda", CIFAR_MEAN, CIFAR_STD)
    cfg = FLConfig(comm_round=1, epochs=1, batch_size=4, lr=0.05, dense_ratio=0.5, seed=1, frac=1.0)
    r = make_runner("subavg", eng, splits, cfg, rt.DistInfo(device=torch.device("cuda")), model)
    before = r.theta.clone()
    res = r.run_round(0)
    torch.cuda.synchronize()
    assert torch.isfinite(r.theta).all() and not torch.equal(before, r.theta)
    assert all(np.isfinite(float(v)) for v in res.values() if isinstance(v, (float, int)))


C2_SHAPES = [  # cin, cout, k, pad, H
    (1, 20, 5, 0, 28), (20, 50, 5, 0, 12), (3, 6, 5, 0, 32), (6, 16, 5, 0, 14), (3, 64, 5, 0, 32), (64, 64, 5, 0, 14),
    (1, 32, 5, 2, 28), (32, 64, 5, 2, 14), (3, 64, 3, 1, 32), (64, 128, 3, 1, 16), (256, 512, 3, 1, 4),
    (512, 512, 3, 1, 2)]


@pytest.mark.parametrize("cin,cout,k,pad,H", C2_SHAPES)
def test_conv2d_any_fwd_dgrad_wgrad_match_fp32(cin, cout, k, pad, H):
    """conv2d_any.hip (forward, data gradient through the flipped image, weight and bias gradients) against fp32
    autograd of the same bf16-rounded operands, per client."""
    import torch.nn.functional as F
    from neuroimagedisttraining_amd.engine.conv2d_hip import HipConv2dFn
    G, B = 3, 4
    torch.manual_seed(cin * 7 + cout + k)
    x = torch.randn(G * B, cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(G, cout, cin, k, k, device="cuda") * (cin * k * k) ** -0.5).requires_grad_(True)
    b = (torch.randn(G, cout, device="cuda") * 0.1).requires_grad_(True)
    xr = x.float().requires_grad_(True)
    y = HipConv2dFn.apply(x.requires_grad_(True), w, b, G, pad)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    ref = torch.cat([F.conv2d(xr[g * B:(g + 1) * B], wr[g], br[g], padding=pad) for g in range(G)])
    assert y.shape == ref.shape
    rel = lambda a, c: float((a.float() - c).norm() / (c.norm() + 1e-12))  # noqa: E731
    assert rel(y, ref) < 1e-2
    dy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16)
    y.backward(dy)
    ref.backward(dy.float())
    torch.cuda.synchronize()
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2
    assert rel(b.grad, br.grad) < 1e-3


@pytest.mark.parametrize("name,ds", [("lenet5", "mnist"), ("cnn_cifar10", "cifar10"), ("vgg11", "cifar10")])
def test_batched2d_hip_layers_match_vmap_and_issue_no_library_conv(name, ds, monkeypatch):
    """The grouped HIP path of the batched 2-D engine gives the vmapped library path's step (loss, gradients), and a
    step issues no aten convolution (the profiler's op list)."""
    from neuroimagedisttraining_amd.engine.batched2d import BatchedModuleEngine
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.engine.resnet2d_hip import CIFAR_MEAN, CIFAR_STD
    from neuroimagedisttraining_amd.models import create_model
    G, B = 4, 8
    torch.manual_seed(1)
    model = create_model(name, dataset=ds, class_num=10)
    c = 1 if ds == "mnist" else 3
    S = 28 if ds == "mnist" else 32
    x8 = torch.randint(0, 256, (G * B, S, S, c), dtype=torch.uint8)
    y = torch.randint(0, 10, (G * B,))
    mean, std = ((0.1307,), (0.3081,)) if c == 1 else (CIFAR_MEAN, CIFAR_STD)
    out = {}
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cuda()
    rows = flat.expand(G, -1) + torch.randn(G, flat.numel(), device="cuda") * 0.01  # one draw for both paths
    for hip in ("1", "0"):
        monkeypatch.setenv("NIDT_B2D_HIP", hip)
        eng = BatchedModuleEngine(create_model(name, dataset=ds, class_num=10), x8, y, "cuda", mean, std)
        assert eng.uses_hip_layers == (hip == "1")
        theta = padded_rows(G, eng.players.total, "cuda")
        theta.copy_(rows)
        grads = padded_rows(G, eng.players.total, "cuda")
        idx = torch.arange(G * B, dtype=torch.int32, device="cuda")
        if hip == "1":
            with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
                loss = eng.train_step(theta, None, grads, idx, G, B, 1.0, 7)
                logits = eng.eval_logits(theta, None, idx, G, B)
                torch.cuda.synchronize()
            ops_seen = {e.name for e in prof.events()}
            assert not [o for o in ops_seen if "conv" in o.lower() and o.startswith("aten::")], sorted(ops_seen)
        else:
            loss = eng.train_step(theta, None, grads, idx, G, B, 1.0, 7)
            logits = eng.eval_logits(theta, None, idx, G, B)
        out[hip] = (loss.float().cpu(), grads.float().cpu(), logits.float().cpu())
    assert torch.allclose(out["1"][0], out["0"][0], rtol=2e-2, atol=2e-2), (out["1"][0], out["0"][0])
    assert float((out["1"][2] - out["0"][2]).norm() / out["0"][2].norm()) < 3e-2
    for g in range(G):
        a, b = out["1"][1][g], out["0"][1][g]
        cos = float(torch.dot(a, b) / (a.norm() * b.norm()))
        assert cos > 0.99, (g, cos)
