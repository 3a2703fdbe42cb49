"""CPU tests of the client-batched ResNet-18-GN engine (engine/resnet2d_hip.py): the explicit lockstep
forward/backward (fp32 CPU twin of the HIP path) against per-client autograd through the reference-shaped
``customized_resnet18`` (``fedml_api/model/cv/resnet.py:91-124``), GroupNorm formulas, and every algorithm runner
stepping on it."""
import numpy as np
import pytest
import torch
from torch.func import functional_call

from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, padded_rows
from neuroimagedisttraining_amd.engine.resnet2d_hip import (CIFAR_MEAN, CIFAR_STD, GroupNormG, ResNetHipEngine,
                                                            synthetic_cifar)
from neuroimagedisttraining_amd.models import customized_resnet18


def test_groupnorm_fwd_bwd_formulas():
    torch.manual_seed(0)
    G, B, H, W, C = 2, 3, 4, 4, 64
    theta = torch.randn(G, 2 * C)
    grads = torch.zeros_like(theta)
    gn = GroupNormG(0, C, C, hip=False)
    t = torch.randn(G * B, H, W, C)
    dy = torch.randn(G * B, H, W, C)
    y, saved = gn.fwd(t, theta, G)
    dt = gn.bwd(dy, None, t, saved, theta, grads, G)
    tt = t.clone().requires_grad_(True)
    th = theta.clone().requires_grad_(True)
    ref = torch.cat([torch.nn.functional.group_norm(tt[g * B:(g + 1) * B].permute(0, 3, 1, 2), 32, th[g, :C],
                                                    th[g, C:], 1e-5).permute(0, 2, 3, 1) for g in range(G)])
    assert torch.allclose(ref, y, atol=1e-5)
    ref.backward(dy)
    assert torch.allclose(tt.grad, dt, atol=1e-5)
    assert torch.allclose(th.grad, grads, atol=1e-4)


def test_resnet18gn_lockstep_step_matches_per_client_autograd():
    torch.manual_seed(0)
    G, B = 2, 4
    m = customized_resnet18(class_num=10)
    x8, y = synthetic_cifar(G * B, seed=1)
    eng = ResNetHipEngine(m, x8, y, "cpu")
    L = eng.players
    theta = padded_rows(G, L.total, "cpu")
    for g in range(G):
        theta[g].copy_(torch.cat([p.detach().reshape(-1) for p in customized_resnet18(class_num=10).parameters()]))
    grads = padded_rows(G, L.total, "cpu")
    losses = eng.train_step(theta, None, grads, torch.arange(G * B, dtype=torch.int32), G, B, 1.0, 0)
    m64 = customized_resnet18(class_num=10).double()
    for g in range(G):
        row = theta[g].double().clone().requires_grad_(True)
        pv = {n: row[o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        xb = (x8[g * B:(g + 1) * B].double() / 255.0 - torch.tensor(CIFAR_MEAN, dtype=torch.float64)) / \
            torch.tensor(CIFAR_STD, dtype=torch.float64)
        loss = torch.nn.functional.cross_entropy(functional_call(m64, pv, (xb.permute(0, 3, 1, 2),)),
                                                 y[g * B:(g + 1) * B])
        loss.backward()
        assert abs(float(loss) - float(losses[g])) < 1e-4
        rel = float((grads[g].double() - row.grad).norm() / row.grad.norm())
        assert rel < 5e-3, (g, rel)  # fp32 vs fp64 (random-init GN nets amplify rounding ~1e-3)


@pytest.mark.parametrize("alg", ["subavg", "dispfl", "fedavg", "local"])
def test_resnet18gn_runners_step(alg):
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    C, ntr, nte = 4, 5, 3
    x8, y = synthetic_cifar(C * (ntr + nte), seed=2)
    splits = [ClientSplit(train=np.arange(c * (ntr + nte), c * (ntr + nte) + ntr),
                          test=np.arange(c * (ntr + nte) + ntr, (c + 1) * (ntr + nte))) for c in range(C)]
    info = rt.init_distributed(prefer_gpu=False)
    m = customized_resnet18(class_num=10)
    eng = ResNetHipEngine(m, x8, y, "cpu")
    cfg = FLConfig(comm_round=1, epochs=1, batch_size=4, dense_ratio=0.3, seed=0, frac=0.5,
                   frequency_of_the_test=1, final_round=False)
    r = make_runner(alg, eng, splits, cfg, info, m)
    before = r.theta.clone()
    res = r.run_round(0)
    assert torch.isfinite(r.theta).all()
    assert not torch.equal(before, r.theta)
    vals = [float(v) for v in res.values() if isinstance(v, (float, int))]
    assert vals and all(np.isfinite(v) for v in vals)
