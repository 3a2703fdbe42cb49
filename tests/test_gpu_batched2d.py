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
