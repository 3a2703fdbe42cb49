"""CPU tests of the client-batched engine for the non-ResNet image models (engine/batched2d.py): device draws of
the augmentation hash equal the ResNet engine's host twin, the vectorised crop/flip equals the per-sample one, a
vmapped lockstep step equals per-client autograd through the reference-shaped model, and the runners step on it
(the CLI routes ``lenet5 / cnn_cifar10 / cnn_cifar100 / vgg11`` on CIFAR to it)."""
import argparse

import numpy as np
import pytest
import torch
from torch.func import functional_call

from neuroimagedisttraining_amd.engine.batched2d import BatchedModuleEngine, aug_draws_t, augment_batch, mix64_t
from neuroimagedisttraining_amd.engine.executor import ClientSplit, FLConfig, padded_rows
from neuroimagedisttraining_amd.engine.resnet2d_hip import (CIFAR_MEAN, CIFAR_STD, aug_draws, augment_u8, mix64,
                                                            synthetic_cifar)
from neuroimagedisttraining_amd.models import create_model


def test_device_augmentation_hash_equals_host_twin():
    for seed in (0, 5, (7 << 40) + 123, (1 << 63) + 99, (1 << 64) - 1):
        cids = [0, 3, 99, 4096]
        want = aug_draws(seed, cids, 6)
        st = torch.tensor(seed - (1 << 64) if seed >= (1 << 63) else seed, dtype=torch.int64)
        got = aug_draws_t(st, torch.tensor(cids, dtype=torch.int64), 6)
        for a, b in zip(want, got):
            assert np.array_equal(a, b.numpy()), seed
        z = mix64_t(st.view(1), torch.tensor([3]), torch.tensor([2]))
        assert int(z) & ((1 << 64) - 1) == mix64(seed, 3, 2)


def test_vectorised_crop_flip_equals_per_sample():
    x8, _ = synthetic_cifar(7, seed=2)
    g = torch.Generator().manual_seed(1)
    oy, ox = torch.randint(0, 9, (7,), generator=g), torch.randint(0, 9, (7,), generator=g)
    fl = torch.randint(0, 2, (7,), generator=g)
    assert torch.equal(augment_batch(x8, oy, ox, fl), augment_u8(x8, oy, ox, fl))


def _theta(model_fn, G, L, seed=0):
    theta = padded_rows(G, L.total, "cpu")
    for g in range(G):
        torch.manual_seed(seed + g)
        theta[g].copy_(torch.cat([p.detach().reshape(-1) for p in model_fn().parameters()]))
    return theta


@pytest.mark.parametrize("name", ["cnn_cifar10", "lenet5", "vgg11"])
def test_vmapped_step_matches_per_client_autograd(name):
    G, B = 3, 4
    mk = lambda: create_model(name, dataset="cifar10", class_num=10)  # noqa: E731
    x8, y = synthetic_cifar(G * B, seed=1)
    eng = BatchedModuleEngine(mk(), x8, y, "cpu", CIFAR_MEAN, CIFAR_STD, augment=True)
    L = eng.players
    theta = _theta(mk, G, L)
    grads = padded_rows(G, L.total, "cpu")
    seed_dev = torch.tensor([17], dtype=torch.int64)
    losses = eng.train_step(theta, None, grads, torch.arange(G * B, dtype=torch.int32), G, B, 1.0, 1 << 40,
                            cids=[5, 2, 9], seed_dev=seed_dev)
    oy, ox, fl = aug_draws((1 << 40) + 17, [5, 2, 9], B)
    img = augment_u8(x8, oy, ox, fl)
    m64 = mk().double()
    for g in range(G):
        row = theta[g].double().clone().requires_grad_(True)
        pv = {n: row[o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        xb = (img[g * B:(g + 1) * B].double() / 255.0 - torch.tensor(CIFAR_MEAN, dtype=torch.float64)) / \
            torch.tensor(CIFAR_STD, dtype=torch.float64)
        loss = torch.nn.functional.cross_entropy(functional_call(m64, pv, (xb.permute(0, 3, 1, 2),)),
                                                 y[g * B:(g + 1) * B])
        loss.backward()
        assert abs(float(loss.detach()) - float(losses[g])) < 1e-4, (name, g)
        rel = float((grads[g].double() - row.grad).norm() / row.grad.norm())
        assert rel < 5e-3, (name, g, rel)  # fp32 vs fp64 (random-init GN VGG amplifies rounding ~2e-3)
    # evaluation: the same logits as the per-client model
    logits = eng.eval_logits(theta, None, torch.arange(G * B, dtype=torch.int32), G, B)
    for g in range(G):
        pv = {n: theta[g, o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        xb = (x8[g * B:(g + 1) * B].float() / 255.0 - torch.tensor(CIFAR_MEAN)) / torch.tensor(CIFAR_STD)
        ref = functional_call(mk().eval(), pv, (xb.permute(0, 3, 1, 2),))
        assert torch.allclose(logits[g * B:(g + 1) * B], ref, atol=1e-4), (name, g)


@pytest.mark.parametrize("alg", ["subavg", "fedavg", "ditto"])
def test_runners_step_on_the_batched_engine(alg):
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.parallel import runtime as rt
    N, per = 4, 10
    x8, y = synthetic_cifar(N * per, seed=3)
    splits = [ClientSplit(np.arange(c * per, c * per + 7 - (c % 2)), np.arange(c * per + 7, (c + 1) * per))
              for c in range(N)]
    model = create_model("cnn_cifar10", dataset="cifar10", class_num=10)
    eng = BatchedModuleEngine(model, x8, y, "cpu", CIFAR_MEAN, CIFAR_STD)
    cfg = FLConfig(comm_round=2, epochs=1, batch_size=4, lr=0.05, dense_ratio=0.5, seed=1, frac=1.0)
    r = make_runner(alg, eng, splits, cfg, rt.DistInfo(0, 1, 0, torch.device("cpu"), "none"), model)
    before = r.theta.clone()
    for k in range(2):
        res = r.run_round(k)
    r.finish()
    assert torch.isfinite(r.theta).all() and not torch.equal(before, r.theta)
    vals = [float(v) for v in res.values() if isinstance(v, (float, int))]
    assert vals and all(np.isfinite(v) for v in vals)


def test_cli_routes_the_zoo_models_to_the_batched_engine():
    from neuroimagedisttraining_amd.cli import hip_family
    for m in ("lenet5", "cnn_cifar10", "cnn_cifar100", "vgg11"):
        assert hip_family(argparse.Namespace(model=m, dataset="cifar10")) == "batched2d"
    assert hip_family(argparse.Namespace(model="resnet18", dataset="cifar10")) == "resnet2d"
    assert hip_family(argparse.Namespace(model="lenet5", dataset="mnist")) is None
