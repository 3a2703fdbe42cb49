"""CPU tests of the train-time image augmentation (reference ``cifar10/data_loader.py:46-52``,
``tiny_imagenet/data_loader.py:51-57``: RandomCrop(S, padding=4) + RandomHorizontalFlip): the on-device draw rule
(crop offsets uniform in [0, 8], flip p = 1/2, keyed by (step seed, client, position)), the crop/flip semantics with
zero padding against a direct torchvision-style implementation, the eager loaders, and the Tiny-ImageNet ResNet-18
(64x64, adaptive pooling, 200 classes) on the engine's CPU twin against per-client autograd."""
import numpy as np
import pytest
import torch
from torch.func import functional_call

from neuroimagedisttraining_amd.engine import resnet2d_hip as R


def test_aug_draws_are_uniform_and_keyed():
    oy, ox, fl = [], [], []
    for step in range(40):
        a, b, c = R.aug_draws(1234 + step, list(range(16)), 16)
        oy.append(a), ox.append(b), fl.append(c)
    oy, ox, fl = np.concatenate(oy), np.concatenate(ox), np.concatenate(fl)
    n = len(oy)
    for v in (oy, ox):
        assert v.min() == 0 and v.max() == 8
        cnt = np.bincount(v, minlength=9)
        chi2 = float(((cnt - n / 9) ** 2 / (n / 9)).sum())
        assert chi2 < 30.0, cnt  # 8 dof: p ~ 2e-4
    assert abs(fl.mean() - 0.5) < 0.03
    # offsets independent of each other (joint 9x9 table roughly flat)
    joint = np.bincount(oy * 9 + ox, minlength=81)
    assert joint.min() > 0.5 * n / 81
    # keyed draws: same (seed, client, position) -> same draw, independent of the client group it trains in
    a = R.aug_draws(77, [3, 5, 9], 4)
    b = R.aug_draws(77, [5], 4)
    for k in range(3):
        assert np.array_equal(a[k][4:8], b[k])
    c = R.aug_draws(78, [3, 5, 9], 4)
    assert any(not np.array_equal(a[k], c[k]) for k in range(3))


def _torchvision_crop_flip(img, top, left, flip, pad=4):
    """RandomCrop(size, padding=pad) with fill 0 then RandomHorizontalFlip, written directly (HWC uint8)."""
    H, W, C = img.shape
    canvas = np.zeros((H + 2 * pad, W + 2 * pad, C), dtype=img.dtype)
    canvas[pad:pad + H, pad:pad + W] = img
    out = canvas[top:top + H, left:left + W]
    return out[:, ::-1] if flip else out


def test_augment_u8_matches_crop_flip_semantics():
    g = np.random.default_rng(0)
    img = g.integers(1, 256, size=(6, 32, 32, 3)).astype(np.uint8)
    oy = np.array([0, 8, 4, 2, 8, 0])
    ox = np.array([0, 8, 4, 7, 0, 8])
    fl = np.array([0, 1, 1, 0, 0, 1])
    out = R.augment_u8(torch.from_numpy(img), oy, ox, fl).numpy()
    for n in range(6):
        assert np.array_equal(out[n], _torchvision_crop_flip(img[n], oy[n], ox[n], fl[n]))
    # zero padding: offset (0, 0) shifts the image down-right by 4 and the uncovered band is 0
    assert (out[0, :4] == 0).all() and (out[0, :, :4] == 0).all() and np.array_equal(out[0, 4:, 4:], img[0, :28, :28])


def test_eager_loader_augments_train_only_with_black_padding():
    from neuroimagedisttraining_amd.data.images import NORM, AugmentedTensorDataset, load_partition_data
    mean, std = NORM["cifar10"]
    x = torch.randn(4, 3, 32, 32)
    y = torch.arange(4)
    ds = AugmentedTensorDataset(x, y, mean, std)
    fill = (-torch.tensor(mean) / torch.tensor(std)).view(3, 1, 1)
    torch.manual_seed(5)
    seen_flip, tops = 0, []
    for _ in range(400):
        out, lab = ds[1]
        assert out.shape == (3, 32, 32) and int(lab) == 1
        # recover the draw: the output is a shifted (maybe flipped) copy of x[1] inside a black border
        for f in (0, 1):
            o = out.flip(-1) if f else out
            for t in range(9):
                for l_ in range(9):
                    ref = torch.zeros(3, 40, 40) + fill
                    ref[:, 4:36, 4:36] = x[1]
                    if torch.equal(o, ref[:, t:t + 32, l_:l_ + 32]):
                        tops.append(t)
                        seen_flip += f
                        break
                else:
                    continue
                break
            else:
                continue
            break
    assert len(tops) == 400
    assert abs(seen_flip / 400 - 0.5) < 0.1 and set(tops) == set(range(9))
    ds8 = load_partition_data("cifar10", None, "homo", 0.5, 2, 8, n_train=40, n_test=20, seed=1)
    train, test = ds8[5][0], ds8[6][0]
    assert isinstance(train.dataset, AugmentedTensorDataset)
    assert not isinstance(test.dataset, AugmentedTensorDataset)
    plain = load_partition_data("cifar10", None, "homo", 0.5, 2, 8, n_train=40, n_test=20, seed=1, augment=False)
    assert not isinstance(plain[5][0].dataset, AugmentedTensorDataset)


def test_engine_cpu_twin_applies_the_keyed_augmentation():
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.models import customized_resnet18
    torch.manual_seed(0)
    G, B = 2, 3
    x8, y = R.synthetic_cifar(G * B, seed=4)
    m = customized_resnet18(class_num=10)
    eng = R.ResNetHipEngine(m, x8, y, "cpu")
    idx = torch.arange(G * B, dtype=torch.int32)
    seed_dev = torch.tensor([17], dtype=torch.int64)
    cids = [4, 9]
    x_aug = eng.net.input(eng.x8, idx, (seed_dev, 1 << 40, None, cids, B))
    oy, ox, fl = R.aug_draws((1 << 40) + 17, cids, B)
    want = R.augment_u8(x8, oy, ox, fl)
    x_ref = eng.net.input(want, idx)
    assert torch.equal(x_aug, x_ref)
    assert not torch.equal(x_aug, eng.net.input(eng.x8, idx))
    th = padded_rows(G, eng.players.total, "cpu")
    th.copy_(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).expand(G, -1))
    gr = padded_rows(G, eng.players.total, "cpu")
    loss = eng.train_step(th, None, gr, idx, G, B, 1.0, 1 << 40, cids=cids, seed_dev=seed_dev)
    assert torch.isfinite(loss).all() and float(gr.abs().sum()) > 0


@pytest.mark.slow
def test_tiny_resnet18_twin_matches_per_client_autograd():
    """64x64 inputs, 200 classes, AdaptiveAvgPool2d over the final 8x8 map, Tiny normalisation (0.5, 0.5)."""
    from neuroimagedisttraining_amd.engine.executor import padded_rows
    from neuroimagedisttraining_amd.models import tiny_resnet18
    torch.manual_seed(0)
    G, B = 2, 2
    g = np.random.default_rng(3)
    x8 = torch.from_numpy(g.integers(0, 256, size=(G * B, 64, 64, 3)).astype(np.uint8))
    y = torch.from_numpy(g.integers(0, 200, size=G * B))
    m = tiny_resnet18(class_num=200)
    eng = R.ResNetHipEngine(m, x8, y, "cpu")
    assert eng.net.mean == R.TINY_MEAN and eng.net.ncls == 200
    L = eng.players
    theta = padded_rows(G, L.total, "cpu")
    for gi in range(G):
        theta[gi].copy_(torch.cat([p.detach().reshape(-1) for p in tiny_resnet18(class_num=200).parameters()]))
    grads = padded_rows(G, L.total, "cpu")
    losses = eng.train_step(theta, None, grads, torch.arange(G * B, dtype=torch.int32), G, B, 1.0, 0)
    m64 = tiny_resnet18(class_num=200).double()
    for gi in range(G):
        row = theta[gi].double().clone().requires_grad_(True)
        pv = {n: row[o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        xb = (x8[gi * B:(gi + 1) * B].double() / 255.0 - 0.5) / 0.5
        loss = torch.nn.functional.cross_entropy(functional_call(m64, pv, (xb.permute(0, 3, 1, 2),)),
                                                 y[gi * B:(gi + 1) * B])
        loss.backward()
        assert abs(float(loss) - float(losses[gi])) < 1e-4
        rel = float((grads[gi].double() - row.grad).norm() / row.grad.norm())
        assert rel < 5e-3, (gi, rel)
