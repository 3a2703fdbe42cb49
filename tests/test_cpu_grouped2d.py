"""The grouped-twin graph of the small 2-D models (engine/conv2d_hip.py): the model's own forward over a
group-stacked batch, with Conv2d / Linear / GroupNorm swapped for twins that read G clients' parameter rows, equals
G separate per-client forward / backward passes.  On the CPU the conv twin is a grouped library conv (the GPU runs
conv2d_any.hip; tests/test_gpu_batched2d.py checks that against fp32 PyTorch)."""
import pytest
import torch
import torch.nn.functional as F

from neuroimagedisttraining_amd.engine import conv2d_hip
from neuroimagedisttraining_amd.engine.flat import ParamLayout
from neuroimagedisttraining_amd.models import create_model

CASES = [("lenet5", "mnist", (1, 28, 28)), ("cnn_cifar10", "cifar10", (3, 32, 32)), ("vgg11", "cifar10", (3, 32, 32))]


@pytest.mark.parametrize("name,ds,shape", CASES)
def test_grouped_twins_match_per_client(name, ds, shape):
    torch.manual_seed(0)
    model = create_model(name, dataset=ds, class_num=10)
    assert conv2d_hip.supports(model)
    gm, grp = conv2d_hip.grouped_model(model)
    pl = ParamLayout.from_tensors(list(model.named_parameters()))
    G, B = 3, 2
    theta = torch.randn(G, pl.total) * 0.05
    x = torch.randn(G * B, *shape)
    y = torch.randint(0, 10, (G * B,))
    leaves = {n: theta[:, o:o + pl.numel(i)].clone().view((G,) + tuple(pl.shapes[i])).requires_grad_(True)
              for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
    grp.G, grp.params = G, leaves
    gm.eval()
    out = gm(x)
    loss = F.cross_entropy(out, y, reduction="none").view(G, B).mean(1)
    gs = torch.autograd.grad(loss.sum(), list(leaves.values()))
    model.eval()
    for g in range(G):
        with torch.no_grad():
            for i, (n, p) in enumerate(model.named_parameters()):
                p.copy_(leaves[n][g])
        model.zero_grad()
        o = model(x[g * B:(g + 1) * B])
        torch.testing.assert_close(out[g * B:(g + 1) * B], o, rtol=1e-4, atol=1e-5)
        F.cross_entropy(o, y[g * B:(g + 1) * B]).backward()
        for gi, (n, p) in zip(gs, model.named_parameters()):
            torch.testing.assert_close(gi[g], p.grad, rtol=1e-4, atol=1e-6)


def test_unsupported_layers_keep_the_vmap_path():
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, stride=2), torch.nn.Flatten())
    assert not conv2d_hip.supports(m)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8))
    assert not conv2d_hip.supports(m)
