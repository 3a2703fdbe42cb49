"""DARTS / GDAS search space, genotype derivation and the second-order architect (CPU)."""
import argparse

import pytest
import torch
import torch.nn as nn

from neuroimagedisttraining_amd.nas import (GENOTYPES, PRIMITIVES, Architect, ModelForModelSizeMeasure,
                                            Network, Network_GumbelSoftmax, NetworkCIFAR, NetworkImageNet,
                                            derive_genotype, genotype_from_string)
from neuroimagedisttraining_amd.nas.search import n_edges


def _args(**kw):
    d = dict(momentum=0.9, weight_decay=3e-4, arch_learning_rate=3e-4, arch_weight_decay=1e-3)
    d.update(kw)
    return argparse.Namespace(**d)


def test_genotype_string_roundtrip():
    for name, g in GENOTYPES.items():
        assert genotype_from_string(str(g)) == g
        assert genotype_from_string(name) == g
    assert len(GENOTYPES["DARTS_V2"].normal) == 8 and GENOTYPES["DARTS"] is GENOTYPES["DARTS_V2"]


def test_derive_genotype_picks_top2_non_none():
    k = n_edges(4)
    an = torch.full((k, len(PRIMITIVES)), -5.0)
    # node 0 (edges 0,1): edge 1 prefers sep_conv_3x3 strongly, edge 0 'none' (ignored) then max_pool
    an[0, PRIMITIVES.index("none")] = 9.0
    an[0, PRIMITIVES.index("max_pool_3x3")] = 1.0
    an[1, PRIMITIVES.index("sep_conv_3x3")] = 3.0
    g, n_conv_normal, _ = derive_genotype(an, an.clone())
    assert g.normal[0] == ("sep_conv_3x3", 1)
    assert g.normal[1] == ("max_pool_3x3", 0)
    assert g.normal_concat == [2, 3, 4, 5]
    assert n_conv_normal >= 1


@pytest.mark.parametrize("cls", [Network, Network_GumbelSoftmax])
def test_search_network_forward_backward(cls):
    torch.manual_seed(0)
    net = cls(4, 10, 3, nn.CrossEntropyLoss())
    x, y = torch.randn(4, 3, 16, 16), torch.randint(0, 10, (4,))
    loss = net.loss(x, y)
    loss.backward()
    assert net.alphas_normal.grad is not None and net.alphas_normal.grad.abs().sum() > 0
    assert len(net.arch_parameters()) == 2
    assert len(net.weight_parameters()) + 2 == len(list(net.parameters()))
    assert net.get_current_model_size() > 0
    g = net.genotype()[0]
    ev = NetworkCIFAR(4, 10, 3, True, g)
    ev.train()
    out, aux = ev(torch.randn(2, 3, 32, 32))
    assert out.shape == (2, 10) and aux.shape == (2, 10)


def test_imagenet_network_shapes():
    net = NetworkImageNet(8, 5, 3, True, GENOTYPES["DARTS"])
    net.eval()
    out, aux = net(torch.randn(1, 3, 224, 224))
    assert out.shape == (1, 5) and aux is None


def test_size_model_matches_argmax_genotype_params():
    torch.manual_seed(1)
    net = Network(4, 10, 3, nn.CrossEntropyLoss())
    m = ModelForModelSizeMeasure(4, 10, 3, None, net.alphas_normal, net.alphas_reduce)
    assert m(torch.randn(2, 3, 16, 16)).shape == (2, 10)


def _tiny_net():
    torch.manual_seed(0)
    net = Network(2, 3, 3, nn.CrossEntropyLoss(), steps=2, multiplier=2).double()
    net.eval()  # BN in eval mode -> loss is a smooth deterministic function of (w, alpha)
    return net


def test_hessian_vector_product_matches_exact():
    net = _tiny_net()
    arch = Architect(net, nn.CrossEntropyLoss(), _args())
    x, y = torch.randn(4, 3, 8, 8, dtype=torch.float64), torch.randint(0, 3, (4,))
    ws = net.weight_parameters()
    v = [torch.randn_like(w) for w in ws]
    approx = arch._hessian_vector_product(v, x, y, r=1e-4)
    # exact: d/d alpha of <grad_w L, v>
    loss = net.loss(x, y)
    gw = torch.autograd.grad(loss, ws, create_graph=True)
    dot = sum((g * vv).sum() for g, vv in zip(gw, v))
    exact = torch.autograd.grad(dot, net.arch_parameters(), allow_unused=True)
    R = 1e-4 / torch.cat([t.reshape(-1) for t in v]).norm()
    for a, e in zip(approx, exact):
        e = torch.zeros_like(a) if e is None else e
        # finite difference approximates grad_a <grad_w L, v> scaled by ||v||-normalised step
        assert torch.allclose(a, e, rtol=1e-3, atol=1e-6 / float(R)), (a - e).abs().max()


def test_unrolled_step_updates_alphas_and_keeps_weights():
    net = _tiny_net()
    arch = Architect(net, nn.CrossEntropyLoss(), _args())
    opt = torch.optim.SGD(net.weight_parameters(), 0.1, momentum=0.9)
    x, y = torch.randn(4, 3, 8, 8, dtype=torch.float64), torch.randint(0, 3, (4,))
    w0 = [w.detach().clone() for w in net.weight_parameters()]
    a0 = [a.detach().clone() for a in net.arch_parameters()]
    arch.step(x, y, x, y, 0.1, opt, unrolled=True)
    for w, w_ in zip(net.weight_parameters(), w0):
        assert torch.allclose(w, w_, atol=1e-12)  # finite-difference perturbations restored
    assert any(not torch.equal(a, b) for a, b in zip(net.arch_parameters(), a0))
    for m in ("step_v2", "step_single_level", "step_AOS"):
        if m == "step_v2":
            arch.step_v2(x, y, x, y, 1.0, 1.0)
        elif m == "step_single_level":
            arch.step_single_level(x, y)
        else:
            arch.step_AOS(x, y, x, y)
    arch.step_v2_2ndorder(x, y, x, y, 0.1, opt, 1.0, 1.0)
    arch.step_v2_2ndorder2(x, y, x, y, 0.1, opt, 1.0, 1.0)


def test_unrolled_alpha_grad_matches_exact_first_order_limit():
    """With eta=0 the unrolled gradient equals the plain validation alpha gradient."""
    net = _tiny_net()
    arch = Architect(net, nn.CrossEntropyLoss(), _args(momentum=0.0, weight_decay=0.0))
    x, y = torch.randn(4, 3, 8, 8, dtype=torch.float64), torch.randint(0, 3, (4,))
    params = arch._unrolled_params(x, y, 0.0, None)
    g = arch._second_order_alpha(params, x, y, x, y, 0.0)
    ref = torch.autograd.grad(net.loss(x, y), net.arch_parameters())
    for a, b in zip(g, ref):
        assert torch.allclose(a, b, atol=1e-10)
