"""CPU test of the client-batched 3D ResNet engine's wiring (engine/resnet3d_hip.py, fp32 torch twin of the HIP
path): one lockstep step of two clients through the full Bottleneck ResNet-50 equals per-client autograd through
``models.resnet3d.resnet3d_50`` (loss, gradients, BatchNorm running statistics)."""
import torch
import torch.nn.functional as F
from torch.func import functional_call

from neuroimagedisttraining_amd.engine.executor import padded_rows
from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
from neuroimagedisttraining_amd.models.resnet3d import resnet3d_50


def test_resnet3d50_lockstep_matches_per_client_autograd_fp32():
    torch.manual_seed(0)
    G, B = 2, 2
    vol = torch.randint(0, 256, (G * B, 40, 48, 40), dtype=torch.uint8)
    lab = torch.tensor([0.0, 1.0, 1.0, 0.0])
    m = resnet3d_50(num_classes=1)
    eng = ResNet3DHipEngine(m, vol, lab, "cpu")
    L, Lb = eng.players, eng.blayers
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    bflat = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()])
    th, gr = padded_rows(G, L.total, "cpu"), padded_rows(G, L.total, "cpu")
    bu = padded_rows(G, Lb.total, "cpu")
    th.copy_(flat.expand(G, -1))
    bu.copy_(bflat.expand(G, -1))
    losses = eng.train_step(th, bu, gr, torch.arange(G * B, dtype=torch.int32), G, B, 1.0, 0)
    mref = resnet3d_50(num_classes=1)
    mref.train()
    for g in range(G):
        row = flat.clone().requires_grad_(True)
        pv = {n: row[o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
        bv = {n: bflat[o:o + Lb.numel(i)].view(Lb.shapes[i]).clone().to(Lb.dtypes[i])
              for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets))}
        x = vol[g * B:(g + 1) * B].float().unsqueeze(1) / 255.0
        loss = F.binary_cross_entropy_with_logits(functional_call(mref, {**pv, **bv}, (x,)).view(-1),
                                                  lab[g * B:(g + 1) * B])
        loss.backward()
        assert abs(float(loss) - float(losses[g])) < 1e-4
        rel = float((gr[g] - row.grad).norm() / row.grad.norm())
        assert rel < 5e-2, rel  # fp32; BN over 16 voxels per channel in layer4 amplifies rounding to ~1e-2
        for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets)):
            assert torch.allclose(bu[g, o:o + Lb.numel(i)], bv[n].float(), atol=1e-4, rtol=1e-3), n
