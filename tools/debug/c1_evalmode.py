"""Debug: conv1 fused forward p1 of the eval-mode train step (bn_train=False) against fp64 for each client, at the
slot layout chosen by NIDT_C1_TAPORD."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_gpu_kernels import _alexnet_setup, _cf  # noqa: E402
from neuroimagedisttraining_amd.engine.alexnet_hip import HipAlexNet3D  # noqa: E402
from neuroimagedisttraining_amd.engine.executor import padded_rows  # noqa: E402

DEV = "cuda"
G, B = 2, 3
store, x8, mom, pl, bl, theta, bufs = _alexnet_setup(G, B, seed=3)
for i, n in enumerate(bl.names):
    o, k = bl.offsets[i], bl.numel(i)
    if n.endswith("running_mean"):
        bufs[:, o:o + k] = 0.1 * torch.randn(G, k, device=DEV)
    if n.endswith("running_var"):
        bufs[:, o:o + k] = 0.5 + torch.rand(G, k, device=DEV)
for i, n in enumerate(pl.names):
    if n in ("features.1.weight", "features.9.weight"):
        o = pl.offsets[i]
        theta[:, o:o + 8] *= -1
net = HipAlexNet3D(pl, bl, DEV)
grads = padded_rows(G, pl.total, DEV)
idx = torch.arange(G * B, dtype=torch.int32, device=DEV)
for mode in ("eval", "train"):
    net.train_step(theta, bufs.clone(), grads, x8, mom, idx, store.labels.float(), G, B, keep=1.0, seed=3,
                   bn_train=mode == "train")
    torch.cuda.synchronize()
    b = net._cache[(G, B, True)]
    for g in range(G):
        sl = slice(g * B, (g + 1) * B)
        pv = {n: theta[g, o:o + pl.numel(i)].double().view(pl.shapes[i]) for i, (n, o) in enumerate(zip(pl.names, pl.offsets))}
        bv = {n: bufs[g, o:o + bl.numel(i)].double().view(bl.shapes[i]) for i, (n, o) in enumerate(zip(bl.names, bl.offsets))}
        h = (store.volumes[sl].double() / 255.0).unsqueeze(1)
        y = F.conv3d(h, pv["features.0.weight"], pv["features.0.bias"], 2, 0)
        if mode == "eval":
            z = F.batch_norm(y, bv["features.1.running_mean"], bv["features.1.running_var"], pv["features.1.weight"],
                             pv["features.1.bias"], False, 0.1, 1e-5)
        else:
            z = F.batch_norm(y, None, None, pv["features.1.weight"], pv["features.1.bias"], True, 0.1, 1e-5)
        ref = F.max_pool3d(torch.relu(z), 3, 3)
        ours = _cf(b["p1"][sl].double())
        e = float((ours - ref).norm() / ref.norm())
        print(mode, "client", g, "p1 relerr %.3e" % e, "s1", b["s1"][g, :4].tolist(), "t1", b["t1"][g, :4].tolist(),
              flush=True)
