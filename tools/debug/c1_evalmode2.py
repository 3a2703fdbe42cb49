"""Debug: dump the eval-mode train step's activations / gradients (argv[1] = output .pt) for a cross-layout diff."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_gpu_kernels import _alexnet_setup  # noqa: E402
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
net.train_step(theta, bufs, grads, x8, mom, idx, store.labels.float(), G, B, keep=0.5, seed=3, bn_train=False)
torch.cuda.synchronize()
b = net._cache[(G, B, True)]
out = {k: v.detach().cpu().clone() for k, v in b.items() if torch.is_tensor(v)}
out["__grads"] = grads.detach().cpu().clone()
out["__names"] = [(n, o, pl.numel(i)) for i, (n, o) in enumerate(zip(pl.names, pl.offsets))]
torch.save(out, sys.argv[1])
print("saved", len(out))
