"""Debug: HIP vs torch engine per (G, B) train step gradients and per-client runner updates."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from test_gpu_personalized import _fed, _run, _relerr
from neuroimagedisttraining_amd.engine.executor import HipEngine, TorchEngine, padded_rows
from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
DEV = "cuda"
sizes = [20, 12, 20, 9, 16, 11, 20, 13]
fed = _fed(sizes)
st, x8, mom, splits = fed
torch.manual_seed(0)
model = AlexNet3D_Dropout(num_classes=1)
he = HipEngine(model, x8, mom, st.labels.float(), DEV)
te = TorchEngine(model, st.volumes, st.labels.float(), DEV)
P, Q = he.players.total, he.blayers.total
flat = he.players.flatten_state(dict(model.named_parameters()), DEV)
fb = he.blayers.flatten_state(dict(model.named_buffers()), DEV)
for G, B in [(1, 1), (1, 3), (1, 4), (1, 5), (1, 8), (2, 8), (3, 8), (8, 8)]:
    th = padded_rows(G, P, DEV); th.copy_(flat.expand(G, P))
    bu = padded_rows(G, Q, DEV); bu.copy_(fb.expand(G, Q))
    gh = padded_rows(G, P, DEV); gt = padded_rows(G, P, DEV)
    idx = torch.arange(G * B, dtype=torch.int32, device=DEV)
    bu2 = bu.clone()
    lh = he.train_step(th, bu, gh, idx, G, B, 1.0, 0, cids=list(range(G)))
    lt = te.train_step(th, bu2, gt, idx, G, B, 1.0, 0, cids=list(range(G)))
    torch.cuda.synchronize()
    print("G=%d B=%d grad relerr %.4f loss %s vs %s bufs relerr %.4f" % (G, B, _relerr(gh, gt), lh.tolist(), lt.tolist(), _relerr(bu, bu2)), flush=True)
for algo in ["fedavg", "local"]:
    a, w0 = _run(algo, "hip", fed, rounds=1, epochs=1)
    b, _ = _run(algo, "torch", fed, rounds=1, epochs=1)
    for i, c in enumerate(a.local):
        print(algo, "client", c, "size", sizes[c], "upd relerr %.4f" % _relerr(a.theta[i, :P] - w0[i, :P], b.theta[i, :P] - w0[i, :P]), "norm", float((b.theta[i, :P] - w0[i, :P]).norm()), flush=True)
