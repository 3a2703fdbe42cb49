"""Debug: divergence of HIP vs torch engine over consecutive local steps of one client (per-layer)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
from test_gpu_personalized import _fed, _relerr
from neuroimagedisttraining_amd.engine.executor import HipEngine, TorchEngine, padded_rows
from neuroimagedisttraining_amd.engine.runner import StepSpec
from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
DEV = "cuda"
fed = _fed([48, 48])
st, x8, mom, splits = fed
torch.manual_seed(0)
model = AlexNet3D_Dropout(num_classes=1)
he = HipEngine(model, x8, mom, st.labels.float(), DEV)
te = TorchEngine(model, st.volumes, st.labels.float(), DEV)
pl = he.players
P, Q = pl.total, he.blayers.total
flat = pl.flatten_state(dict(model.named_parameters()), DEV)
fb = he.blayers.flatten_state(dict(model.named_buffers()), DEV)
G, B = 1, 8
tha = padded_rows(G, P, DEV); tha.copy_(flat.expand(G, P)); thb = padded_rows(G, P, DEV); thb.copy_(tha)
bua = padded_rows(G, Q, DEV); bua.copy_(fb.expand(G, Q)); bub = padded_rows(G, Q, DEV); bub.copy_(bua)
ga = padded_rows(G, P, DEV); gb = padded_rows(G, P, DEV)
w0 = tha.clone()
for step in range(6):
    idx = torch.arange(step * B, (step + 1) * B, dtype=torch.int32, device=DEV)
    la = he.train_step(tha, bua, ga, idx, G, B, 1.0, 0, cids=[0])
    lb = te.train_step(thb, bub, gb, idx, G, B, 1.0, 0, cids=[0])
    # cross-check: HIP gradient at the torch weights
    gx = padded_rows(G, P, DEV); bux = bub.clone()
    he.train_step(thb, bux, gx, idx, G, B, 1.0, 0, cids=[0])
    torch.cuda.synchronize()
    per = {}
    for i, n in enumerate(pl.names):
        o, k = pl.offsets[i], pl.numel(i)
        per[n] = round(_relerr(gx[0, o:o + k], gb[0, o:o + k]), 3)
    print("step", step, "loss", float(la), float(lb), "grad(a) vs grad(b) %.3f" % _relerr(ga, gb),
          "hip grad at torch weights vs torch grad %.3f" % _relerr(gx, gb), "gnorm", float(ga.norm()), float(gb.norm()), flush=True)
    print("   per-layer", per, flush=True)
    spec = StepSpec()
    he.local_opt(tha, ga, None, spec, 0.01, 5e-4, 0.0, 10.0)
    te.local_opt(thb, gb, None, spec, 0.01, 5e-4, 0.0, 10.0)
    print("   update relerr %.4f" % _relerr(tha - w0, thb - w0), flush=True)
