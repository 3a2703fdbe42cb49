"""Debug: block-by-block forward activations of the client-batched ResNet3D vs the reference module (client 0)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from torch.func import functional_call
from neuroimagedisttraining_amd.engine.executor import padded_rows
from neuroimagedisttraining_amd.engine.resnet3d_hip import ResNet3DHipEngine
from neuroimagedisttraining_amd.models.resnet3d import resnet3d_50
dev = torch.device("cuda")
torch.manual_seed(0)
G, B = 2, 2
vol = torch.randint(0, 256, (G * B, 40, 48, 40), dtype=torch.uint8, device=dev)
m = resnet3d_50(num_classes=1)
eng = ResNet3DHipEngine(m, vol, torch.zeros(G * B, device=dev), dev)
L, Lb = eng.players, eng.blayers
flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(dev)
bflat = torch.cat([b.detach().float().reshape(-1) for b in m.buffers()]).to(dev)
th = padded_rows(G, L.total, dev); bu = padded_rows(G, Lb.total, dev)
th.copy_(flat.expand(G, -1)); bu.copy_(bflat.expand(G, -1))
with torch.no_grad():
    logits, pooled, saved, stem = eng.net.forward(vol, th, bu, G, True)
mref = resnet3d_50(num_classes=1).to(dev); mref.train()
acts = {}
def hook(name):
    def f(mod, inp, out):
        acts[name] = out.detach()
    return f
hs = [mref.maxpool.register_forward_hook(hook("stem"))]
names = []
for li in range(1, 5):
    for bi, blk in enumerate(getattr(mref, "layer%d" % li)):
        nm = "layer%d.%d" % (li, bi); names.append(nm)
        hs.append(blk.register_forward_hook(hook(nm)))
pv = {n: flat[o:o + L.numel(i)].view(L.shapes[i]) for i, (n, o) in enumerate(zip(L.names, L.offsets))}
bv = {n: bflat[o:o + Lb.numel(i)].view(Lb.shapes[i]).clone().to(Lb.dtypes[i]) for i, (n, o) in enumerate(zip(Lb.names, Lb.offsets))}
with torch.no_grad():
    out = functional_call(mref, {**pv, **bv}, (vol[:B].float().unsqueeze(1) / 255.0,))
def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())
st = stem[0][:B]
print("stem", tuple(st.shape), rel(st, acts["stem"].permute(0, 2, 3, 4, 1)))
for nm, sv in zip(names, saved):
    a = sv[-1][:B]
    r = acts[nm].permute(0, 2, 3, 4, 1)
    print(nm, tuple(a.shape), tuple(r.shape), rel(a, r))
print("logits", logits[:B].flatten().tolist(), out.flatten().tolist())
