"""Compare two c1_evalmode2 dumps tensor by tensor (per client where the leading dim is G or G*B)."""
import sys

import torch

a, b = torch.load(sys.argv[1], weights_only=False), torch.load(sys.argv[2], weights_only=False)
for k in sorted(a):
    if k.startswith("__") or not torch.is_tensor(a[k]) or a[k].shape != b[k].shape:
        continue
    x, y = a[k].double(), b[k].double()
    if a[k].dtype in (torch.uint8, torch.int32, torch.int64, torch.int16):
        d = float((a[k] != b[k]).double().mean())
        if d:
            print("%-10s %-24s mismatch frac %.3e" % (k, tuple(a[k].shape), d))
        continue
    n = float(y.norm()) + 1e-30
    e = float((x - y).norm()) / n
    if e > 1e-3:
        print("%-10s %-24s relerr %.3e" % (k, tuple(a[k].shape), e))
ga, gb = a["__grads"], b["__grads"]
for n, o, k in a["__names"]:
    for g in range(ga.shape[0]):
        e = float((ga[g, o:o + k] - gb[g, o:o + k]).norm() / (gb[g, o:o + k].norm() + 1e-30))
        if e > 1e-3:
            print("grad %-22s client %d relerr %.3e" % (n, g, e))
