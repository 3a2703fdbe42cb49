"""Probe: PyTorch-ROCm (MIOpen) timings for AlexNet3D layers at ABCD shape.

Used once to anchor the eager baseline and size the HIP kernel work.  Prints one line per case.
"""
import sys, time, json
import torch
import torch.nn.functional as F

dev = "cuda"
torch.backends.cudnn.benchmark = True


def timeit(fn, iters=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
layers = [  # name, cin, cout, k, s, p, in spatial
    ("conv1", 1, 64, 5, 2, 0, (121, 145, 121)),
    ("conv2", 64, 128, 3, 1, 0, (19, 23, 19)),
    ("conv3", 128, 192, 3, 1, 1, (5, 7, 5)),
    ("conv4", 192, 192, 3, 1, 1, (5, 7, 5)),
    ("conv5", 192, 128, 3, 1, 1, (5, 7, 5)),
]
res = {}
for dt in (torch.bfloat16, torch.float32):
    for cl in (False, True):
        for name, ci, co, k, s, p, sp in layers:
            x = torch.randn(B, ci, *sp, device=dev, dtype=dt)
            w = torch.randn(co, ci, k, k, k, device=dev, dtype=dt) * 0.05
            b = torch.zeros(co, device=dev, dtype=dt)
            if cl:
                x = x.contiguous(memory_format=torch.channels_last_3d)
                w = w.contiguous(memory_format=torch.channels_last_3d)
            x.requires_grad_(name != "conv1")
            w.requires_grad_(True)
            try:
                y = F.conv3d(x, w, b, s, p)
                gy = torch.randn_like(y)
                tf = timeit(lambda: F.conv3d(x, w, b, s, p))
                def fb():
                    yy = F.conv3d(x, w, b, s, p)
                    yy.backward(gy)
                tfb = timeit(fb)
                fl = 2.0 * y.numel() * ci * k ** 3
                res[f"{name}-{str(dt)[6:]}-cl{int(cl)}"] = (tf, tfb)
                print(f"{name} {dt} cl={cl} fwd {tf:.3f} ms ({fl/tf/1e9:.1f} TF/s)  fwd+bwd {tfb:.3f} ms ({fl*(3 if name!='conv1' else 2)/tfb/1e9:.1f} TF/s)", flush=True)
            except Exception as e:
                print(f"{name} {dt} cl={cl} FAILED {e}", flush=True)

# full model eager fwd+bwd (reference semantics, fp32) at batch B
sys.path.insert(0, ".")
from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
for dt in (torch.float32, torch.bfloat16):
    m = AlexNet3D_Dropout(num_classes=1).to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=0.01, weight_decay=5e-4)
    x = torch.rand(B, 1, 121, 145, 121, device=dev)
    y = torch.randint(0, 2, (B, 1), device=dev).float()
    lossf = torch.nn.BCEWithLogitsLoss()
    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == torch.bfloat16)):
            out = m(x)
        loss = lossf(out.float(), y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 10)
        opt.step()
    t = timeit(step, iters=5, warm=2)
    print(f"full-model eager train step B={B} {dt}: {t:.2f} ms  ({22.4*B/t:.1f} TF/s eff @22.4GF/sample)", flush=True)
