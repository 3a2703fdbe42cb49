"""Per-layer timing of the 2-D 3x3 stride-1 convs (CIFAR / Tiny ResNet-18 layers 1-3, B = 16 per client) on the
per-tap client-grouped kernel (``conv_fwd``) vs the kd-slab union kernel (``conv2d_fwd_slab``), for several client
counts.  CUDA-event timing of 50 launches after 5 warmups, interleaved per shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuroimagedisttraining_amd import ops  # noqa: E402
from neuroimagedisttraining_amd.engine import resnet2d_hip as R  # noqa: E402


def main():
    m = ops.ext()
    dev = torch.device("cuda:0")
    B = 16
    shapes = [(32, 64, 64), (16, 128, 128), (8, 256, 256), (64, 64, 64), (32, 128, 128), (16, 256, 256)]
    Gs = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 10, 100]
    print("H=W Cin Cout G | per-tap us | slab us | ratio")
    for H, cin, cout in shapes:
        if not m.conv2d_fwd_slab_ok(B, H, H, cin, cout):
            continue
        for G in Gs:
            x = torch.randn(G * B, H, H, cin, device=dev).bfloat16()
            w = (torch.randn(G, cout, 9, cin, device=dev) * 0.05).bfloat16()
            y = torch.empty(G * B, H, H, cout, device=dev, dtype=torch.bfloat16)
            tab = torch.empty(m.conv3d_fwd_slab_table_size(B, 1, H, H, 1), device=dev, dtype=torch.int32)
            m.conv3d_fwd_slab_table(tab.data_ptr(), B, 1, H, H, 1, R._stream())

            def tap():
                R.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, 1, H, H, cin, cout, 9, 1, 1, 0, dev)

            def slab():
                m.conv2d_fwd_slab(x.data_ptr(), w.data_ptr(), y.data_ptr(), G, B, H, H, cin, cout, tab.data_ptr(),
                                  R._stream())

            res = {}
            for name, fn in (("tap", tap), ("slab", slab), ("tap2", tap), ("slab2", slab)):
                for _ in range(5):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[name] = e0.elapsed_time(e1) * 1000 / 50
            t = min(res["tap"], res["tap2"])
            s = min(res["slab"], res["slab2"])
            print(f"{H:3d} {cin:4d} {cout:4d} {G:4d} | {t:9.1f} | {s:9.1f} | {s / t:.3f}", flush=True)


if __name__ == "__main__":
    main()
