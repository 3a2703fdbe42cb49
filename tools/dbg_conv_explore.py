"""Explore synthetic-cohort difficulty on the HIP engine (fast) for the convergence parity test."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import test_gpu_convergence as T
from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes
for sig in (0.15, 0.25, 0.4):
    for lr, ep in ((0.05, 2), (0.1, 2)):
        vol, labels, local = build_fl_volumes(list(range(6)), 6, 32, 16, "cuda", seed=21, alpha=1.0, label_signal=sig)
        splits = [local[c] for c in range(6)]
        from neuroimagedisttraining_amd.engine.executor import FLConfig
        orig = FLConfig.__init__
        acc, loss = T._trajectory("hip", vol, labels, splits) if False else (None, None)
        import neuroimagedisttraining_amd.engine.personalized as PZ
        from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
        from neuroimagedisttraining_amd.engine.executor import HipEngine
        from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
        from neuroimagedisttraining_amd.parallel import runtime as rt
        torch.manual_seed(0)
        model = AlexNet3D_Dropout(num_classes=1)
        x8, mom = to_hip_store(vol)
        eng = HipEngine(model, x8, mom, labels, "cuda")
        cfg = FLConfig(comm_round=20, epochs=ep, batch_size=8, lr=lr, dense_ratio=0.5, seed=5, dropout_keep=1.0, test_batch=64, final_round=False)
        r = PZ.make_runner("salientgrads", eng, splits, cfg, rt.DistInfo(device=torch.device("cuda")), model)
        r.generate_global_mask_snip()
        for k in range(20):
            r.run_round(k)
        print("signal", sig, "lr", lr, "ep", ep, "acc", np.round(r.stat_info["global_test_acc"], 2).tolist(), flush=True)
