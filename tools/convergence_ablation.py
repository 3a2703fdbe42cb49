"""Where does the bf16 engine's trajectory lag come from?  Ablations of the 20-round convergence federation of
tests/test_gpu_convergence.py (6 clients, SalientGrads, weak label signal, lr 0.05, dropout off):

  fp32        TorchEngine, fp32 (MIOpen)                          - the reference trajectory
  fp32_pert   the same with the initial weights perturbed by 1 ulp-scale noise (x (1 + 1e-6 N(0,1))): the
              chaos control — how far two fp32 runs that differ only at rounding level drift apart
  fp32_sum    TorchEngine fp32 with every conv's reduction order changed (cudnn/MIOpen benchmark algorithm
              selection off vs on): a second rounding-level control
  amp_bf16    TorchEngine under bf16 autocast (MIOpen bf16 convs, fp32 BN / head): bf16 operand rounding only
  hip         the client-batched HIP engine (bf16 MFMA operands, fp32 accumulate and BN statistics)

Prints one JSON line per arm (global test acc / loss per round) and the distances between trajectories.
Usage: python tools/convergence_ablation.py [arm ...] [--rounds 20]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEV = "cuda"


def run(arm, rounds, lr, signal):
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes, to_hip_store
    from neuroimagedisttraining_amd.engine.executor import FLConfig, HipEngine, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.parallel import runtime as rt
    C = 6
    vol, labels, local = build_fl_volumes(list(range(C)), C, 32, 16, DEV, seed=21, alpha=1.0, label_signal=signal)
    splits = [local[c] for c in range(C)]
    torch.manual_seed(0)
    model = AlexNet3D_Dropout(num_classes=1)
    if arm == "fp32_pert":
        g = torch.Generator().manual_seed(99)
        with torch.no_grad():
            for p in model.parameters():
                p.mul_(1 + 1e-6 * torch.randn(p.shape, generator=g))
    torch.backends.cudnn.benchmark = arm == "fp32_sum"
    if arm == "hip":
        x8, mom = to_hip_store(vol)
        eng = HipEngine(model, x8, mom, labels, DEV)
    else:
        eng = TorchEngine(model, vol, labels, DEV, amp=arm == "amp_bf16")
    cfg = FLConfig(comm_round=rounds, epochs=2, batch_size=8, lr=lr, dense_ratio=0.5, seed=5, dropout_keep=1.0,
                   test_batch=64, final_round=False)
    r = make_runner("salientgrads", eng, splits, cfg, rt.DistInfo(device=torch.device(DEV)), model)
    r.generate_global_mask_snip()
    for k in range(rounds):
        r.run_round(k)
        print(arm, "round", k, round(r.stat_info["global_test_acc"][-1], 3),
              round(r.stat_info["global_test_loss"][-1], 4), flush=True)
    return np.array(r.stat_info["global_test_acc"]), np.array(r.stat_info["global_test_loss"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("arms", nargs="*", default=["hip", "fp32", "fp32_pert", "amp_bf16"])
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--signal", type=float, default=0.25)
    args = ap.parse_args()
    out = {}
    for a in args.arms:
        acc, loss = run(a, args.rounds, args.lr, args.signal)
        out[a] = (acc, loss)
        print(json.dumps({"arm": a, "lr": args.lr, "signal": args.signal, "acc": np.round(acc, 3).tolist(),
                          "loss": np.round(loss, 4).tolist()}), flush=True)
    ref = out.get("fp32")
    if ref is not None:
        for a, (acc, loss) in out.items():
            if a == "fp32":
                continue
            rel = np.abs(loss - ref[1]) / ref[1]
            print(json.dumps({"vs_fp32": a, "max_rel_loss_r0_9": round(float(rel[:10].max()), 4),
                              "max_rel_loss_all": round(float(rel.max()), 4),
                              "last5_acc_diff": round(float(abs(acc[-5:].mean() - ref[0][-5:].mean())), 3),
                              "last5_loss_rel": round(float(abs(loss[-5:].mean() - ref[1][-5:].mean())
                                                            / ref[1][-5:].mean()), 4)}), flush=True)


if __name__ == "__main__":
    main()
