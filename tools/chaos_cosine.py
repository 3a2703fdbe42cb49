"""Chaos control for the HIP-vs-fp32 update-direction comparison of tests/test_gpu_personalized.py: after R rounds
of each algorithm, the cosine between the HIP engine's update and the fp32 engine's, next to the cosine between two
fp32 runs whose initial weights differ by 1e-6 relative noise and to the bf16-autocast fp32 engine's.
Usage: python tools/chaos_cosine.py [algo ...] [--rounds R]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import test_gpu_personalized as T
    ap = argparse.ArgumentParser()
    ap.add_argument("algos", nargs="*", default=["fedavg", "salientgrads", "local", "ditto"])
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    fed = T._fed(T.SIZES)
    for algo in a.algos:
        kw = T._extra(algo)
        runs = {k: T._run(algo, e, fed, rounds=a.rounds, **dict(kw, **x))
                for k, e, x in (("hip", "hip", {}), ("fp32", "torch", {}), ("fp32_pert", "torch", {"perturb": 1e-6}),
                                ("amp", "amp", {}))}
        ref, w0 = runs["fp32"]
        u_ref = (ref.theta[:, :ref.P] - w0[:, :ref.P]).double().flatten()
        out = {"algo": algo, "rounds": a.rounds}
        for k in ("hip", "fp32_pert", "amp"):
            r, _ = runs[k]
            u = (r.theta[:, :r.P] - w0[:, :r.P]).double().flatten()
            out["cos_" + k] = round(float(F.cosine_similarity(u, u_ref, dim=0)), 4)
            out["loss_" + k] = r.stat_info.get("global_test_loss", r.stat_info.get("test_loss", [None]))[-1:]
        out["loss_fp32"] = ref.stat_info.get("global_test_loss", ref.stat_info.get("test_loss", [None]))[-1:]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
