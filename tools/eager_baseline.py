"""Reference-semantics eager baseline on MI355X (the anchor for vs_baseline in bench.py / BASELINE.md).

Re-implements the reference's SalientGrads round loop as the reference runs it — one shared nn.Module,
clients trained sequentially, ``load_state_dict`` / ``deepcopy(model.cpu().state_dict())`` per client, SGD
rebuilt per client, ``clip_grad_norm_(10)``, the mask multiplied into every parameter after every step with
the mask tensors moved host->device each time (``sailentgrads/my_model_trainer.py:201-235``), CPU-side
sample-weighted aggregation (``sailentgrads_api.py:212-227``) and global + personal evaluation of every client
(``:231-285``) — in PyTorch-ROCm eager fp32 (MIOpen).  Data is kept resident on the GPU (the reference re-reads
an HDF5 file per batch; skipping that makes this baseline *faster* than the reference would be).

Usage: python tools/eager_baseline.py [--clients 64] [--rounds 1] [--dtype fp32|bf16]
"""
import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--train", type=int, default=144)
    ap.add_argument("--test", type=int, default=36)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="fp32")
    args = ap.parse_args()
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    vol, labels, splits = build_fl_volumes(list(range(args.clients)), args.clients, args.train, args.test, dev, seed=1024)
    model = AlexNet3D_Dropout(num_classes=1).to(dev)
    # SNIP-style mask: random 50% for the timing baseline (mask generation is one-time, outside the round)
    masks = {}
    for n, p in model.named_parameters():
        masks[n] = ((torch.rand_like(p) > 0.5).float() if p.dim() > 1 else torch.ones_like(p)).cpu()
    crit = nn.BCEWithLogitsLoss()
    amp = args.dtype == "bf16"
    w_global = copy.deepcopy(model.cpu().state_dict())
    model.to(dev)
    w_per = [copy.deepcopy(w_global) for _ in range(args.clients)]

    def batches(c, rnd, ep):
        tr = splits[c].train
        perm = np.random.RandomState(rnd * 1000 + ep * 100 + c).permutation(len(tr))
        for s in range(0, len(tr), args.batch):
            yield torch.from_numpy(tr[perm[s:s + args.batch]]).to(dev)

    def test(w, c):
        model.load_state_dict(w)
        model.eval()
        correct = tot = loss = 0.0
        with torch.no_grad():
            te = torch.from_numpy(splits[c].test).to(dev)
            for s in range(0, te.numel(), args.batch):
                ix = te[s:s + args.batch]
                x = (vol[ix].float() / 255.0).unsqueeze(1)
                y = labels[ix]
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                    pred = torch.sigmoid(model(x).float())
                loss += crit(pred, y.view(-1, 1)).item() * ix.numel()
                correct += ((pred >= 0.5).float().squeeze(1) == y).float().sum().item()
                tot += ix.numel()
        return correct / tot, loss / tot

    times = []
    for rnd in range(args.rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w_locals = []
        for c in range(args.clients):
            model.load_state_dict(w_global)
            model.to(dev)
            model.train()
            opt = torch.optim.SGD(model.parameters(), lr=0.01 * 0.998 ** rnd, momentum=0, weight_decay=5e-4)
            for ep in range(args.epochs):
                el = []
                for ix in batches(c, rnd, ep):
                    x = (vol[ix].float() / 255.0).unsqueeze(1)
                    y = labels[ix]
                    model.zero_grad()
                    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                        out = model(x)
                    loss = crit(out.float(), y.view(-1, 1))
                    loss.backward()
                    torch.nn.utils.clip_grad_norm_(model.parameters(), 10)
                    opt.step()
                    el.append(loss.item())
                    for n, p in model.named_parameters():
                        p.data *= masks[n].to(dev)
            w = copy.deepcopy(model.cpu().state_dict())
            model.to(dev)
            w_per[c] = w
            w_locals.append((len(splits[c].train), w))
        tot = sum(n for n, _ in w_locals)
        w_global = copy.deepcopy(w_locals[0][1])
        for k in w_global:
            for i, (n, w) in enumerate(w_locals):
                if i == 0:
                    w_global[k] = w[k] * (n / tot)
                else:
                    w_global[k] += w[k] * (n / tot)
        g_acc = [test(w_global, c)[0] for c in range(args.clients)]
        p_acc = [test(w_per[c], c)[0] for c in range(args.clients)]
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        print(json.dumps({"round": rnd, "seconds": round(times[-1], 2), "global_acc": float(np.mean(g_acc)),
                          "person_acc": float(np.mean(p_acc))}), flush=True)
    steady = times[1:] if len(times) > 1 else times  # round 0 includes MIOpen find / allocator warm-up
    print(json.dumps({"eager_baseline_rounds_per_s": round(1.0 / float(np.mean(steady)), 5), "dtype": args.dtype,
                      "clients": args.clients, "seconds_per_round": round(float(np.mean(steady)), 2),
                      "first_round_s": round(times[0], 2), "rounds_timed": len(steady)}), flush=True)


if __name__ == "__main__":
    main()
