"""Convergence parity of the bf16 HIP engine against the fp32 PyTorch engine over a multi-round federation.

The default synthetic cohort is too easy to reveal a numerics regression (accuracy saturates at 1.0), so this test
uses a weak label signal: the fp32 reference needs ~10 rounds to leave the majority-class plateau, and the HIP
engine's global loss / accuracy trajectories must track it (round by round before the transition, without lagging
after it).  6 clients, SalientGrads (SNIP mask + masked FedAvg), 20 rounds, every
round evaluated.  The fp32 side is the recorded trajectory of the fp32 engine on this cohort; the extended tier
(``NIDT_EXTENDED_GPU_TESTS=1``) recomputes it and checks the record is current."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROUNDS = 20


def _trajectory(kind, vol, labels, splits):
    from neuroimagedisttraining_amd.data.synthetic_fl import to_hip_store
    from neuroimagedisttraining_amd.engine.executor import FLConfig, HipEngine, TorchEngine
    from neuroimagedisttraining_amd.engine.personalized import make_runner
    from neuroimagedisttraining_amd.models.alexnet3d import AlexNet3D_Dropout
    from neuroimagedisttraining_amd.parallel import runtime as rt
    torch.manual_seed(0)
    model = AlexNet3D_Dropout(num_classes=1)
    if kind == "hip":
        x8, mom = to_hip_store(vol)
        eng = HipEngine(model, x8, mom, labels, DEV)
    else:
        eng = TorchEngine(model, vol, labels, DEV)
    cfg = FLConfig(comm_round=ROUNDS, epochs=2, batch_size=8, lr=0.05, dense_ratio=0.5, seed=5, dropout_keep=1.0,
                   test_batch=64, final_round=False)
    r = make_runner("salientgrads", eng, splits, cfg, rt.DistInfo(device=torch.device(DEV)), model)
    r.generate_global_mask_snip()
    for k in range(ROUNDS):
        res = r.run_round(k)
        print(kind, "round", k, res, flush=True)  # progress (the fp32 engine takes minutes)
    return np.array(r.stat_info["global_test_acc"]), np.array(r.stat_info["global_test_loss"])


REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "convergence_fp32_reference.json")


def _cohort():
    from neuroimagedisttraining_amd.data.synthetic_fl import build_fl_volumes
    C = 6
    vol, labels, local = build_fl_volumes(list(range(C)), C, 32, 16, DEV, seed=21, alpha=1.0, label_signal=0.25)
    return vol, labels, [local[c] for c in range(C)]


def _reference():
    with open(REF) as f:
        d = json.load(f)
    return np.array(d["acc"]), np.array(d["loss"])


def _fingerprint(vol, labels, splits):
    """Hash of the cohort the recorded fp32 trajectory belongs to: labels, client splits, per-subject voxel sums and a
    strided voxel sample.  A change of build_fl_volumes / the synthetic RNG shows up here instead of silently
    comparing the bf16 run against a stale trajectory."""
    h = hashlib.sha256()
    h.update(labels.detach().float().cpu().numpy().tobytes())
    for sp in splits:
        for part in (getattr(sp, "train", None), getattr(sp, "test", None)):
            h.update(np.asarray(part if part is not None else sp, dtype=np.int64).tobytes())
    h.update(vol.reshape(vol.shape[0], -1).to(torch.int64).sum(1).cpu().numpy().tobytes())
    h.update(vol.reshape(-1)[::9973].cpu().numpy().tobytes())
    return h.hexdigest()[:16]


def _check_fingerprint(vol, labels, splits):
    with open(REF) as f:
        want = json.load(f).get("fingerprint")
    got = _fingerprint(vol, labels, splits)
    print("cohort fingerprint", got, flush=True)
    assert want is not None, "record the cohort fingerprint %s in %s" % (got, REF)
    assert got == want, "cohort changed (%s != recorded %s): re-record the fp32 trajectory (extended tier)" % (got, want)


def test_hip_bf16_tracks_fp32_over_twenty_rounds():
    """HIP bf16 trajectory against the fp32 engine's trajectory on the same cohort.  The fp32 run (~4-5 minutes of
    MIOpen fp32 at full resolution) is the recorded one (``tests/data/convergence_fp32_reference.json``); the
    extended tier recomputes it live (:func:`test_fp32_reference_trajectory_is_current` and
    ``NIDT_CONVERGENCE_LIVE=1`` here)."""
    vol, labels, splits = _cohort()
    live = os.environ.get("NIDT_CONVERGENCE_LIVE", "0") == "1"
    if not live:
        _check_fingerprint(vol, labels, splits)
    acc_h, loss_h = _trajectory("hip", vol, labels, splits)
    if live:
        acc_t, loss_t = _trajectory("torch", vol, labels, splits)
    else:
        acc_t, loss_t = _reference()
    print("fp32 acc ", np.round(acc_t, 3).tolist())
    print("bf16 acc ", np.round(acc_h, 3).tolist())
    print("fp32 loss", np.round(loss_t, 4).tolist())
    print("bf16 loss", np.round(loss_h, 4).tolist())
    # learning is chaotic at the transition off the majority-class plateau (rounds ~10-15): two fp32 runs whose
    # initial weights differ by 1e-6 relative noise end up to 6.7 % apart in loss there, bf16 autocast 4.8 %
    # (tools/convergence_ablation.py, profiles/r3_convergence_ablation.txt).  Before it the trajectories are
    # deterministic functions of the numerics and are compared round by round; after it, on window means, one-sided
    # where the question is "does bf16 lag fp32".
    assert np.mean(acc_t[-10:]) < 0.97, "cohort too easy: the comparison would not see a numerics regression"
    assert acc_t[-5:].max() > 0.85 and acc_h[-5:].max() > 0.85, "both engines must learn the task"
    assert np.max(np.abs(loss_h[:10] - loss_t[:10]) / loss_t[:10]) <= 0.03       # ablation: 0.018 (chaos ctl 0.017)
    first = lambda a: int(np.argmax(a >= 0.7)) if (a >= 0.7).any() else len(a)  # noqa: E731
    assert first(acc_h) <= first(acc_t) + 2, "bf16 leaves the plateau later than fp32"
    assert np.mean(acc_h[-5:]) >= np.mean(acc_t[-5:]) - 0.05                     # no accuracy lag
    assert abs(np.mean(acc_h[-5:]) - np.mean(acc_t[-5:])) <= 0.1
    assert np.mean(loss_h[-5:]) <= 1.05 * np.mean(loss_t[-5:])                   # no loss lag


@pytest.mark.extended
def test_fp32_reference_trajectory_is_current():
    """The recorded fp32 trajectory is what the fp32 engine produces today: rounds 0-9 (before the chaotic
    transition) within the run-to-run spread of fp32 itself (1.7 % under 1e-6 weight noise, r3 ablation)."""
    vol, labels, splits = _cohort()
    _check_fingerprint(vol, labels, splits)
    acc_t, loss_t = _trajectory("torch", vol, labels, splits)
    acc_r, loss_r = _reference()
    assert np.max(np.abs(loss_t[:10] - loss_r[:10]) / loss_r[:10]) <= 0.02
    assert acc_t[-5:].max() > 0.85
