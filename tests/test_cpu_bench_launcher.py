"""bench.py's multi-GPU contract, rehearsed on the CPU twin engine with gloo (``--device cpu``).

* ``--gpus N`` without torchrun self-launches N ranks (verdict r3 item 1) and reports ``n_gpus == N``;
* the torchrun launch shape gives the same result;
* the sharded run's round metrics equal the single-process run's (clients sharded over ranks, one all-reduce);
* a rank count that disagrees with ``--gpus`` fails loudly instead of reporting the wrong ``n_gpus``.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
TINY = ["--device", "cpu", "--clients", "8", "--train-per-client", "8", "--test-per-client", "4", "--batch", "4",
        "--steps", "1", "--warmup", "1"]


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, env=env or _env(), cwd=ROOT, timeout=300)
    return r


def _json(r, strict=True):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    if not strict:  # torchrun: gloo's C++ connection banner also lands on the ranks' stdout
        lines = [ln for ln in lines if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0's JSON line is the only stdout line
    return json.loads(lines[0])


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_self_launch_four_ranks_matches_one_process():
    one = _json(_run([sys.executable, BENCH, "--gpus", "1"] + TINY))
    env = _env()
    env["NIDT_DEFER_METRICS"] = "force"   # the GPU default: metrics read back one round late (pinned copy + event)
    four = _json(_run([sys.executable, BENCH, "--gpus", "4"] + TINY, env=env))
    assert one["n_gpus"] == 1 and four["n_gpus"] == 4
    assert four["config"]["parallelism"].endswith("dp4") and len(four["rank_wall_s"]) == 4
    assert four["metric"] == one["metric"]
    for k, v in one["last_round_metrics"].items():
        assert np.isclose(four["last_round_metrics"][k], v, rtol=1e-5, atol=1e-6), (k, v, four["last_round_metrics"])


def test_eight_ranks_headline_layout_matches_one_process():
    """The headline layout of the driver's 8-GPU scaling run: 64 clients, 8 per rank, deferred metrics."""
    big = ["--device", "cpu", "--clients", "64", "--train-per-client", "4", "--test-per-client", "2", "--batch", "4",
           "--steps", "1", "--warmup", "1"]
    one = _json(_run([sys.executable, BENCH, "--gpus", "1"] + big))
    env = _env()
    env["NIDT_DEFER_METRICS"] = "force"
    eight = _json(_run([sys.executable, BENCH, "--gpus", "8"] + big, env=env))
    assert eight["n_gpus"] == 8 and len(eight["rank_wall_s"]) == 8
    assert eight["config"]["parallelism"].endswith("dp8") and eight["config"]["clients"] == 64
    for k, v in one["last_round_metrics"].items():
        assert np.isclose(eight["last_round_metrics"][k], v, rtol=1e-5, atol=1e-6), (k, v, eight["last_round_metrics"])


def test_torchrun_launch_shape_still_works():
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), BENCH, "--gpus", "2"] + TINY)
    assert _json(r, strict=False)["n_gpus"] == 2


def test_rank_count_mismatch_fails_loudly():
    env = _env()
    env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = _run([sys.executable, BENCH, "--gpus", "2"] + TINY, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
    assert not r.stdout.strip()
