"""Process-per-GPU runtime: init, client sharding, bucketed collectives.

One process per MI355X; ``torch.distributed`` with backend ``"nccl"`` (= RCCL on ROCm) rides xGMI
between the GPUs of a node.  On CPU (tests) the same code runs on ``gloo``.

Collective sizing for FL aggregation (SURVEY.md §5 "Distributed communication backend"): one
AlexNet3D state is 10.3 MB fp32, so a round's aggregation is ONE all-reduce of the
``[P + Q + 1]`` partial-sum vector (weighted params, weighted buffers, sample count) — below any
sensible bucket size; :func:`all_reduce_buckets` splits larger payloads (3D ResNet-50 ≈185 MB per
model) into ``bucket_mb`` chunks, launched back to back on the communication stream so RCCL's
channels over the 7 xGMI links stay busy while the previous chunk is reduced.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self):
        return self.rank == 0

    @property
    def enabled(self):
        return self.world > 1 and dist.is_available() and dist.is_initialized()


def init_distributed(prefer_gpu=True, timeout_s=600) -> DistInfo:
    """Initialise from torchrun-style env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/PORT).

    Single process (no env) -> world 1 without a process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # NIDT_DIST_BACKEND=gloo rehearses the multi-rank GPU path on ONE GPU (several ranks on cuda:0, gloo
        # collectives on device tensors) where RCCL refuses two ranks on the same device
        backend = os.environ.get("NIDT_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        if not dist.is_initialized():
            kw = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if use_gpu and backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(**kw)
    return DistInfo(rank, world, local, device, backend)


def shard_clients(sizes, world):
    """Contiguous client blocks per rank, balanced by sample count (greedy prefix split).

    Clients of equal size (the headline config) get exactly ``N/world`` clients per rank."""
    n = len(sizes)
    if world <= 1:
        return [list(range(n))]
    sizes = np.asarray(sizes, dtype=np.float64)
    if np.allclose(sizes, sizes[0]) and n % world == 0:
        per = n // world
        return [list(range(r * per, (r + 1) * per)) for r in range(world)]
    target = sizes.sum() / world
    out, cur, acc = [], [], 0.0
    for i, s in enumerate(sizes):
        remaining_ranks = world - len(out)
        remaining_clients = n - i
        if cur and (acc + s / 2 > target and remaining_ranks > 1 or remaining_clients < remaining_ranks):
            out.append(cur)
            cur, acc = [], 0.0
        cur.append(i)
        acc += s
    out.append(cur)
    while len(out) < world:
        out.append([])
    return out


def all_reduce_buckets(t: torch.Tensor, info: DistInfo, bucket_mb=256.0, op=None):
    """In-place SUM all-reduce of a flat tensor in ``bucket_mb`` chunks (async, then wait)."""
    if not info.enabled:
        return t
    op = op or dist.ReduceOp.SUM
    flat = t.view(-1)
    step = max(1, int(bucket_mb * 1024 * 1024 // flat.element_size()))
    works = [dist.all_reduce(flat[s:s + step], op=op, async_op=True) for s in range(0, flat.numel(), step)]
    for w in works:
        w.wait()
    return t


def all_gather_cat(t: torch.Tensor, info: DistInfo):
    """All-gather variable-length 1-D tensors (size exchange, pad, gather, trim)."""
    if not info.enabled:
        return t
    n = torch.tensor([t.numel()], device=t.device, dtype=torch.long)
    sizes = [torch.zeros_like(n) for _ in range(info.world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    pad = torch.zeros(m, device=t.device, dtype=t.dtype)
    pad[:t.numel()] = t.view(-1)
    bufs = [torch.zeros_like(pad) for _ in range(info.world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


def all_gather_sized(t: torch.Tensor, sizes, info: DistInfo):
    """All-gather 1-D tensors whose per-rank lengths ``sizes`` every rank already knows (e.g. k values per sampled
    client of each rank): one padded all-gather, no size exchange and no host sync."""
    if not info.enabled:
        return t
    m = max(int(s) for s in sizes)
    pad = torch.zeros(max(1, m), device=t.device, dtype=t.dtype)
    pad[:t.numel()] = t.view(-1)
    bufs = [torch.empty_like(pad) for _ in range(info.world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:int(s)] for b, s in zip(bufs, sizes)])


def exchange_rows(info: DistInfo, owner, needs, row_of, width, device, dtype=torch.float32):
    """Point-to-point fetch of client rows (gossip neighbours, FedFomo candidates) — RCCL send/recv over xGMI
    instead of an all-gather of every client.

    ``owner[c]``: rank holding client c; ``needs[r]``: clients rank r needs (every rank passes the same ``needs``,
    so both sides of each transfer agree on the schedule); ``row_of(c)`` -> 1-D tensor [width] of a client this rank
    owns; ``width``: an int, or a function of the client (variable-length payloads, e.g. a client's sample rows).
    Returns {c: tensor [width]} for this rank's remote needs.  All transfers go out as one batched group."""
    if not info.enabled:
        return {}
    import torch.distributed as dist
    # gloo moves device tensors through slow internal staging: stage through host memory ourselves (the RCCL
    # path sends the device rows directly over xGMI)
    stage = info.backend == "gloo" and torch.device(device).type == "cuda"
    p2p, recv = [], {}
    for r in range(info.world):
        for c in sorted(set(needs[r])):
            o = int(owner[c])
            if o == r:
                continue
            if o == info.rank:
                t = row_of(c).contiguous()
                p2p.append(dist.P2POp(dist.isend, t.cpu() if stage else t, r))
            if r == info.rank:
                w = width(c) if callable(width) else width
                buf = torch.empty(w, dtype=dtype, device="cpu" if stage else device)
                recv[c] = buf
                p2p.append(dist.P2POp(dist.irecv, buf, o))
    if p2p:
        for q in dist.batch_isend_irecv(p2p):
            q.wait()
    if stage:
        recv = {c: b.to(device) for c, b in recv.items()}
    return recv


def barrier(info: DistInfo):
    if info.enabled:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def max_over_ranks(x: float, info: DistInfo, device=None):
    if not info.enabled:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown(info: DistInfo):
    if info.enabled:
        dist.destroy_process_group()
