#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box (2 ranks on cuda:0, gloo collectives: RCCL refuses two ranks on one device):
# headline config at 16 clients, then FedAvg frac 0.5 with per-round rebalancing (row migration), then 1 rank.
set -o pipefail
mkdir -p gpurun_out/reh
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 > gpurun_out/reh/two_ranks.txt 2>&1 || { tail -20 gpurun_out/reh/two_ranks.txt; exit 1; }
grep '^{' gpurun_out/reh/two_ranks.txt | cut -c1-250
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 --algorithm fedavg --frac 0.5 --size-skew 1.0 --rebalance 1 --phase-timers > gpurun_out/reh/two_ranks_rebalance.txt 2>&1 || { tail -20 gpurun_out/reh/two_ranks_rebalance.txt; exit 1; }
grep '^{' gpurun_out/reh/two_ranks_rebalance.txt | cut -c1-400
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 --algorithm fedavg --frac 0.5 --size-skew 1.0 --rebalance 0 --phase-timers > gpurun_out/reh/two_ranks_static.txt 2>&1 || { tail -20 gpurun_out/reh/two_ranks_static.txt; exit 1; }
grep '^{' gpurun_out/reh/two_ranks_static.txt | cut -c1-400
timeout -k 10 300 python bench.py --clients 16 --steps 2 --warmup 1 > gpurun_out/reh/one_rank.txt 2>&1 || exit 1
grep '^{' gpurun_out/reh/one_rank.txt | cut -c1-250
