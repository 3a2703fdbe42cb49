#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box (2 ranks on cuda:0, gloo collectives: RCCL refuses two ranks on one device):
# headline config at 16 clients (2 ranks) and 32 clients (4 ranks), FedAvg frac 0.5 with per-round rebalancing (row
# migration) and static, then 1 rank.  Round-3 code (slab kernels, sharded rebalancing data, radix top-k aggregation).
set -o pipefail
mkdir -p gpurun_out/r3reh
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 > gpurun_out/r3reh/two_ranks.txt 2>&1 || { tail -20 gpurun_out/r3reh/two_ranks.txt; exit 1; }
grep '^{' gpurun_out/r3reh/two_ranks.txt | cut -c1-250
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 --algorithm fedavg --frac 0.5 --size-skew 1.0 --rebalance 1 --phase-timers > gpurun_out/r3reh/two_ranks_rebalance.txt 2>&1 || { tail -20 gpurun_out/r3reh/two_ranks_rebalance.txt; exit 1; }
grep '^{' gpurun_out/r3reh/two_ranks_rebalance.txt | cut -c1-400
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 --algorithm fedavg --frac 0.5 --size-skew 1.0 --rebalance 0 --phase-timers > gpurun_out/r3reh/two_ranks_static.txt 2>&1 || { tail -20 gpurun_out/r3reh/two_ranks_static.txt; exit 1; }
grep '^{' gpurun_out/r3reh/two_ranks_static.txt | cut -c1-400
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --clients 32 --steps 2 --warmup 1 > gpurun_out/r3reh/four_ranks.txt 2>&1 || { tail -20 gpurun_out/r3reh/four_ranks.txt; exit 1; }
grep '^{' gpurun_out/r3reh/four_ranks.txt | cut -c1-250
timeout -k 10 300 python bench.py --clients 16 --steps 2 --warmup 1 > gpurun_out/r3reh/one_rank.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3reh/one_rank.txt | cut -c1-250
