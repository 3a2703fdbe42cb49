#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box: 2 ranks on cuda:0 with gloo collectives (RCCL refuses two ranks on one
# device) through torchrun, exactly the driver's launch line otherwise; then the same config on 1 rank.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NIDT_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --clients 16 --steps 2 --warmup 1 > gpurun_out/rehearse2.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --clients 16 --steps 2 --warmup 1 > gpurun_out/rehearse1.txt 2>&1 || exit $?
