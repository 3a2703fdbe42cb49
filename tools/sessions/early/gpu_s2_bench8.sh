#!/bin/bash
# 1-GPU bench at the headline load (64 clients) and at the 8-clients-per-GPU load of an 8-GPU node
set -o pipefail
mkdir -p gpurun_out/b8
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/b8/bench64.txt 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --clients 8 --steps 20 --warmup 3 > gpurun_out/b8/bench8.txt 2>&1 || exit 1
grep -h '^{' gpurun_out/b8/bench64.txt gpurun_out/b8/bench8.txt | cut -c1-200
