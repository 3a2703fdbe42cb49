#!/bin/bash
# Other BASELINE configs on one MI355X: config 2 (FedAvg, 8 clients) and config 4 (FedProx + Krum / median,
# 128 Dirichlet clients), through the same bench harness.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --algorithm fedavg --clients 8 --steps 3 --warmup 1 > gpurun_out/cfg2.txt 2>&1 || exit $?
timeout -k 10 500 python bench.py --algorithm fedprox --aggregator krum --clients 128 --steps 2 --warmup 1 > gpurun_out/cfg4_krum.txt 2>&1 || exit $?
timeout -k 10 500 python bench.py --algorithm fedprox --aggregator median --clients 128 --steps 2 --warmup 1 > gpurun_out/cfg4_median.txt 2>&1 || exit $?
