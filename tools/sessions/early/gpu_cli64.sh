#!/bin/bash
# Headline-scale run through the reference entry point (64 clients, 3 rounds, HIP engine) and a longer bench.
set -o pipefail
mkdir -p gpurun_out/cli64
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/gpurun_out/cli64"
R="$GRAFT_REPO_ROOT/fedml_experiments/standalone"
timeout -k 10 400 python $R/sailentgrads/main_sailentgrads.py --client_num_in_total 64 --comm_round 3 --n_per_client 180 --engine hip > sg64.txt 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 12 --warmup 2 > gpurun_out/cli64/bench64_12steps.txt 2>&1 || exit $?
