#!/bin/bash
# Reference-compatible entry points on the GPU: SalientGrads and FedAvg through the HIP engine, DisPFL (torch engine).
set -o pipefail
mkdir -p gpurun_out/cli
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/gpurun_out/cli"
R="$GRAFT_REPO_ROOT/fedml_experiments/standalone"
timeout -k 10 300 python $R/sailentgrads/main_sailentgrads.py --client_num_in_total 8 --comm_round 2 --n_per_client 40 --engine hip > sg.txt 2>&1 || exit $?
timeout -k 10 300 python $R/fedavg/main_fedavg.py --client_num_in_total 8 --comm_round 2 --n_per_client 40 --engine hip > fa.txt 2>&1 || exit $?
ls -R LOG > logs.txt 2>&1 || true
