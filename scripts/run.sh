#!/bin/bash
# Launch a reference-compatible entry point on one MI355X node: one process per GPU (torchrun, RCCL over xGMI).
#   scripts/run.sh <algo> [NGPUS] [flags...]
# <algo>: sailentgrads | fedavg | fedprox | DisPFL | subavg | ditto | dpsgd | fedfomo | local
# The SLURM job files of the reference (fedml_experiments/standalone/*/Jobs, *.sh) map onto this with the same
# flags; LOG/<dataset>/<identity>.log is written by rank 0.
set -euo pipefail
ALGO=${1:?algo}; shift
NGPU=${1:-1}; [[ $# -gt 0 ]] && shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
case $ALGO in DisPFL) MAIN=main_dispfl.py;; *) MAIN=main_${ALGO}.py;; esac
export HSA_ENABLE_IPC_MODE_LEGACY=${HSA_ENABLE_IPC_MODE_LEGACY:-0}
if [[ $NGPU -gt 1 ]]; then
  exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
       --master-port "${MASTER_PORT:-29511}" "$ROOT/fedml_experiments/standalone/$ALGO/$MAIN" "$@"
else
  exec python "$ROOT/fedml_experiments/standalone/$ALGO/$MAIN" "$@"
fi
