#!/bin/bash
# SalientGrads sparsity / IterSNIP sweep (the reference's Jobs/*sparsity* presets: dense_ratio 0.5/0.3/0.2/0.1/0.05
# = "50/70/80/90/95 sps", itersnip_iteration 1/20/50/100), 64 ABCD-shape clients on the HIP executor.
#   scripts/sailentgrads_sweep.sh [NGPUS] [extra flags...]
set -euo pipefail
NGPU=${1:-8}; [[ $# -gt 0 ]] && shift
DIR=$(cd "$(dirname "$0")" && pwd)
for DR in 0.5 0.3 0.2 0.1 0.05; do
  for IT in 1 20 50 100; do
    "$DIR/run.sh" sailentgrads "$NGPU" --engine hip --client_num_in_total 64 --frac 1 --comm_round 200 \
        --batch_size 16 --lr 0.01 --epochs 2 --dense_ratio "$DR" --itersnip_iteration "$IT" \
        --partition_method dir --partition_alpha 0.3 --seed 2022 "$@"
  done
done
