#!/bin/bash
# Headline benchmark at 1/2/4/8 GPUs of one node (strong scaling: the 64 clients are sharded over ranks).
# bench.py spawns its N ranks itself (one process per GPU, RCCL); TORCHRUN=1 launches them with torch.distributed.run
# instead -- both shapes report the same JSON line.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
STEPS=${STEPS:-5}; WARMUP=${WARMUP:-1}; GPUS=${GPUS:-"1 2 4 8"}
for N in $GPUS; do
  if [[ $N -eq 1 || "${TORCHRUN:-0}" != "1" ]]; then
    python "$ROOT/bench.py" --gpus "$N" --steps "$STEPS" --warmup "$WARMUP" "$@"
  else
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((29600 + N)) "$ROOT/bench.py" --gpus "$N" --steps "$STEPS" --warmup "$WARMUP" "$@"
  fi
done
