#!/bin/bash
# ragged federations after the session-2 kernels: equal sizes vs Dirichlet size skew 1.0 / 0.3 (same total samples)
set -o pipefail
mkdir -p gpurun_out/skew2
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for skew in 0 1.0 0.3; do
  timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --size-skew $skew > gpurun_out/skew2/skew_$skew.txt 2>&1 || exit 1
  grep '^{' gpurun_out/skew2/skew_$skew.txt | cut -c1-200
done
