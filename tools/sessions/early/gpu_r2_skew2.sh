#!/bin/bash
# size-skew bench with two warmup rounds (eager + capture) so the timed rounds only replay graphs
set -o pipefail
mkdir -p gpurun_out/skew2
export PYTHONUNBUFFERED=1
for A in 0 1.0 0.3; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --size-skew $A > gpurun_out/skew2/skew_$A.txt 2>&1 || { tail -20 gpurun_out/skew2/skew_$A.txt; exit 1; }
  grep '^{' gpurun_out/skew2/skew_$A.txt | cut -c1-260
done
