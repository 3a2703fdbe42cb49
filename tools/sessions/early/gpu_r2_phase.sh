#!/bin/bash
# synchronised phase split (train / aggregate / eval) of the equal-size and size-skewed headline rounds
set -o pipefail
mkdir -p gpurun_out/ph
export PYTHONUNBUFFERED=1
for A in 1.0 0; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --size-skew $A --phase-timers > gpurun_out/ph/skew_$A.txt 2>&1 || { tail -20 gpurun_out/ph/skew_$A.txt; exit 1; }
  grep '^{' gpurun_out/ph/skew_$A.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skew', '$A', d['ms_per_step'], d.get('phase_s'))"
done
