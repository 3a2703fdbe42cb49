#!/bin/bash
# concurrent ragged launches per lockstep step: graphs(+side streams) == eager bit for bit; size-skew bench A/B
set -o pipefail
mkdir -p gpurun_out/st
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_personalized.py -k "bit_identical" > gpurun_out/st/pytest.txt 2>&1 || { tail -30 gpurun_out/st/pytest.txt; exit 1; }
tail -1 gpurun_out/st/pytest.txt
for A in 1.0 0.3; do
  for S in 4 1; do
    timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --size-skew $A --step-streams $S > gpurun_out/st/skew_${A}_s$S.txt 2>&1 || { tail -20 gpurun_out/st/skew_${A}_s$S.txt; exit 1; }
    echo "skew $A streams $S: $(grep '^{' gpurun_out/st/skew_${A}_s$S.txt | cut -c90-220)"
  done
done
