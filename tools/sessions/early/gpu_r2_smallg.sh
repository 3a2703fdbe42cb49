#!/bin/bash
# split-K default for one/two-client conv3-5 launches: numerics, kbench G=1/2/4/8/64, skew bench, headline bench
set -o pipefail
mkdir -p gpurun_out/sg
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "splitk or train_step or eval_matches" > gpurun_out/sg/pytest.txt 2>&1 || { tail -30 gpurun_out/sg/pytest.txt; exit 1; }
tail -1 gpurun_out/sg/pytest.txt
for G in 1 2 4 8 64; do
  timeout -k 10 200 python -u tools/kbench.py $G 20 > gpurun_out/sg/kb$G.txt 2>&1 || exit 1
  grep -E "step" gpurun_out/sg/kb$G.txt
done
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --size-skew 1.0 > gpurun_out/sg/skew1.txt 2>&1 || exit 1
grep '^{' gpurun_out/sg/skew1.txt | cut -c90-220
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/sg/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/sg/bench.txt | cut -c1-220
