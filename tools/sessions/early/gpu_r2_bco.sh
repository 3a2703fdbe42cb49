#!/bin/bash
# A/B: 64-channel forward blocks (4 waves, 2 per CU) vs 128-channel (8 waves) for Cout = 128 layers (conv2/conv5 fwd,
# conv3 dgrad); kbench at G=64 / G=8 and the 1-GPU headline bench
set -o pipefail
mkdir -p gpurun_out/bco
export PYTHONUNBUFFERED=1
NIDT_FWD_BCO=64 timeout -k 10 200 python -u -m pytest -x -q --timeout 200 tests/test_gpu_kernels.py -k "fwd_stats or train_step" > gpurun_out/bco/pytest.txt 2>&1 || { tail -20 gpurun_out/bco/pytest.txt; exit 1; }
tail -1 gpurun_out/bco/pytest.txt
for G in 64 8; do
  timeout -k 10 200 python -u tools/kbench.py $G 10 > gpurun_out/bco/kb${G}_128.txt 2>&1 || exit 1
  NIDT_FWD_BCO=64 timeout -k 10 200 python -u tools/kbench.py $G 10 > gpurun_out/bco/kb${G}_64.txt 2>&1 || exit 1
  echo "== G=$G default (128-ch blocks) vs forced 64"; grep -E "step|fwd|dgrad" gpurun_out/bco/kb${G}_128.txt | head -12
  grep -E "step|fwd|dgrad" gpurun_out/bco/kb${G}_64.txt | head -12
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bco/bench_128.txt 2>&1 || exit 1
NIDT_FWD_BCO=64 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bco/bench_64.txt 2>&1 || exit 1
grep '^{' gpurun_out/bco/bench_128.txt | cut -c1-200; grep '^{' gpurun_out/bco/bench_64.txt | cut -c1-200
