#!/bin/bash
# kernel change check: conv numerics tests, kbench G=64 and G=8, 1-GPU headline bench
set -o pipefail
mkdir -p gpurun_out/kb
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 tests/test_gpu_kernels.py -k "wgrad or train_step or fwd_stats" > gpurun_out/kb/pytest.txt 2>&1 || { tail -20 gpurun_out/kb/pytest.txt; exit 1; }
tail -1 gpurun_out/kb/pytest.txt
timeout -k 10 200 python -u tools/kbench.py 64 10 > gpurun_out/kb/kb64.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench.py 8 20 > gpurun_out/kb/kb8.txt 2>&1 || exit 1
grep -E "step|wgrad" gpurun_out/kb/kb64.txt gpurun_out/kb/kb8.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/kb/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/kb/bench.txt | cut -c1-200
