#!/bin/bash
# conv1 sparse wgrad change: numerics (fused fwd + sparse wgrad, full train step), kbench G=64 / G=8, headline bench
set -o pipefail
mkdir -p gpurun_out/c1
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv1 or train_step" > gpurun_out/c1/pytest.txt 2>&1 || { tail -30 gpurun_out/c1/pytest.txt; exit 1; }
tail -1 gpurun_out/c1/pytest.txt
timeout -k 10 200 python -u tools/kbench.py 64 10 > gpurun_out/c1/kb64.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/kbench.py 8 20 > gpurun_out/c1/kb8.txt 2>&1 || exit 1
grep -E "step|conv1" gpurun_out/c1/kb64.txt gpurun_out/c1/kb8.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/c1/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/c1/bench.txt | cut -c1-200
