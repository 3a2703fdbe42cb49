#!/bin/bash
# Iteration loop on the GPU box: numerics tests -> bench -> rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python -m pytest tests/test_gpu_kernels.py -q -s -m gpu > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.txt 2>&1 || exit $?
rm -rf gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_bench.txt 2>&1
