#!/bin/bash
# GPU check: numerics tests, smoke, short bench.  Each GPU step has its own time limit; stop at a crash/timeout.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -m pytest tests/test_gpu_kernels.py -q -s -m gpu > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --phase-timers > gpurun_out/bench.txt 2>&1
