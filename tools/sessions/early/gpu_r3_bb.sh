#!/bin/bash
# final verification of the tree: full GPU suite, smoke, headline bench at the driver's shape
set -o pipefail
mkdir -p gpurun_out/r3bb
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r3bb/pytest_gpu.txt 2>&1
rc=$?; tail -1 gpurun_out/r3bb/pytest_gpu.txt; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r3bb/pytest_gpu.txt | head -20; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3bb/smoke.txt 2>&1 || { tail -20 gpurun_out/r3bb/smoke.txt; exit 1; }
echo "smoke ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3bb/bench.txt 2>&1 || { tail -20 gpurun_out/r3bb/bench.txt; exit 1; }
tail -1 gpurun_out/r3bb/bench.txt | cut -c1-200
