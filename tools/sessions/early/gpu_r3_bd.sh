#!/bin/bash
# short verification of the final tree: runner / personalized / CLI GPU tests (the evaluation path changed), smoke, bench
set -o pipefail
mkdir -p gpurun_out/r3bd
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_personalized.py tests/test_gpu_cli.py -x -v -s \
  --timeout 300 --timeout-method thread > gpurun_out/r3bd/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3bd/pytest.txt; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r3bd/pytest.txt | head -20; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3bd/smoke.txt 2>&1 || { tail -20 gpurun_out/r3bd/smoke.txt; exit 1; }
echo "smoke ok"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3bd/bench.txt 2>&1 || { tail -20 gpurun_out/r3bd/bench.txt; exit 1; }
tail -1 gpurun_out/r3bd/bench.txt | cut -c1-200
