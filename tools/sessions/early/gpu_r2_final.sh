#!/bin/bash
# round-end rehearsal: whole GPU suite, smoke(), the driver's 1-GPU bench line
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 1300 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/final/pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/final/pytest.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/final/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/final/bench.txt | cut -c1-300
