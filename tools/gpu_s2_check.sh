#!/bin/bash
# state check after a rebuild: whole GPU suite, smoke(), the driver's 1-GPU bench line, kbench at 64 clients
set -o pipefail
mkdir -p gpurun_out/s2
export PYTHONUNBUFFERED=1
timeout -k 10 840 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/s2/pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/s2/pytest.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/s2/smoke.txt
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/s2/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/s2/bench.txt | cut -c1-300
timeout -k 10 120 python tools/kbench.py 64 10 > gpurun_out/s2/kbench64.txt 2>&1 || exit 1
