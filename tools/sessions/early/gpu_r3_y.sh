#!/bin/bash
# full GPU suite + smoke + headline bench + a rocprofv3 kernel timeline of bench rounds (slab forward kernels)
set -o pipefail
mkdir -p gpurun_out/r3y
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
  > gpurun_out/r3y/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r3y/pytest_gpu.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r3y/pytest_gpu.txt | tail -2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3y/smoke.txt 2>&1 || { tail -20 gpurun_out/r3y/smoke.txt; exit 1; }
tail -1 gpurun_out/r3y/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3y/bench.txt 2>&1 || { tail -20 gpurun_out/r3y/bench.txt; exit 1; }
grep '^{' gpurun_out/r3y/bench.txt | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/profy -o run -- python3 -u bench.py --steps 2 --warmup 1 \
  > gpurun_out/r3y/prof.txt 2>&1 || { tail -20 gpurun_out/r3y/prof.txt; exit 1; }
db=$(find /tmp/profy -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/prof_summary.py "$db" gpurun_out/r3y/round_kernels.txt --top 40 > /dev/null 2>&1
head -16 gpurun_out/r3y/round_kernels.txt; grep -E "TOTAL|TIMELINE" gpurun_out/r3y/round_kernels.txt
