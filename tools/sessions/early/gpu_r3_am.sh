#!/bin/bash
# the per-GPU load of the 8-GPU run (8 clients per GPU): kbench + bench at 8 clients + round timeline
set -o pipefail
mkdir -p gpurun_out/r3am
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/kbench.py 8 10 > gpurun_out/r3am/kbench8.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3am/kbench8.txt
timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > gpurun_out/r3am/bench8.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3am/bench8.txt | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profam -o run -- python3 -u bench.py --clients 8 --steps 3 --warmup 1 \
  > gpurun_out/r3am/prof.txt 2>&1 || exit 1
db=$(find /tmp/profam -name "*.db" | head -1)
python3 tools/prof_summary.py --top 40 --window-ms 75 "$db" > gpurun_out/r3am/round_kernels8.txt 2>&1
head -30 gpurun_out/r3am/round_kernels8.txt; grep -E "TOTAL|TIMELINE" gpurun_out/r3am/round_kernels8.txt
