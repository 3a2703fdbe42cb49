#!/bin/bash
# CIFAR SubAvg: host-side time per step phase; step timeline without the wgrad side stream
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3c; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/debug/step_host_times.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/host_times.txt 2>&1 || { tail -20 $OUT/host_times.txt; exit 1; }
grep "^host" $OUT/host_times.txt
NIDT_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cfn -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/nows_prof.txt 2>&1 || { tail -20 $OUT/nows_prof.txt; exit 1; }
db=$(find /tmp/cfn -name "*.db" | head -1)
python3 tools/step_timeline.py "$db" $OUT/nows_step.txt && tail -3 $OUT/nows_step.txt
