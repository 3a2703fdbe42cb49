#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k2; mkdir -p $OUT
NIDT_CIFAR_EVAL_PROBE=1 timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/probe.txt 2>&1 || { tail -20 $OUT/probe.txt; exit 1; }
grep -E "probe|^round" $OUT/probe.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/sprof -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/subavg_prof.txt 2>&1 || { tail -20 $OUT/subavg_prof.txt; exit 1; }
db=$(find /tmp/sprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/subavg_kernels.txt --top 45 --window-ms 715 > /dev/null 2>&1
head -40 $OUT/subavg_kernels.txt | cut -c1-150; grep -E "TOTAL|TIMELINE" $OUT/subavg_kernels.txt
