#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5u; mkdir -p $OUT
NIDT_CIFAR_EVAL_PROBE=1 timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/probe.txt 2>&1 || { tail -20 $OUT/probe.txt; exit 1; }
grep -E "probe|^round" $OUT/probe.txt
NIDT_CIFAR_EVAL_PROBE=exit timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/eprof -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 1 --warmup 1 > $OUT/probe_prof.txt 2>&1 || { tail -20 $OUT/probe_prof.txt; exit 1; }
db=$(find /tmp/eprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/eval_kernels.txt --top 30 --window-ms 230 > /dev/null 2>&1
head -24 $OUT/eval_kernels.txt | cut -c1-140; grep -E "TIMELINE|GAP" $OUT/eval_kernels.txt | head -5
