#!/bin/bash
# GN register kernels + direct wgrad epilogue: full GPU suite, CIFAR profiles, A/B of the held-dy backward
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1 \
  || { grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.txt | tail -20; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/dprof -o run -- python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/dispfl_prof.txt 2>&1 || { tail -20 $OUT/dispfl_prof.txt; exit 1; }
db=$(find /tmp/dprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/dispfl_kernels.txt --top 40 --window-ms 3500 > /dev/null 2>&1
head -24 $OUT/dispfl_kernels.txt | cut -c1-150; grep -E "TOTAL|TIMELINE" $OUT/dispfl_kernels.txt
for H in 4 8; do
  NIDT_GN_HOLD=$H timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 2 --warmup 1 > $OUT/dispfl_h$H.txt 2>&1 || { tail -20 $OUT/dispfl_h$H.txt; exit 1; }
  echo "== HOLD=$H"; tail -1 $OUT/dispfl_h$H.txt | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg.txt 2>&1 || { tail -20 $OUT/subavg.txt; exit 1; }
tail -1 $OUT/subavg.txt | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt | cut -c1-200
