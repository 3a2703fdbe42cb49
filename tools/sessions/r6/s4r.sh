#!/bin/bash
# [WG2-EARLY] default for <= 8 clients: runner / personalized tests, then 8 clients default vs NIDT_WG2_EARLY=0
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runner.py tests/test_gpu_personalized.py > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
tail -1 $OUT/t1.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
for rep in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export NIDT_WG2_EARLY=0; else unset NIDT_WG2_EARLY; fi
    timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/c8_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/c8_${arm}_$rep.txt; exit 1; }
    echo "== clients 8 rep $rep $arm $(tail -1 $OUT/c8_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
unset NIDT_WG2_EARLY
