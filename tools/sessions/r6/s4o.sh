#!/bin/bash
# [EAGER-BRANCH] default (eager steps + wgrad branch for <= 32 clients) vs NIDT_AX_EAGER_MAXG=0 (captured everywhere,
# the previous default): runner / personalized / CLI tests, then 8 / 16 / 32 / 64 clients interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4o; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_runner.py tests/test_gpu_personalized.py tests/test_gpu_cli.py tests/test_gpu_compat_api.py tests/test_gpu_convergence.py > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
tail -1 $OUT/t1.txt
for c in 8 16 32 64; do
  for rep in 1 2; do
    for arm in new old; do
      if [ $arm = old ]; then export NIDT_AX_EAGER_MAXG=0; else unset NIDT_AX_EAGER_MAXG; fi
      timeout -k 10 300 python -u bench.py --clients $c --steps 10 --warmup 3 > $OUT/c${c}_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/c${c}_${arm}_$rep.txt; exit 1; }
      echo "== clients $c rep $rep $arm $(tail -1 $OUT/c${c}_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
unset NIDT_AX_EAGER_MAXG
