#!/bin/bash
# evaluation forms at the headline config: one launch sequence over a 2C-row copy (NIDT_EVAL_STAGE=1) vs personal
# rows in place + reused global copies (=0), interleaved; then the runner GPU tests
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4w; mkdir -p $OUT
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_EVAL_STAGE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_s$arm.json 2>&1 || exit 1
  echo "stage=$arm: $(grep -o '"value": [0-9.]*' $OUT/bench_s$arm.json)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2>&1 || exit 1
echo "default: $(grep -o '"value": [0-9.]*' $OUT/bench_default.json)"
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_runner.py \
  tests/test_gpu_convergence.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
grep -E "passed|failed" $OUT/pytest.txt | tail -1
