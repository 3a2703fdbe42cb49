#!/bin/bash
# validation after the evaluation change: full GPU suite with durations, the headline bench (twice), the 8-client
# round, CIFAR SubAvg / DisPFL and Tiny rounds
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4v; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --durations=40 \
  > $OUT/pytest_gpu.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20; exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench$i.json 2>&1 || exit 1
  echo "bench 64 clients: $(grep -o '"value": [0-9.]*' $OUT/bench$i.json)"
done
timeout -k 10 300 python bench.py --clients 8 --steps 20 --warmup 3 > $OUT/bench_c8.json 2>&1 || exit 1
echo "bench 8 clients: $(grep -o '"value": [0-9.]*' $OUT/bench_c8.json)"
for spec in "subavg --rounds 3 --warmup 1" "dispfl --rounds 1 --warmup 1" "subavg --dataset tiny --batch 128 --rounds 2 --warmup 1"; do
  name=$(echo $spec | tr -d ' -' | cut -c1-24)
  timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $spec > $OUT/$name.txt 2>&1 || exit 1
  echo "$spec: $(grep -o '"s_round_each": [^]]*]' $OUT/$name.txt)"
done
