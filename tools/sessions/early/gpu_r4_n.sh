#!/bin/bash
# full GPU suite with per-test durations (budget audit, graph reuse across client groups, batched 2-D engine,
# row counter), then SubAvg / Tiny round times with graphs on (reused across rounds) vs off, and the benches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4n; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --durations=70 \
  > $OUT/pytest_gpu.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -2
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20; exit $rc; fi
run() {  # name, env..., -- args
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u tools/bench_cifar.py "$@" > $OUT/$name.txt 2>&1 || { tail -5 $OUT/$name.txt; exit 1; }
  echo "$name: $(grep -o '"s_round_each": [^]]*]' $OUT/$name.txt) $(grep -o '"graph_stats": {[^}]*}' $OUT/$name.txt)"
}
S="--algorithm subavg --rounds 3 --warmup 1"
T="--algorithm subavg --dataset tiny --batch 128 --rounds 2 --warmup 1"
run subavg_g1 X=1 -- $S
run subavg_g0 NIDT_HIP_GRAPHS=0 -- $S
run subavg_g1b X=1 -- $S
run tiny_g1 X=1 -- $T
run tiny_g0 NIDT_HIP_GRAPHS=0 -- $T
run dispfl_g1 X=1 -- --algorithm dispfl --rounds 1 --warmup 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.json 2>&1 || exit 1
echo "bench 64 clients: $(grep -o '"value": [0-9.]*' $OUT/bench.json)"
timeout -k 10 300 python bench.py --clients 8 --steps 20 --warmup 3 > $OUT/bench_c8.json 2>&1 || exit 1
echo "bench 8 clients: $(grep -o '"value": [0-9.]*' $OUT/bench_c8.json)"
