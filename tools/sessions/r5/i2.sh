#!/bin/bash
# branch stream also takes GN parameter sums and the dgrad-image transposes: resnet2d GPU tests + CIFAR benches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5i2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py > $OUT/pytest.txt 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" $OUT/pytest.txt | tail -20; exit 1; }
tail -1 $OUT/pytest.txt
for cfg in "cifar10 subavg" "cifar10 dispfl" "tiny subavg"; do
  set -- $cfg
  timeout -k 10 400 python -u tools/bench_cifar.py --dataset $1 --algorithm $2 --rounds 2 --warmup 1 > $OUT/$1_$2.txt 2>&1 || { tail -20 $OUT/$1_$2.txt; exit 1; }
  echo "== $1 $2 $(tail -1 $OUT/$1_$2.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d.get("last_round_metrics"))')"
done
NIDT_WGRAD_STREAM=1 timeout -k 10 400 python -u tools/bench_cifar.py --dataset tiny --algorithm dispfl --rounds 2 --warmup 1 > $OUT/tiny_dispfl_forced.txt 2>&1 || { tail -20 $OUT/tiny_dispfl_forced.txt; exit 1; }
echo "== tiny dispfl forced-on $(tail -1 $OUT/tiny_dispfl_forced.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
