#!/bin/bash
# fused optimizer + pack: GPU tests, then CIFAR benches with and without it
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5d2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py tests/test_gpu_batched2d.py > $OUT/pytest.txt 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" $OUT/pytest.txt | tail -20; exit 1; }
tail -1 $OUT/pytest.txt
for alg in dispfl subavg; do
  for V in 0 1; do
    NIDT_PACK_FUSE=$V timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $alg --rounds 2 --warmup 1 > $OUT/${alg}_$V.txt 2>&1 || { tail -20 $OUT/${alg}_$V.txt; exit 1; }
    echo "== $alg PACK_FUSE=$V $(tail -1 $OUT/${alg}_$V.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"], d.get("last_round_metrics"))')"
  done
done
