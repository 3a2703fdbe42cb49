#!/bin/bash
# [GN-EPI]: 2-D ResNet GPU tests, then CIFAR SubAvg / DisPFL with GroupNorm statistics from the slab conv epilogue
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3u; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resnet2d.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for alg in subavg dispfl; do
  for f in 1 0; do
    NIDT_GN_EPI=$f timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/${alg}_$f.txt 2>&1 || { tail -20 $OUT/${alg}_$f.txt; exit 1; }
    echo "== $alg gn_epi=$f $(tail -1 $OUT/${alg}_$f.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
  done
done
