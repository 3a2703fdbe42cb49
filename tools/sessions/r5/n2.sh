#!/bin/bash
# end-of-session check: full GPU suite, smoke, headline + 8-client benches, config 5, CIFAR SubAvg / DisPFL
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5n3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.txt 2>&1 \
  || { grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.txt | tail -20; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python -u bench.py > $OUT/bench_default.txt 2>&1 || { tail -20 $OUT/bench_default.txt; exit 1; }
tail -1 $OUT/bench_default.txt | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench64.txt 2>&1 || { tail -20 $OUT/bench64.txt; exit 1; }
tail -1 $OUT/bench64.txt | cut -c1-300
timeout -k 10 300 python -u bench.py --clients 8 --steps 30 --warmup 5 > $OUT/bench8.txt 2>&1 || { tail -20 $OUT/bench8.txt; exit 1; }
tail -1 $OUT/bench8.txt | cut -c1-300
timeout -k 10 500 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5.txt 2>&1 || { tail -20 $OUT/c5.txt; exit 1; }
grep -E '^round' $OUT/c5.txt
for alg in subavg dispfl; do
  timeout -k 10 300 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/$alg.txt 2>&1 || { tail -20 $OUT/$alg.txt; exit 1; }
  tail -1 $OUT/$alg.txt | cut -c1-220
done
