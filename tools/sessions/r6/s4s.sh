#!/bin/bash
# full GPU suite + smoke + default bench on the current tree
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4s; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_all.txt 2>&1 || { tail -40 $OUT/gpu_all.txt; exit 1; }
tail -2 $OUT/gpu_all.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt | cut -c1-400
for alg in subavg dispfl; do
  timeout -k 10 400 python -u tools/bench_cifar.py --algorithm $alg --rounds 3 --warmup 1 > $OUT/${alg}.txt 2>&1 || { tail -20 $OUT/${alg}.txt; exit 1; }
  echo "== $alg $(tail -1 $OUT/${alg}.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["s_round_each"])')"
done
timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/bench8.txt 2>&1 || { tail -20 $OUT/bench8.txt; exit 1; }
echo "== bench c8 $(tail -1 $OUT/bench8.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
