#!/bin/bash
# New defaults (conv1 forward original tap order; 3-wave conv2 wgrad split at small groups): conv1/AlexNet numerics,
# kbench G=8 / G=64, 8-client round kernel timeline, headline bench; then the Tiny / SubAvg regression switches
# (tools/sessions/early/gpu_r3_bc.sh)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4m; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "conv1 or alexnet or wgrad" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for g in 8 64; do
  timeout -k 10 200 python tools/kbench.py $g 10 > $OUT/kb_g$g.txt 2>&1 || { tail -5 $OUT/kb_g$g.txt; exit 1; }
  grep 'full train' $OUT/kb_g$g.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c8prof -o run -- python3 bench.py --clients 8 --steps 20 \
  --warmup 3 > $OUT/bench_c8.json 2>&1 || { tail -5 $OUT/bench_c8.json; exit 1; }
grep '^{' $OUT/bench_c8.json | cut -c1-200
db=$(find /tmp/c8prof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c8_round_kernels.txt --top 45 --window-ms 700 > /dev/null 2>&1
tail -3 $OUT/c8_round_kernels.txt
timeout -k 10 300 python bench.py --clients 8 --steps 10 --warmup 3 > $OUT/bench_c8_noprof.json 2>&1 || exit 1
echo "bench 8 clients: $(grep -o '"value": [0-9.]*' $OUT/bench_c8_noprof.json)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.json 2>&1 || exit 1
echo "bench 64 clients: $(grep -o '"value": [0-9.]*' $OUT/bench.json)"
bash tools/sessions/early/gpu_r3_bc.sh
