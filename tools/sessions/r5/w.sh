#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5w; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batched2d.py tests/test_gpu_resnet2d.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg.txt 2>&1 || { tail -20 $OUT/subavg.txt; exit 1; }
tail -3 $OUT/subavg.txt
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm dispfl --rounds 3 --warmup 1 > $OUT/dispfl.txt 2>&1 || { tail -20 $OUT/dispfl.txt; exit 1; }
tail -3 $OUT/dispfl.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
tail -1 $OUT/bench.txt
timeout -k 10 400 python -u -m cProfile -o /tmp/sa.prof tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 --no-eval > $OUT/prun.txt 2>&1 || { tail -20 $OUT/prun.txt; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('/tmp/sa.prof')
p.sort_stats('tottime').print_stats(40)
" > $OUT/prof_tottime.txt 2>&1
python3 -c "
import pstats
p = pstats.Stats('/tmp/sa.prof')
p.sort_stats('cumulative').print_stats(70)
" > $OUT/prof_cum.txt 2>&1
grep -E "^round|rounds/s" $OUT/prun.txt | tail -3
