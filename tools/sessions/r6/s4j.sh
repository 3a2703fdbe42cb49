#!/bin/bash
# [ONEPASS] shifted sums (row_newbcast sample shift): large-mean statistics test on the unshifted build (build_ab/,
# informational) and the shifted build, conv tests, epilogue cost, then headline / 8 clients interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4j; mkdir -p $OUT
NIDT_EXT_DIR=build_ab timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k large_mean > $OUT/t_old.txt 2>&1
echo "unshifted build: $(tail -1 $OUT/t_old.txt)"; grep -m3 "assert _relerr\|AssertionError\|^E " $OUT/t_old.txt | head -6
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_batched2d.py tests/test_gpu_resnet2d.py tests/test_gpu_resnet3d.py > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
tail -1 $OUT/t1.txt
timeout -k 10 120 python3 -u tools/debug/slab_stats_cost.py > $OUT/cost.txt 2>&1 || { tail -20 $OUT/cost.txt; exit 1; }
grep -v amdgpu.ids $OUT/cost.txt
for rep in 1 2; do
  for arm in shift plain; do
    if [ $arm = plain ]; then export NIDT_EXT_DIR=build_ab; else unset NIDT_EXT_DIR; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/b_${arm}_$rep.txt; exit 1; }
    timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/b8_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/b8_${arm}_$rep.txt; exit 1; }
    echo "== $arm rep $rep: 64 clients $(tail -1 $OUT/b_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')  8 clients $(tail -1 $OUT/b8_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
unset NIDT_EXT_DIR
