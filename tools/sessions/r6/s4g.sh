#!/bin/bash
# [COEF1] clip coefficient once per client row (k_opt_coef) vs per step block (build_ab/, NIDT_EXT_DIR): optimizer
# tests, then CIFAR DisPFL / SubAvg and the 64-client headline interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_personalized.py tests/test_gpu_resnet2d.py > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
tail -1 $OUT/t1.txt
for rep in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export NIDT_EXT_DIR=build_ab; else unset NIDT_EXT_DIR; fi
    timeout -k 10 400 python -u tools/bench_cifar.py --algorithm dispfl --rounds 3 --warmup 1 > $OUT/d_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/d_${arm}_$rep.txt; exit 1; }
    timeout -k 10 400 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/s_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/s_${arm}_$rep.txt; exit 1; }
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/b_${arm}_$rep.txt; exit 1; }
    v() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])'; }
    echo "== $arm rep $rep: dispfl $(v $OUT/d_${arm}_$rep.txt)  subavg $(v $OUT/s_${arm}_$rep.txt)  64 clients $(v $OUT/b_${arm}_$rep.txt)"
  done
done
unset NIDT_EXT_DIR
