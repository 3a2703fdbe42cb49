#!/bin/bash
# [STEM-FOLD] per-buffer folded image (first-in-process DisPFL graphs-vs-eager test), then [DPP-SUM] A/B: the
# statistics epilogue's row sums with DPP (default build) vs __shfl_xor (build_ab/, NIDT_EXT_DIR) on the headline
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s4a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_resnet2d.py -k graphs_match_eager > $OUT/t1.txt 2>&1 || { tail -30 $OUT/t1.txt; exit 1; }
tail -1 $OUT/t1.txt
for rep in 1 2; do
  for arm in dpp shfl; do
    if [ $arm = shfl ]; then export NIDT_EXT_DIR=build_ab; else unset NIDT_EXT_DIR; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/b_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/b_${arm}_$rep.txt; exit 1; }
    timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/b8_${arm}_$rep.txt 2>&1 || { tail -20 $OUT/b8_${arm}_$rep.txt; exit 1; }
    echo "== $arm rep $rep: 64 clients $(tail -1 $OUT/b_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')  8 clients $(tail -1 $OUT/b8_${arm}_$rep.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
unset NIDT_EXT_DIR
