#!/bin/bash
# gemm1x1.hip: correctness (all tile configs, > 2^31-element operand, the engine's conv tests), per-shape timing vs the
# general conv kernel, then config 5 end to end with and without it
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py -k "gemm1x1 or gconv3 or lockstep or packer" > $OUT/t.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/t.txt | tail -30; exit 1; }
grep -E "passed|failed" $OUT/t.txt | tail -1
timeout -k 10 300 python -u tools/bench_gemm1x1.py > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
cat $OUT/bench.txt | grep -v amdgpu.ids
for V in 1 0; do
  NIDT_R3D_G1=$V timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5_$V.txt 2>&1 || { tail -20 $OUT/c5_$V.txt; exit 1; }
  echo "== NIDT_R3D_G1=$V"; grep -E '^round' $OUT/c5_$V.txt; grep '^{' $OUT/c5_$V.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steady', d['steady_s_per_round'], d['metrics'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_resnet2d.py -k "alexnet or resnet or conv" > $OUT/t2.txt 2>&1 || { grep -E "FAIL|Error|assert" $OUT/t2.txt | tail -30; exit 1; }
tail -1 $OUT/t2.txt
timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64.txt 2>&1 || exit 1
grep "full train step" $OUT/kb64.txt
