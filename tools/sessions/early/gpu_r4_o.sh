#!/bin/bash
# output-space union swizzle in the slab conv (NIDT_SLAB_LSWZ): numerics of the slab kernels, then interleaved A/B
# of the AlexNet conv2 forward / data gradient (kbench G=64 and G=8) and a CIFAR SubAvg round (2-D slab convs)
set -o pipefail
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4o; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "slab or alexnet" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py \
  > $OUT/pytest_r2d.txt 2>&1 || { tail -30 $OUT/pytest_r2d.txt; exit 1; }
tail -1 $OUT/pytest_r2d.txt
kb() {  # name, env..., -- G
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python tools/kbench.py "$@" 10 > $OUT/kb_$name.txt 2>&1 || { tail -5 $OUT/kb_$name.txt; exit 1; }
  echo "$name: $(grep 'full train' $OUT/kb_$name.txt | head -1) | $(grep -E '^conv2_fwd|^conv2_dgrad' $OUT/kb_$name.txt | tr -s ' ' | tr '\n' ';')"
}
kb g64_l1 X=1 -- 64
kb g64_l0 NIDT_SLAB_LSWZ=0 -- 64
kb g64_l1b X=1 -- 64
kb g64_l0b NIDT_SLAB_LSWZ=0 -- 64
kb g8_l1 X=1 -- 8
kb g8_l0 NIDT_SLAB_LSWZ=0 -- 8
for arm in 1 0 1b 0b; do
  v=${arm%b}
  NIDT_SLAB_LSWZ=$v timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 \
    > $OUT/subavg_l$arm.txt 2>&1 || { tail -5 $OUT/subavg_l$arm.txt; exit 1; }
  echo "subavg lswz=$arm: $(grep -o '"s_round_each": [^]]*]' $OUT/subavg_l$arm.txt)"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $OUT/bench.json 2>&1 || exit 1
echo "bench 64 clients: $(grep -o '"value": [0-9.]*' $OUT/bench.json)"
