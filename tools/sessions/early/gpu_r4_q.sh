#!/bin/bash
# three weight-tile stages in the 64-channel slab conv (NIDT_SLAB_NA=3): numerics under the switch, kbench A/B
# (conv2 data gradient), CIFAR SubAvg A/B
set -o pipefail
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4q; mkdir -p $OUT
NIDT_SLAB_NA=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "slab or alexnet" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
NIDT_SLAB_NA=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_resnet2d.py > $OUT/pytest_r2d.txt 2>&1 || { tail -30 $OUT/pytest_r2d.txt; exit 1; }
tail -1 $OUT/pytest_r2d.txt
kb() {  # name, env..., -- G
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python tools/kbench.py "$@" 10 > $OUT/kb_$name.txt 2>&1 || { tail -5 $OUT/kb_$name.txt; exit 1; }
  echo "$name: $(grep 'full train' $OUT/kb_$name.txt | head -1) | $(grep -E '^conv2_fwd|^conv2_dgrad' $OUT/kb_$name.txt | tr -s ' ' | tr '\n' ';')"
}
kb g64_na3 NIDT_SLAB_NA=3 -- 64
kb g64_na2 NIDT_SLAB_NA=2 -- 64
kb g64_na3b NIDT_SLAB_NA=3 -- 64
kb g64_na2b NIDT_SLAB_NA=2 -- 64
kb g8_na3 NIDT_SLAB_NA=3 -- 8
kb g8_na2 NIDT_SLAB_NA=2 -- 8
for arm in 3 2 3b 2b; do
  v=${arm%b}
  NIDT_SLAB_NA=$v timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 \
    > $OUT/subavg_na$arm.txt 2>&1 || { tail -5 $OUT/subavg_na$arm.txt; exit 1; }
  echo "subavg na=$arm: $(grep -o '"s_round_each": [^]]*]' $OUT/subavg_na$arm.txt)"
done
