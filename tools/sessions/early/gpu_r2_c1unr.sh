#!/bin/bash
# A/B of the conv1 sparse wgrad cell-loop unroll (NIDT_C1WG_UNROLL = 1 / 2 / 4): numerics with 2, kbench G=64 and 8
set -o pipefail
mkdir -p gpurun_out/c1u
export PYTHONUNBUFFERED=1
NIDT_C1WG_UNROLL=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv1" > gpurun_out/c1u/pytest.txt 2>&1 || { tail -30 gpurun_out/c1u/pytest.txt; exit 1; }
tail -1 gpurun_out/c1u/pytest.txt
for U in 1 2 4; do
  for G in 64 8; do
    NIDT_C1WG_UNROLL=$U timeout -k 10 200 python -u tools/kbench.py $G 10 > gpurun_out/c1u/kb_u${U}_g$G.txt 2>&1 || exit 1
    echo "unroll $U G=$G: $(grep -E 'conv1_wgrad' gpurun_out/c1u/kb_u${U}_g$G.txt)"
  done
done
