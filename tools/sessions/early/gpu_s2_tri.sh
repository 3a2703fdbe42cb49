#!/bin/bash
# three-tap union wgrad (64-channel blocks, occupancy-aware split model): numerics, kbench A/B vs the 4-tap kernel
# (NIDT_WG_TRI=0) at 64 and 8 clients, 1-GPU bench
set -o pipefail
mkdir -p gpurun_out/tri6
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "wgrad or alexnet or graph" > gpurun_out/tri6/pytest.txt 2>&1 || { tail -30 gpurun_out/tri6/pytest.txt; exit 1; }
tail -1 gpurun_out/tri6/pytest.txt
for G in 64 8; do
  KBENCH_EVAL=0 timeout -k 10 150 python tools/kbench.py $G 10 > gpurun_out/tri6/kb${G}_tri.txt 2>&1 || exit 1
  KBENCH_EVAL=0 NIDT_WG_TRI=0 timeout -k 10 150 python tools/kbench.py $G 10 > gpurun_out/tri6/kb${G}_dma.txt 2>&1 || exit 1
done
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/tri6/bench.txt 2>&1 || exit 1
grep -H "wgrad\|full train" gpurun_out/tri6/kb*.txt | grep -v conv1; grep '^{' gpurun_out/tri6/bench.txt | cut -c1-200
