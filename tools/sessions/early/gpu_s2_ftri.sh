#!/bin/bash
# A/B: union-staged forward/dgrad (k_conv_fwd_tri, default) vs per-tap LDS-DMA (NIDT_FWD_TRI=0) at 64 / 8 clients,
# numerics first, then the 1-GPU bench
set -o pipefail
mkdir -p gpurun_out/ftri2
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "conv3d or alexnet or graph" > gpurun_out/ftri2/pytest.txt 2>&1 || { tail -30 gpurun_out/ftri2/pytest.txt; exit 1; }
tail -1 gpurun_out/ftri2/pytest.txt
for G in 64 8; do
  timeout -k 10 150 python tools/kbench.py $G 10 > gpurun_out/ftri2/kb${G}_tri.txt 2>&1 || exit 1
done
NIDT_FWD_TRI=0 timeout -k 10 150 python tools/kbench.py 64 10 > gpurun_out/ftri2/kb64_dma.txt 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/ftri2/bench.txt 2>&1 || exit 1
grep -H "_fwd\|_dgrad\|full train\|eval" gpurun_out/ftri2/kb*.txt | grep -v conv1_w | cut -c1-180; grep '^{' gpurun_out/ftri2/bench.txt | cut -c1-200
