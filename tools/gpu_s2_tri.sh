#!/bin/bash
# conv2 wgrad with three-tap union staging (k_conv_wgrad_tri): numerics, kbench at 64 / 8 clients, 1-GPU bench
set -o pipefail
mkdir -p gpurun_out/tri3
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "conv3d or alexnet or graph" > gpurun_out/tri3/pytest.txt 2>&1 || { tail -30 gpurun_out/tri3/pytest.txt; exit 1; }
tail -1 gpurun_out/tri3/pytest.txt
for G in 64 8; do
  timeout -k 10 150 python tools/kbench.py $G 10 > gpurun_out/tri3/kb${G}.txt 2>&1 || exit 1
done
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/tri3/bench.txt 2>&1 || exit 1
grep -H "conv2_wgrad\|full train" gpurun_out/tri3/kb*.txt; grep '^{' gpurun_out/tri3/bench.txt | cut -c1-220
