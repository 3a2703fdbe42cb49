#!/bin/bash
# depth-tap skipping in k_conv_fwd_dma: conv kernel tests + kbench at 64 clients + bench
set -o pipefail
mkdir -p gpurun_out/r3u
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resnet3d.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r3u/pytest.txt 2>&1
rc=$?; tail -2 gpurun_out/r3u/pytest.txt; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3u/kbench.txt 2>&1 || exit 1
cat gpurun_out/r3u/kbench.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r3u/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/r3u/bench.txt | cut -c1-200
