#!/bin/bash
# 3D ResNet-50 engine with sub-pixel stride-2 dgrad + batched packing: kernel tests, then config 5 at a realistic
# workload (256 clients x 36 train / 9 test volumes, batch 4, 1 epoch) with a rocprofv3 kernel timeline
set -o pipefail
mkdir -p gpurun_out/r3c
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_resnet3d.py tests/test_gpu_resnet2d.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r3c/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/r3c/pytest.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 1 \
  > gpurun_out/r3c/config5.txt 2>&1 || { tail -30 gpurun_out/r3c/config5.txt; exit 1; }
grep '^{' gpurun_out/r3c/config5.txt | cut -c1-600
f=$(find /tmp/c5prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/r3c/config5_kernel_stats.csv
db=$(find /tmp/c5prof -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/prof_summary.py "$db" gpurun_out/r3c/config5_kernels.txt --top 40 > /dev/null 2>&1
head -45 gpurun_out/r3c/config5_kernels.txt
