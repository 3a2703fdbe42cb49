#!/bin/bash
# 3D ResNet-50 engine with the HIP stem (stem.hip): config 5 at a realistic
# workload (256 clients x 36 train / 9 test volumes, batch 4, 1 epoch) with a rocprofv3 kernel timeline
set -o pipefail
mkdir -p gpurun_out/r3g
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/c5profg -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 1 \
  > gpurun_out/r3g/config5.txt 2>&1 || { tail -30 gpurun_out/r3g/config5.txt; exit 1; }
grep '^{' gpurun_out/r3g/config5.txt | cut -c1-600
f=$(find /tmp/c5profg -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/r3g/config5_kernel_stats.csv
db=$(find /tmp/c5profg -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/prof_summary.py "$db" gpurun_out/r3g/config5_kernels.txt --top 40 > /dev/null 2>&1
head -45 gpurun_out/r3g/config5_kernels.txt
