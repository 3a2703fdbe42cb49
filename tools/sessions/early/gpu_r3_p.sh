#!/bin/bash
# BN apply / backward-apply with loop-invariant channel coefficients: 3D ResNet tests + config 5 timeline;
# personalized-runner tests incl. the masked neighbour mean
set -o pipefail
mkdir -p gpurun_out/r3p
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet3d.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3p/pytest3d.txt 2>&1 || { tail -30 gpurun_out/r3p/pytest3d.txt; exit 1; }
tail -1 gpurun_out/r3p/pytest3d.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_personalized.py -x -q --timeout 200 --timeout-method thread \
  -k "masked_mean or dispfl_fire" > gpurun_out/r3p/pytest_pers.txt 2>&1 || { tail -30 gpurun_out/r3p/pytest_pers.txt; exit 1; }
tail -1 gpurun_out/r3p/pytest_pers.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/c5profp -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 1 \
  > gpurun_out/r3p/config5.txt 2>&1 || { tail -30 gpurun_out/r3p/config5.txt; exit 1; }
grep '^{' gpurun_out/r3p/config5.txt | cut -c1-330
db=$(find /tmp/c5profp -name "*.db" | head -1)
[ -n "$db" ] && python3 tools/prof_summary.py "$db" gpurun_out/r3p/config5_kernels.txt --top 40 > /dev/null 2>&1
head -16 gpurun_out/r3p/config5_kernels.txt; grep -E "TOTAL|TIMELINE" gpurun_out/r3p/config5_kernels.txt
