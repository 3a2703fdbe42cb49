#!/bin/bash
# A/B: conv1 fused forward B-fragment prefetch distance 1 (round-2 kernel) / 2 (default) / 3; numerics first.
set -o pipefail
mkdir -p gpurun_out/c1pf
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "conv1 or alexnet" > gpurun_out/c1pf/pytest.txt 2>&1 || { tail -30 gpurun_out/c1pf/pytest.txt; exit 1; }
tail -1 gpurun_out/c1pf/pytest.txt
for PF in 2 1 3; do
  NIDT_C1_PF=$PF timeout -k 10 150 python tools/kbench.py 64 10 > gpurun_out/c1pf/kb64_pf$PF.txt 2>&1 || exit 1
done
grep -H "conv1_fwd\|full train\|eval forward" gpurun_out/c1pf/kb64_pf*.txt | cut -c1-200
