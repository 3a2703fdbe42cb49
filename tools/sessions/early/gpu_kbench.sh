#!/bin/bash
# Per-kernel microbench at G=64 and G=8, then the steady-state eager reference baseline (fp32 and bf16 autocast).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/kbench.py 64 10 > gpurun_out/kbench64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/kbench.py 8 10 > gpurun_out/kbench8.txt 2>&1 || exit $?
timeout -k 10 400 python tools/eager_baseline.py --rounds 3 > gpurun_out/eager_fp32_steady.txt 2>&1 || exit $?
timeout -k 10 400 python tools/eager_baseline.py --rounds 3 --dtype bf16 > gpurun_out/eager_bf16_steady.txt 2>&1 || exit $?
