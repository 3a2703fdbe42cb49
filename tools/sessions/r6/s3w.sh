#!/bin/bash
# cost of the conv statistics epilogue (k_conv_fwd_slab with / without STATS)
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3w; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/debug/slab_stats_cost.py > $OUT/cost.txt 2>&1 || { tail -20 $OUT/cost.txt; exit 1; }
cat $OUT/cost.txt | grep -v amdgpu.ids
