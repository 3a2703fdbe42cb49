#!/bin/bash
# GroupNorm HBM counters (FETCH_SIZE / WRITE_SIZE in separate passes: TCC counter limit), gn kernels only
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5t2; mkdir -p $OUT
RE='k_gn_'
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "$RE" --output-format csv \
      -d /tmp/gpmc/p$i -o run -- python3 tools/bench_gn.py > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py /tmp/gpmc $OUT/pmc_summary.txt > /dev/null 2>&1 || true
cat $OUT/pmc_summary.txt | cut -c1-200
