#!/bin/bash
# full GPU suite, then ragged-size benches (same total samples)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r2_gpu_all.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
for skew in 1.0 0.3; do
  timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --size-skew $skew >> gpurun_out/r2_skew.jsonl 2>> gpurun_out/r2_skew.err
  rc=$?; echo "bench skew $skew rc=$rc"; if [ $rc -ne 0 ]; then break; fi
done
