#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
echo "bench rc=$?"
timeout -k 10 900 python -u -m pytest tests/test_gpu_personalized.py -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r2_pers.log 2>&1
echo "personalized rc=$?"
