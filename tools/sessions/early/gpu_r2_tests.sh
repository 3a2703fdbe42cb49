#!/bin/bash
# round-2 GPU check: new personalized-algorithm kernels/runners, then the existing kernel suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_personalized.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r2_pers.log 2>&1
rc=$?
echo "personalized rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r2_kernels.log 2>&1
echo "kernels rc=$?"
