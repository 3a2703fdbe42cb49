#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
true
echo "kernels rc=$?"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_convergence.py -v -s --timeout 900 --timeout-method thread > gpurun_out/r2_conv.log 2>&1
echo "convergence rc=$?"
