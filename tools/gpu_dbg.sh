#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/dbg_conv_explore.py > gpurun_out/dbg.log 2>&1
echo "rc=$?"
