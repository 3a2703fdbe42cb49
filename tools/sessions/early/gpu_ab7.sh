#!/bin/bash
# Wgrad split factor A/B at 64 clients: forced 2 / 3 for every layer vs the cost model (read the conv3-5 rows).
set -o pipefail
mkdir -p gpurun_out/ab7
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 64 8 > gpurun_out/ab7/kbench64_def.txt 2>&1 || exit $?
NIDT_WG_NSPLIT_FORCE=2 KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 64 8 > gpurun_out/ab7/kbench64_ns2.txt 2>&1 || exit $?
NIDT_WG_NSPLIT_FORCE=3 KBENCH_EVAL=0 timeout -k 10 200 python tools/kbench.py 64 8 > gpurun_out/ab7/kbench64_ns3.txt 2>&1 || exit $?
