#!/bin/bash
# debug: eval-mode step dumps at both slot layouts, diffed on the box
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for T in 2 0; do
  NIDT_C1_TAPORD=$T timeout -k 10 200 python -u tools/debug/c1_evalmode2.py /tmp/dump_$T.pt 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 200 python -u tools/debug/c1_evalmode_cmp.py /tmp/dump_2.pt /tmp/dump_0.pt
