#!/bin/bash
# debug: conv1 p1 in the eval-mode step per slot layout
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for T in 2 0; do
  echo "== TAPORD=$T"; NIDT_C1_TAPORD=$T timeout -k 10 200 python -u tools/debug/c1_evalmode.py 2>&1 | grep -v amdgpu.ids || exit 1
done
