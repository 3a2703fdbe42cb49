#!/bin/bash
# config 5 after the evaluation change (no 2C-row staging buffer): per-round phases, per-phase memory, host gaps of
# the steady rounds; then the runner / personalized GPU tests that exercise the evaluation
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4u; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 \
  > $OUT/config5.txt 2>&1 || { tail -30 $OUT/config5.txt; exit 1; }
grep -E '^round|^\{' $OUT/config5.txt | cut -c1-1600
db=$(find /tmp/c5prof -name "*.db" | head -1)
steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/config5.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'][1:])))")
python3 tools/prof_summary.py "$db" $OUT/config5_steady_kernels.txt --top 45 --window-ms "$steady" > /dev/null 2>&1
grep -E "GAP|TIMELINE" $OUT/config5_steady_kernels.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_runner.py \
  tests/test_gpu_cli.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
grep -E "passed|failed" $OUT/pytest.txt | tail -1
