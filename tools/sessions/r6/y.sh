#!/bin/bash
# [UNP2] stem unpool with two positions' loads in flight: stem tests, config 5 rounds + kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6y; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py -k "stem or lockstep" > $OUT/t.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/t.txt | tail -30; exit 1; }
grep -E "passed|failed" $OUT/t.txt | tail -1
C5="--clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1"
timeout -k 10 600 python3 -u tools/config5_resnet3d.py $C5 > $OUT/config5_plain.txt 2>&1 || { tail -30 $OUT/config5_plain.txt; exit 1; }
echo "== default"; grep -E '^round' $OUT/config5_plain.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py $C5 \
  > $OUT/config5.txt 2>&1 || { tail -30 $OUT/config5.txt; exit 1; }
echo "== default (under rocprofv3)"; grep -E '^round' $OUT/config5.txt
db=$(find /tmp/c5prof -name "*.db" | head -1)
steady=$(python3 -c "
import json
d=[json.loads(l) for l in open('$OUT/config5.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'][1:])))")
python3 tools/prof_summary.py "$db" $OUT/config5_steady_kernels.txt --top 60 --window-ms "$steady" > /dev/null 2>&1
grep -E "stem|TIMELINE" $OUT/config5_steady_kernels.txt | cut -c1-150
