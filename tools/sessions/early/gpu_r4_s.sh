#!/bin/bash
# chunked weight pack (pack.hip): ResNet engine numerics, then config 5 steady state with per-round phase times and
# peak memory, and a kernel trace of the steady rounds with the largest host gaps named
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4s; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_resnet2d.py \
  tests/test_gpu_resnet3d.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py \
  --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 \
  > $OUT/config5.txt 2>&1 || { tail -30 $OUT/config5.txt; exit 1; }
grep '^{' $OUT/config5.txt | cut -c1-900
db=$(find /tmp/c5prof -name "*.db" | head -1)
steady=$(python3 -c "
import json,sys
d=[json.loads(l) for l in open('$OUT/config5.txt') if l.startswith('{')][-1]
print(int(1000*sum(d['s_round_each'][1:])))")
python3 tools/prof_summary.py "$db" $OUT/config5_steady_kernels.txt --top 45 --window-ms "$steady" > /dev/null 2>&1
grep -E "GAP|TIMELINE|k_pack" $OUT/config5_steady_kernels.txt
timeout -k 10 400 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg.txt 2>&1 || exit 1
echo "subavg: $(grep -o '"s_round_each": [^]]*]' $OUT/subavg.txt)"
