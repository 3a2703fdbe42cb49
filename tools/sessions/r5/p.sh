#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5p; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resnet3d.py tests/test_gpu_resnet2d.py tests/test_gpu_kernels.py -k "packer or resnet or alexnet or conv" > $OUT/t.txt 2>&1 || { grep -E "FAIL|Error|assert|error" $OUT/t.txt | tail -40; exit 1; }
tail -1 $OUT/t.txt
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg.txt 2>&1 || { tail -20 $OUT/subavg.txt; exit 1; }
grep -E "^round" $OUT/subavg.txt; tail -1 $OUT/subavg.txt | cut -c1-200
timeout -k 10 400 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/dispfl.txt 2>&1 || { tail -20 $OUT/dispfl.txt; exit 1; }
grep -E "^round" $OUT/dispfl.txt; tail -1 $OUT/dispfl.txt | cut -c1-200
timeout -k 10 200 python -u tools/kbench.py 64 > $OUT/kb64.txt 2>&1 || exit 1
grep -E "full train step|conv1" $OUT/kb64.txt
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/c5prof -o run -- python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5.txt 2>&1 || { tail -20 $OUT/c5.txt; exit 1; }
grep -E '^round' $OUT/c5.txt
db=$(find /tmp/c5prof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c5_kernels.txt --top 40 --window-ms 23000 > /dev/null 2>&1
grep -E "stem|pack_plain|TIMELINE" $OUT/c5_kernels.txt | cut -c1-140
