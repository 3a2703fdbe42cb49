#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5o; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batched2d.py tests/test_gpu_cli.py tests/test_gpu_resnet3d.py > $OUT/t.txt 2>&1 || { grep -E "PASS|FAIL|Error|assert|error" $OUT/t.txt | tail -40; exit 1; }
grep -E "passed|failed" $OUT/t.txt | tail -1
timeout -k 10 300 python -u tools/bench_cifar.py --algorithm subavg --rounds 3 --warmup 1 > $OUT/subavg.txt 2>&1 || { tail -20 $OUT/subavg.txt; exit 1; }
grep -E "^round|^warmup" $OUT/subavg.txt; tail -1 $OUT/subavg.txt | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/cifarprof -o run -- python3 -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > $OUT/subavg_prof.txt 2>&1 || { tail -20 $OUT/subavg_prof.txt; exit 1; }
db=$(find /tmp/cifarprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/subavg_round_kernels.txt --top 45 --window-ms 1500 > /dev/null 2>&1
head -40 $OUT/subavg_round_kernels.txt | cut -c1-140; grep TIMELINE $OUT/subavg_round_kernels.txt
timeout -k 10 400 python -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/dispfl.txt 2>&1 || { tail -20 $OUT/dispfl.txt; exit 1; }
grep -E "^round|^warmup" $OUT/dispfl.txt; tail -1 $OUT/dispfl.txt | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/dprof -o run -- python3 -u tools/bench_cifar.py --algorithm dispfl --rounds 1 --warmup 1 > $OUT/dispfl_prof.txt 2>&1 || { tail -20 $OUT/dispfl_prof.txt; exit 1; }
db=$(find /tmp/dprof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/dispfl_round_kernels.txt --top 45 --window-ms 4500 > /dev/null 2>&1
head -30 $OUT/dispfl_round_kernels.txt | cut -c1-140; grep -E "TIMELINE|GAP" $OUT/dispfl_round_kernels.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench64.txt 2>&1 || { tail -20 $OUT/bench64.txt; exit 1; }
tail -1 $OUT/bench64.txt | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/b64prof -o run -- python3 -u bench.py --steps 3 --warmup 2 > $OUT/b64prof.txt 2>&1 || { tail -20 $OUT/b64prof.txt; exit 1; }
db=$(find /tmp/b64prof -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" $OUT/c64_round_kernels.txt --top 45 --window-ms 1200 > /dev/null 2>&1
head -46 $OUT/c64_round_kernels.txt | cut -c1-140; grep -E "TIMELINE" $OUT/c64_round_kernels.txt
timeout -k 10 400 python3 -u tools/config5_resnet3d.py --clients 256 --train-per-client 36 --test-per-client 9 --batch 4 --group 32 --rounds 3 --warmup 1 > $OUT/c5.txt 2>&1 || { tail -20 $OUT/c5.txt; exit 1; }
grep -E '^round' $OUT/c5.txt
