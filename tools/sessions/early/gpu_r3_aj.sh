#!/bin/bash
# vectorized transpose packs (k_pack_wt / k_pack_trans): numerics (AlexNet + ResNet engines) + kbench + CIFAR round
set -o pipefail
mkdir -p gpurun_out/r3aj
export PYTHONUNBUFFERED=1 KBENCH_EVAL=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "alexnet or graph or conv3d" \
  --timeout 200 --timeout-method thread > gpurun_out/r3aj/pytest.txt 2>&1
rc=$?; tail -1 gpurun_out/r3aj/pytest.txt; if [ $rc -ne 0 ]; then tail -30 gpurun_out/r3aj/pytest.txt; exit $rc; fi
timeout -k 10 300 python -u tools/kbench.py 64 10 > gpurun_out/r3aj/kbench.txt 2>&1 || exit 1
grep "full train step" gpurun_out/r3aj/kbench.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profaj -o run -- python3 -u bench.py --steps 2 --warmup 1 \
  > gpurun_out/r3aj/prof.txt 2>&1 || exit 1
db=$(find /tmp/profaj -name "*.db" | head -1)
python3 tools/prof_summary.py --top 45 --window-ms 460 "$db" > gpurun_out/r3aj/round_kernels.txt 2>&1
grep -E "pack|TOTAL|TIMELINE" gpurun_out/r3aj/round_kernels.txt
timeout -k 10 200 python -u tools/bench_cifar.py --algorithm subavg --rounds 2 --warmup 1 > gpurun_out/r3aj/subavg.txt 2>&1 || exit 1
echo "subavg: $(grep -o '"s_per_round": [0-9.]*' gpurun_out/r3aj/subavg.txt)"
