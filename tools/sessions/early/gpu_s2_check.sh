#!/bin/bash
# full state check: whole GPU suite (pytest.ini timeouts), smoke(), the driver's 1-GPU bench line, kbench at 64 / 8
# clients, and a rocprofv3 kernel-trace of two bench rounds (summary only comes back)
set -o pipefail
mkdir -p gpurun_out/s2; rm -rf gpurun_out/s2/*
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout-method thread > gpurun_out/s2/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/s2/pytest.txt; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/s2/smoke.txt
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/s2/bench.txt 2>&1 || exit 1
grep '^{' gpurun_out/s2/bench.txt | cut -c1-300
for G in 64 8; do timeout -k 10 120 python tools/kbench.py $G 10 > gpurun_out/s2/kbench$G.txt 2>&1 || exit 1; done
grep -H "conv2_fwd\|full train" gpurun_out/s2/kbench*.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_s2 -o run -- python3 bench.py --steps 1 --warmup 1 \
  > gpurun_out/s2/prof_bench.txt 2>&1 || exit 1
db=$(find /tmp/prof_s2 -name "*.db" | head -1)
ms=$(python3 -c "import json; print([json.loads(l) for l in open('gpurun_out/s2/prof_bench.txt') if l.startswith('{')][0]['ms_per_step'])")
python3 tools/prof_summary.py "$db" gpurun_out/s2/round_kernels.txt --window-ms $ms --top 30 > /dev/null || exit 1
rm -rf /tmp/prof_s2
head -12 gpurun_out/s2/round_kernels.txt
timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --size-skew 1.0 > gpurun_out/s2/bench_skew1.txt 2>&1 || exit 1
grep '^{' gpurun_out/s2/bench_skew1.txt | cut -c1-200
