#!/bin/bash
# Round verification: full GPU test suite, smoke, 64-client and 8-client benches, and rocprofv3 kernel stats of both.
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $O/bench64.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --clients 8 --steps 10 --warmup 3 > $O/bench8.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof64.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -- python3 bench.py --clients 8 --steps 3 --warmup 1 > $O/prof8.txt 2>&1 || exit $?
# summaries on the box (the rocpd databases are too large to bring back)
python tools/prof_summary.py --top 45 --window-ms 1150 $O/prof64/run_results.db > $O/prof64_round.txt 2>&1 || exit $?
python tools/prof_summary.py --top 45 --window-ms 245 $O/prof8/run_results.db > $O/prof8_round.txt 2>&1 || exit $?
rm -rf $O/prof64 $O/prof8
