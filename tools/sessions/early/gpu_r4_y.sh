#!/bin/bash
# end-of-round check of the committed tree: full GPU suite, smoke, headline and 8-client benches
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4y; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread --durations=25 \
  > $OUT/pytest_gpu.txt 2>&1; rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.txt | tail -1
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2>&1 || exit 1
grep '^{' $OUT/bench_default.json | cut -c1-400
timeout -k 10 300 python bench.py --clients 8 --steps 20 --warmup 3 > $OUT/bench_c8.json 2>&1 || exit 1
echo "bench 8 clients: $(grep -o '"value": [0-9.]*' $OUT/bench_c8.json)"
