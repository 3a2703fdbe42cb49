#!/bin/bash
# [DPP-SUM] statistics epilogue with DPP row sums: epilogue cost, kernel numerics tests, headline bench / 8 clients
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6s3x; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/debug/slab_stats_cost.py > $OUT/cost.txt 2>&1 || { tail -20 $OUT/cost.txt; exit 1; }
grep -v amdgpu.ids $OUT/cost.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_resnet3d.py tests/test_gpu_resnet2d.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 1; }
echo "== bench $(tail -1 $OUT/bench.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
timeout -k 10 300 python -u bench.py --clients 8 --steps 20 --warmup 5 > $OUT/bench8.txt 2>&1 || { tail -20 $OUT/bench8.txt; exit 1; }
echo "== bench c8 $(tail -1 $OUT/bench8.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
